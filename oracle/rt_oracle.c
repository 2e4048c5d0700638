/*
 * rt_oracle.c — CPU oracle: plain-C restatement of the reference hot path.
 *
 *   TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 *   bench.py's cpu_baseline leg may load this library, and only as the checker
 *   (or, for cpu_baseline, as the timed CPU restatement).  The product
 *   (raytracing_rb_amd / librtx) never links or calls it.
 *
 * Semantics follow the Ruby reference line by line (file:line cited per
 * function) and the Vec3 C extension ext/fast_4d_matrix/fast_4d_matrix.c.
 * Built with gcc -O2 -ffp-contract=off: binary64, no FMA, glibc libm — the
 * arithmetic the Ruby interpreter and the extension (extconf.rb:6-10) perform.
 * Bit-for-bit checked against the Python restatement oracle/rt_ref.py.
 *
 * Parity status: the Vec3 layer is pinned by spec/fast_4d_matrix_spec.rb; the
 * rendering layers are "parity unpinned" against a live reference (no Ruby in
 * this image) and pinned by the two restatements + goldens.
 *
 * Departures (documented in DESIGN.md): counter RNG instead of Random.rand;
 * no LOG tracing.  World#high_lights' lit_area (world.rb:92-93) is evaluated
 * for its raises (its value is always truthy) but not counted in the work
 * counters, which count the brute-force events of local_lights' walks.
 */
#define _GNU_SOURCE
#include "../include/rtx.h"

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#define EPS 1e-5 /* src/libs/algebra.rb:2 */

static int rto_debug = -1;   /* RTO_DEBUG=1: trace leaves/areas to stderr (debugging only) */

/* ------------------------------------------------------------ Vec3 (L0) */
typedef struct { double x, y, z; } V;

typedef struct {
  int err;            /* first rtx_status raised in this trace */
  char msg[160];
  uint64_t cnt[RTX_NCOUNT];
} T;

static void raise_(T* t, int code, const char* what) {
  if (!t->err) {
    t->err = code;
    snprintf(t->msg, sizeof t->msg, "%s", what);
  }
}

static inline V vmk(double x, double y, double z) { V v = {x, y, z}; return v; }
static inline double vr(V a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }   /* :62-73 */
static inline double vr2(V a) { double r = vr(a); return r * r; }                   /* :280-284 */
static inline double vdot(V a, V b) {                                                /* :98-107 */
  double s = 0;
  s += a.x * b.x;
  s += a.y * b.y;
  s += a.z * b.z;
  return s;
}
static inline V vadd(V a, V b) { return vmk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V vsub(V a, V b) { return vmk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V vmul(V a, V b) { return vmk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V vsc(V a, double s) { return vmk(a.x * s, a.y * s, a.z * s); }
static inline V vdiv(V a, double s) { return vmk(a.x / s, a.y / s, a.z / s); }
static inline V vneg(V a) { return vmk(-a.x, -a.y, -a.z); }
static inline V vcross(V a, V b) {                                                   /* :131-141 */
  return vmk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline V vnorm(V a, T* t) {                                                   /* :286-293 */
  double r = sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  if (r == 0) { raise_(t, RTX_EZERO_VEC, "zero vector detected"); return a; }
  return vmk(a.x / r, a.y / r, a.z / r);
}
static inline double vcos(V a, V b, T* t) {                                          /* :109-129 */
  double ret = 0, r1, r2;
  ret += a.x * b.x;
  ret += a.y * b.y;
  ret += a.z * b.z;
  r1 = a.x * a.x + a.y * a.y + a.z * a.z;
  r2 = b.x * b.x + b.y * b.y + b.z * b.z;
  if (r1 == 0 || r2 == 0) { raise_(t, RTX_EZERO_VEC, "zero vector detected!"); return 0; }
  double v = sqrt(ret * ret / r1 / r2);
  if (v > 1) v = 1;
  return v;
}
static inline V vd(const double* a) { return vmk(a[0], a[1], a[2]); }

static double dacos(double x, T* t) {
  if (x < -1 || x > 1) raise_(t, RTX_EDOMAIN, "Math::DomainError acos");
  return acos(x);
}
static double dasin(double x, T* t) {
  if (x < -1 || x > 1) raise_(t, RTX_EDOMAIN, "Math::DomainError asin");
  return asin(x);
}
static double dsqrt(double x, T* t) {
  if (x < 0) raise_(t, RTX_EDOMAIN, "Math::DomainError sqrt");
  return sqrt(x);
}

/* ------------------------------------------------------------ RNG contract */
static inline uint64_t fmix64(uint64_t h) {
  h ^= h >> 33; h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33; h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  return h;
}
double rto_rand(uint64_t seed, int32_t x, int32_t y, int32_t sample, uint64_t path, int32_t draw) {
  uint64_t h = seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  h = fmix64(h ^ (((uint64_t)(uint32_t)x << 32) | (uint32_t)y));
  h = fmix64(h ^ (((uint64_t)(uint32_t)sample << 32) | (uint32_t)draw));
  h = fmix64(h ^ path);
  return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

/* ------------------------------------------------------------ scene (L2) */
typedef struct { V o, d; } Ray; /* Alex::Ray: position, front (algebra.rb:3-17) */

typedef struct {             /* Plane (plane.rb) or one face of a Box (box.rb:20-66) */
  V P, F, U;
  V left_n, up_n;            /* self.left.normalize, self.up.normalize (plane.rb:82-83) */
  double uu, vu;
  int has_rr;
  double rr;
} Pl;

typedef struct { int w, h; double* texel; /* w*h*3, (c>>8)/256.0 */ } Tex;

typedef struct {
  int type, tex;
  int has_rr, has_ra;
  V diffuse, ambient, refl_att, refr_att;
  double rr;
  /* sphere */
  V C; double R;
  V gw_n, east_n, north_n;
  double u_off, v_off;
  /* plane / box */
  Pl pl;
  Pl face[6];
  double hs, vs;
} Obj;

typedef struct {
  V pos, color;
  double radius, hl_rate, hl_angle;
} Light;

typedef struct {
  /* world */
  double max_distance, sse;
  int nobj, nlight, ntex;
  Obj* obj;
  Light* light;
  Tex* tex;
  /* camera */
  rtx_camera_desc cam;
  V cpos, cup, cfront;
  char errmsg[256];
} Scene;

static void plane_reinit(Pl* p, T* t) {                  /* plane.rb:21-23 */
  V left = vnorm(vcross(p->F, p->U), t);
  p->left_n = vnorm(left, t);
  p->up_n = vnorm(p->U, t);
}

void rto_destroy(Scene* s) {
  if (!s) return;
  for (int i = 0; i < s->ntex; i++) free(s->tex[i].texel);
  free(s->tex);
  free(s->obj);
  free(s->light);
  free(s);
}

static void dbg_init(void) { if (rto_debug < 0) rto_debug = getenv("RTO_DEBUG") != NULL; }
Scene* rto_create(const rtx_scene_desc* sd, const rtx_camera_desc* cd, char* err, size_t errlen) {
  dbg_init();
  Scene* s = (Scene*)calloc(1, sizeof(Scene));
  T t; memset(&t, 0, sizeof t);
  s->max_distance = sd->max_distance;
  s->sse = sd->soft_shadow_exponent;
  s->nobj = sd->n_objects;
  s->nlight = sd->n_lights;
  s->ntex = sd->n_textures;
  s->obj = (Obj*)calloc(s->nobj ? s->nobj : 1, sizeof(Obj));
  s->light = (Light*)calloc(s->nlight ? s->nlight : 1, sizeof(Light));
  s->tex = (Tex*)calloc(s->ntex ? s->ntex : 1, sizeof(Tex));
  for (int i = 0; i < s->ntex; i++) {
    const rtx_texture_desc* td = &sd->textures[i];
    Tex* x = &s->tex[i];
    x->w = td->width; x->h = td->height;
    x->texel = (double*)malloc(sizeof(double) * 3 * (size_t)x->w * x->h);
    for (size_t k = 0; k < (size_t)3 * x->w * x->h; k++) x->texel[k] = td->rgb[k] / 256.0;
  }
  for (int i = 0; i < s->nlight; i++) {
    const rtx_light_desc* l = &sd->lights[i];
    s->light[i].pos = vd(l->position);
    s->light[i].color = vd(l->color);
    s->light[i].radius = l->radius;
    s->light[i].hl_rate = l->high_light_rate;
    s->light[i].hl_angle = l->high_light_angle;
  }
  for (int i = 0; i < s->nobj; i++) {
    const rtx_object_desc* d = &sd->objects[i];
    Obj* o = &s->obj[i];
    o->type = d->type;
    o->tex = d->texture_id;
    o->has_rr = d->has_refractive_rate;
    o->has_ra = d->has_refractive_attenuation;
    o->diffuse = vd(d->diffuse_rate);
    o->ambient = vd(d->ambient);
    o->refl_att = vd(d->reflective_attenuation);
    o->refr_att = vd(d->refractive_attenuation);
    o->rr = d->refractive_rate;
    o->hs = d->texture_horizontal_scale;
    o->vs = d->texture_vertical_scale;
    if (d->type == RTX_SPHERE) {
      o->C = vd(d->center);
      o->R = d->radius;
      o->u_off = d->texture_u_offset;
      o->v_off = d->texture_v_offset;
      if (o->tex >= 0) {                               /* sphere.rb:16-22, 111-115 */
        V north = vd(d->north_pole_vec), gw = vd(d->greenwich_vec);
        V east = vcross(north, gw);
        o->gw_n = vnorm(gw, &t);
        o->east_n = vnorm(east, &t);
        o->north_n = vnorm(north, &t);
      }
    } else if (d->type == RTX_PLANE) {
      o->pl.P = vd(d->point); o->pl.F = vd(d->front); o->pl.U = vd(d->up);
      o->pl.uu = d->u_unit; o->pl.vu = d->v_unit;
      o->pl.has_rr = d->has_refractive_rate; o->pl.rr = d->refractive_rate;
      plane_reinit(&o->pl, &t);
    } else if (d->type == RTX_BOX) {                     /* box.rb:15-73 */
      V P = vd(d->point), F = vd(d->front), U = vd(d->up);
      double wf = d->width_front, wu = d->width_up, wl = d->width_left;
      V left = vnorm(vcross(F, U), &t);
      Pl* f = o->face;
      f[0].F = U;        f[0].U = left; f[0].P = vadd(P, vsc(vsc(U, wu), 0.5));    f[0].uu = wf; f[0].vu = wl;
      f[1].F = vneg(U);  f[1].U = left; f[1].P = vsub(P, vsc(vsc(U, wu), 0.5));    f[1].uu = wf; f[1].vu = wl;
      f[2].F = F;        f[2].U = U;    f[2].P = vadd(P, vsc(vsc(F, wf), 0.5));    f[2].uu = wl; f[2].vu = wu;
      f[3].F = vneg(F);  f[3].U = U;    f[3].P = vsub(P, vsc(vsc(F, wf), 0.5));    f[3].uu = wl; f[3].vu = wu;
      f[4].F = left;     f[4].U = U;    f[4].P = vadd(P, vsc(vsc(left, wl), 0.5)); f[4].uu = wf; f[4].vu = wu;
      f[5].F = vneg(left); f[5].U = U;  f[5].P = vsub(P, vsc(vsc(left, wl), 0.5)); f[5].uu = wf; f[5].vu = wu;
      for (int k = 0; k < 6; k++) {
        f[k].has_rr = d->has_refractive_rate; f[k].rr = d->refractive_rate;
        plane_reinit(&f[k], &t);
      }
    } else {
      snprintf(err, errlen, "object %d: unknown type %d", i, d->type);
      rto_destroy(s);
      return NULL;
    }
  }
  s->cam = *cd;
  s->cpos = vd(cd->position); s->cup = vd(cd->up); s->cfront = vd(cd->front);
  if (t.err) {
    snprintf(err, errlen, "scene setup: %s", t.msg);
    rto_destroy(s);
    return NULL;
  }
  return s;
}

/* ------------------------------------------------------------ intersections */
typedef struct { V hit; int in; V delta; int face; } Hit;

static int sphere_hit(const Obj* s, Ray ray, Hit* h, T* t) {   /* sphere.rb:60-85 */
  double tt = vdot(vsub(s->C, ray.o), ray.d) / vr2(ray.d);
  V v = vsc(ray.d, tt);
  V np = vadd(ray.o, v);
  if (!(vr(vsub(np, s->C)) <= s->R)) return 0;                   /* inner? :103-105 */
  double nd = vr(vsub(np, s->C));
  double hh = dsqrt(pow(s->R, 2.0) - pow(nd, 2.0), t);
  V vec = vsc(vnorm(ray.d, t), hh);
  int from_inner = vr(vsub(ray.o, s->C)) <= s->R;
  int in = !from_inner;
  V hit = in ? vsub(np, vec) : vadd(np, vec);
  if (!from_inner && tt < 0) return 0;
  h->hit = hit;
  h->in = in;
  h->delta = vsc(vsc(vsub(hit, s->C), EPS), in ? 1.0 : -1.0);
  h->face = -1;
  return 1;
}

static int plane_hit(const Pl* p, Ray ray, Hit* h) {            /* plane.rb:38-51 */
  double den = vdot(p->F, ray.d);
  if (den == 0) return 0;
  double tt = vdot(vsub(p->P, ray.o), p->F) / den;
  V hit = vadd(ray.o, vsc(ray.d, tt));
  if (tt < 0) return 0;
  double fd = vdot(p->F, ray.d);
  h->in = fd < 0;
  double nd = -fd;
  double sg = nd > 0 ? 1.0 : (nd < 0 ? -1.0 : 0.0);             /* (x <=> 0).to_f */
  h->delta = vsc(vsc(p->F, EPS), sg);
  h->hit = hit;
  h->face = -1;
  return 1;
}

static void plane_uv(const Pl* p, V pos, double* u, double* v) { /* plane.rb:81-85 */
  *u = vdot(vsub(pos, p->P), p->left_n) / p->uu;
  *v = vdot(vsub(pos, p->P), p->up_n) / p->vu;
}

static int box_hit(const Obj* b, Ray ray, Hit* h) {             /* box.rb:79-97 */
  double nearest = INFINITY;
  int found = 0;
  for (int i = 0; i < 6; i++) {
    Hit fh;
    if (plane_hit(&b->face[i], ray, &fh)) {
      double u, v;
      plane_uv(&b->face[i], fh.hit, &u, &v);
      if (-0.5 <= u && u <= 0.5 && -0.5 <= v && v <= 0.5) {
        double d = vr(vsub(fh.hit, ray.o));
        if (d < nearest) {
          nearest = d;
          *h = fh;
          h->face = i;
          found = 1;
        }
      }
    }
  }
  return found;
}

static int obj_hit(const Obj* o, Ray ray, Hit* h, T* t) {
  if (o->type == RTX_SPHERE) return sphere_hit(o, ray, h, t);
  if (o->type == RTX_PLANE) return plane_hit(&o->pl, ray, h);
  return box_hit(o, ray, h);
}

static int world_hit(const Scene* s, Ray ray, Hit* best, T* t) {  /* world.rb:37-59 */
  double nearest = s->max_distance;
  int obj = -1;
  for (int i = 0; i < s->nobj; i++) {
    const Obj* o = &s->obj[i];
    Hit h;
    if (o->type == RTX_SPHERE) t->cnt[RTX_CNT_SPHERE_TESTS]++;
    else if (o->type == RTX_PLANE) t->cnt[RTX_CNT_PLANE_TESTS]++;
    else t->cnt[RTX_CNT_BOX_TESTS]++;
    if (obj_hit(o, ray, &h, t)) {
      if (o->type == RTX_SPHERE) t->cnt[RTX_CNT_SPHERE_HITS]++;
      double nd = vr(vsub(ray.o, h.hit));                          /* Ray#distance */
      if (nd < nearest) {
        nearest = nd;
        obj = i;
        *best = h;
      }
    }
  }
  return obj;
}

/* ------------------------------------------------------------ shadows */
static double cover_area(const Scene* s, const Obj* o, V L, double radius, V T_, T* t) {
  Ray sr = {T_, vsub(L, T_)};                                      /* world_object.rb:41-49 */
  Hit h;
  int factor = 0;
  if (o->type == RTX_SPHERE) t->cnt[RTX_CNT_COVER_SPHERE]++;
  else if (o->type == RTX_PLANE) t->cnt[RTX_CNT_COVER_PLANE]++;
  else t->cnt[RTX_CNT_COVER_BOX]++;
  if (obj_hit(o, sr, &h, t) && vdot(vsub(h.hit, L), vsub(T_, L)) > 0) factor = 1;
  if (o->type != RTX_SPHERE) return (double)factor;
  /* Sphere#cover_area sphere.rb:28-57 */
  V lt = vsub(L, T_);
  double tt = vdot(vsub(o->C, T_), lt) / vr2(lt);
  V x1 = vadd(T_, vsc(lt, tt));
  double r1 = radius * (vr(vsub(x1, T_)) / vr(lt));
  double d = vr(vsub(x1, o->C));
  double R = o->R;
  if (d >= r1 + R) return 0.0;
  double s1 = M_PI * r1 * r1;
  if (d > fabs(R - r1)) {
    double c1 = (r1 * r1 + d * d - R * R) / (2 * r1 * d);
    double c2 = (R * R + d * d - r1 * r1) / (2 * R * d);
    if (c1 > 1.0) c1 = 1.0;
    if (c2 > 1.0) c2 = 1.0;
    double th1 = dacos(c1, t), th2 = dacos(c2, t);
    double ds = ((th1 - sin(th1)) * r1 * r1 + (th2 - sin(th2)) * R * R) / 2;
    return factor * ds / s1;
  }
  if (r1 > R) return factor * M_PI * R * R / s1;
  return (double)factor;
}

static double lit_area(const Scene* s, V target, V L, double radius, T* t) {   /* world.rb:62-69 */
  double total = 1;
  for (int i = 0; i < s->nobj; i++) total -= cover_area(s, &s->obj[i], L, radius, target, t);
  return total > 0 ? total : 0;
}

/* ------------------------------------------------------------ shading */
static V texcolor(const Tex* x, double hs, double vs, double uo, double vo, double uu, double vv, T* t) {
  /* texture.rb:23-28: trunc then Ruby floor-mod */
  double qu = (uu + uo) / hs, qv = (vv + vo) / vs;
  if (!isfinite(qu) || !isfinite(qv)) { raise_(t, RTX_EDOMAIN, "FloatDomainError"); return vmk(0, 0, 0); }
  double tu = fmod(trunc(qu), (double)x->w), tv = fmod(trunc(qv), (double)x->h);
  long iu = (long)tu, iv = (long)tv;
  if (iu < 0) iu += x->w;
  if (iv < 0) iv += x->h;
  const double* p = &x->texel[((size_t)iv * x->w + iu) * 3];
  if (rto_debug > 0) fprintf(stderr, "tex uv %.17g %.17g -> %ld %ld\n", uu, vv, iu, iv);
  return vmk(p[0], p[1], p[2]);
}

typedef struct { int light; V color; } Lit;

static V local_lighting(const Obj* o, V pos, const Lit* lit, int nl, const Scene* s, V nrm,
                        int has_filter, V filter, T* t) {         /* world_object.rb:51-74 */
  V lc = vmk(0.0, 0.0, 0.0);
  for (int k = 0; k < nl; k++) {
    V n = vnorm(nrm, t);
    V l = vnorm(vsub(s->light[lit[k].light].pos, pos), t);
    double ldn = vdot(l, n);
    if (ldn > 1) ldn = 1.0;
    else if (ldn < 0) ldn = 0.0;
    lc = vadd(lc, vsc(lit[k].color, ldn));
    if (rto_debug > 0) fprintf(stderr, "ldn %.17g lcol %.17g n %.17g %.17g %.17g\n", ldn, lit[k].color.x, n.x, n.y, n.z);
  }
  if (nl > 0) lc = vdiv(lc, (double)nl);
  if (has_filter) return vadd(vmul(vmul(lc, o->diffuse), filter), o->ambient);
  return vadd(vmul(lc, o->diffuse), o->ambient);
}

static V vertical(V n, T* t) {                                     /* world_object.rb:105-120 */
  if (vr(n) == 0) { raise_(t, RTX_EZERO_VEC, "zero vector detected"); return vmk(1, 0, 0); }
  if (n.x == 0) {
    if (n.y == 0) return vmk(1.0, 0.0, 0.0);
    return vmk(0.0, -n.z / n.y, 1.0);
  }
  return vmk(-(n.y + n.z) / n.x, 1.0, 1.0);
}

static Ray reflection(Ray ray, V n, V hit, V delta, T* t) {         /* world_object.rb:121-125 */
  double c = vcos(ray.d, vneg(n), t);
  V f = vnorm(vadd(vsc(vnorm(n, t), 2 * c * vr(ray.d)), ray.d), t);
  Ray r = {vadd(hit, delta), f};
  return r;
}

static int refraction(Ray ray, V n, V hit, V refl, double rate, Ray* out, T* t) { /* :127-137 */
  double sin_i = dsqrt(1 - pow(vcos(ray.d, n, t), 2.0), t);
  double sin_r = sin_i / rate;
  if (sin_r >= 1) return 0;
  double r = dasin(sin_r, t);
  V dir = vadd(vsc(vnorm(n, t), -cos(r)), vsc(vnorm(vadd(refl, ray.d), t), sin_r));
  out->d = dir;
  out->o = vsub(hit, vsc(vnorm(n, t), EPS));
  return 1;
}

/* ------------------------------------------------------------ tracer (L3) */
typedef struct { Ray ray; int depth; V att; uint64_t path; } Item;

typedef struct { Item* a; int n, cap; } Stack;
static void push(Stack* st, Item it) {
  if (st->n == st->cap) {
    st->cap = st->cap ? st->cap * 2 : 64;
    st->a = (Item*)realloc(st->a, sizeof(Item) * st->cap);
  }
  st->a[st->n++] = it;
}

typedef struct { const Scene* s; uint64_t seed; int x, y, sample; Stack st; Lit* lit; int gt1; } Tr;

/* ray_tracer.rb:292-298.  The running sum is the FIFO drain's (leaves in
 * emission order), but the drain runs after the whole tree (:39-45): a
 * "color greater than 1" is raised only once every rt_map of the tree has run,
 * so an rt_map raise anywhere in the tree comes first (trace_sync below). */
static void add_leaf(Tr* tr, V* sum, V c) {
  if (rto_debug > 0) fprintf(stderr, "leaf %.17g %.17g %.17g\n", c.x, c.y, c.z);
  *sum = vadd(*sum, c);
  if (!(sum->x <= 1 && sum->y <= 1 && sum->z <= 1)) tr->gt1 = 1;
}

static void rt_map(Tr* tr, Item it, V* sum, T* t) {                /* ray_tracer.rb:50-164 */
  const Scene* s = tr->s;
  if (it.depth <= 0 || vr(it.att) < 0.0001) return;
  t->cnt[RTX_CNT_RAYS]++;
  /* World#high_lights world.rb:83-98 */
  int nfired = 0;
  for (int l = 0; l < s->nlight; l++) {
    t->cnt[RTX_CNT_HIGHLIGHT_TESTS]++;
    double c = vcos(it.ray.d, vsub(s->light[l].pos, it.ray.o), t);
    if (c < -1) c = -1;
    if (c > 1) c = 1;
    if (dacos(c, t) < (s->light[l].hl_angle / 180.0 * M_PI)) {
      /* `&& lit_area(ray.position, light.position, light.radius, object)`
       * (world.rb:92-93): a number, always truthy, but its Sphere#cover_area
       * can raise (Math.acos, sphere.rb:45-46) */
      uint64_t keep[RTX_NCOUNT];
      memcpy(keep, t->cnt, sizeof keep);
      (void)lit_area(s, it.ray.o, s->light[l].pos, s->light[l].radius, t);
      memcpy(t->cnt, keep, sizeof keep);
      tr->lit[nfired++].light = l;
    }
  }
  if (nfired) {
    for (int k = 0; k < nfired; k++) {
      const Light* L = &s->light[tr->lit[k].light];
      add_leaf(tr, sum, vdiv(vmul(it.att, vsc(L->color, L->hl_rate)), (double)nfired));
    }
    return;
  }
  Hit h;
  int oi = world_hit(s, it.ray, &h, t);
  if (oi < 0) return;
  t->cnt[RTX_CNT_SHADE_HITS]++;
  const Obj* o = &s->obj[oi];
  /* intersect_parameters: sphere.rb:88-101, plane.rb:54-67, box.rb:100-105 */
  V n;
  Ray refl, refr;
  int has_refr;
  const int pt = s->cam.monte_carlo_diffusion_times;
  if (o->type == RTX_SPHERE) {
    n = h.in ? vsub(h.hit, o->C) : vsub(o->C, h.hit);
    refl = reflection(it.ray, n, h.hit, h.delta, t);
    double rate = h.in ? o->rr : 1.0 / o->rr;
    has_refr = refraction(it.ray, n, h.hit, refl.d, rate, &refr, t);
  } else {
    const Pl* p = (o->type == RTX_PLANE) ? &o->pl : &o->face[h.face];
    n = vdot(p->F, it.ray.d) > 0 ? vneg(p->F) : p->F;
    refl = reflection(it.ray, n, h.hit, h.delta, t);
    has_refr = p->has_rr ? refraction(it.ray, n, h.hit, refl.d, p->rr, &refr, t) : 0;
  }
  uint64_t R = (uint64_t)pt + 3;
  Item c1 = {refl, it.depth - 1, vmul(it.att, o->refl_att), it.path * R + 1};
  push(&tr->st, c1);
  if (has_refr) {
    Item c2 = {refr, it.depth - 1, vmul(it.att, o->refr_att), it.path * R + 2};
    push(&tr->st, c2);
  }
  /* World#local_lights world.rb:72-80 at intersection + delta */
  V target = vadd(h.hit, h.delta);
  int nl = 0;
  for (int l = 0; l < s->nlight; l++) {
    double area = lit_area(s, target, s->light[l].pos, s->light[l].radius, t);
    if (rto_debug > 0) fprintf(stderr, "area obj=%d %.17g target %.17g %.17g %.17g\n", oi, area, target.x, target.y, target.z);
    if (area > 0) {
      tr->lit[nl].light = l;
      tr->lit[nl].color = vsc(s->light[l].color, pow(area, s->sse) / s->nlight);
      nl++;
    }
  }
  if (nl == 0) {                                                  /* path_tracing world_object.rb:76-90 */
    V att = vdiv(o->diffuse, (double)pt);
    for (int k = 0; k < pt; k++) {
      V front = vnorm(n, t);
      V left = vnorm(vertical(n, t), t);
      V up = vcross(front, left);
      double theta = rto_rand(tr->seed, tr->x, tr->y, tr->sample, it.path, 2 * k) * M_PI / 2;
      double phi = rto_rand(tr->seed, tr->x, tr->y, tr->sample, it.path, 2 * k + 1) * M_PI * 2;
      V dir = vadd(vsc(front, sin(theta)), vsc(vadd(vsc(left, cos(phi)), vsc(up, sin(phi))), cos(theta)));
      Item ci = {{target, dir}, it.depth - 1, vmul(it.att, att), it.path * R + 3 + (uint64_t)k};
      push(&tr->st, ci);
    }
  } else {
    int has_filter = 0;
    V filter = vmk(1.0, 1.0, 1.0);
    if (o->type == RTX_SPHERE) {                                  /* sphere.rb:122-129 */
      has_filter = 1;
      if (o->tex >= 0) {
        V vec = vsub(h.hit, o->C);                                /* get_uv :111-120 */
        double x = vdot(vec, o->gw_n) / o->R;
        double y = vdot(vec, o->east_n) / o->R;
        double z = vdot(vec, o->north_n) / o->R;
        double m = dsqrt(x * x + y * y + z * z + 2 * x + 1, t);
        double u = (y / m + 1) / 2, v = (-z / m + 1) / 2;
        filter = vmul(texcolor(&s->tex[o->tex], o->hs, o->vs, o->u_off, o->v_off, u, v, t), filter);
      }
    } else if (o->type == RTX_PLANE) {                            /* plane.rb:87-94 */
      has_filter = 1;
      if (o->tex >= 0) {
        double u, v;
        plane_uv(&o->pl, h.hit, &u, &v);
        filter = vmul(texcolor(&s->tex[o->tex], o->hs, o->vs, 0.0, 0.0, u, v, t), filter);
      }
    }
    add_leaf(tr, sum, vmul(it.att, local_lighting(o, h.hit, tr->lit, nl, s, n, has_filter, filter, t)));
  }
}

static V trace_sync(Tr* tr, Ray ray, T* t) {                      /* ray_tracer.rb:16-46 */
  V sum = vmk(0.0, 0.0, 0.0);
  tr->st.n = 0;
  Item root = {ray, tr->s->cam.trace_depth, vmk(1.0, 1.0, 1.0), 1};
  push(&tr->st, root);
  tr->gt1 = 0;
  while (tr->st.n > 0) {
    Item it = tr->st.a[--tr->st.n];
    rt_map(tr, it, &sum, t);
  }
  if (tr->gt1) raise_(t, RTX_ECOLOR_GT1, "color greater than 1");   /* the drain, after the tree */
  return sum;
}

/* ------------------------------------------------------------ camera (L4) */
static Ray lens(const Scene* s, int x, int y, int j, uint64_t seed, T* t) {   /* camera.rb:129-151 */
  const rtx_camera_desc* c = &s->cam;
  V left = vnorm(vcross(s->cup, s->cfront), t);
  V rc = vsub(s->cpos, vsc(vnorm(s->cfront, t), c->image_distance));
  V rp = vadd(vadd(rc, vsc(left, 2.0 * ((double)x / c->width - 0.5) * c->retina_width)),
              vsc(vnorm(s->cup, t), 2 * ((double)y / c->height - 0.5) * c->retina_height));
  double theta = rto_rand(seed, x, y, j, 0, 0);
  V rv = vsc(vadd(vsc(vnorm(left, t), cos(theta)), vsc(vnorm(s->cup, t), sin(theta))), c->aperture_radius);
  V ap = vadd(s->cpos, rv);
  double od = c->focal_distance * c->image_distance / (c->image_distance - c->focal_distance);
  V pofp = vadd(s->cpos, vsc(vnorm(s->cfront, t), od));
  Ray r = {rp, vsub(s->cpos, rp)};
  double tt = vdot(vsub(pofp, r.o), s->cfront) / vdot(s->cfront, r.d);   /* intersect_plane :123-127 */
  V target = vadd(r.o, vsc(r.d, tt));
  Ray out = {ap, vsub(target, ap)};
  return out;
}

static V render_at(Tr* tr, int x, int y, T* t) {                    /* camera.rb:70-99 */
  const Scene* s = tr->s;
  const int pre = s->cam.pre_sample_times, mx = s->cam.max_sample_times;
  V avg = vmk(0.0, 0.0, 0.0);
  V* smp = (V*)alloca(sizeof(V) * (pre > 0 ? pre : 1));
  tr->x = x; tr->y = y;
  for (int j = 0; j < pre; j++) {
    tr->sample = j;
    t->cnt[RTX_CNT_PRIMARY]++;
    V v = trace_sync(tr, lens(s, x, y, j, tr->seed, t), t);
    smp[j] = v;
    avg = vadd(avg, v);
  }
  double variance = 0;
  avg = vdiv(avg, (double)pre);
  for (int j = 0; j < pre; j++) {
    V dd = vsub(smp[j], avg);
    double m = dd.x;
    if (dd.y > m) m = dd.y;
    if (dd.z > m) m = dd.z;
    variance += pow(m, 2.0);
  }
  variance /= pre;
  if (variance >= s->cam.variant_threshold) {
    V cv = vmk(0.0, 0.0, 0.0);
    for (int j = pre; j < mx; j++) {
      tr->sample = j;
      t->cnt[RTX_CNT_PRIMARY]++;
      cv = vadd(cv, trace_sync(tr, lens(s, x, y, j, tr->seed, t), t));
    }
    avg = vdiv(vadd(vsc(avg, (double)pre), cv), (double)mx);
  }
  return avg;
}

static void tr_init(Tr* tr, const Scene* s, uint64_t seed) {
  memset(tr, 0, sizeof *tr);
  tr->s = s;
  tr->seed = seed;
  tr->lit = (Lit*)calloc(s->nlight ? s->nlight : 1, sizeof(Lit));
}
static void tr_free(Tr* tr) { free(tr->st.a); free(tr->lit); }

/* ------------------------------------------------------------ exported API */
const char* rto_last_error(const Scene* s) { return s ? s->errmsg : ""; }

/* Render rows [y0,y1) x cols [x0,x1) (x outer, y inner like render_sync).
 * status[(y-y0)*(x1-x0)+(x-x0)] receives the per-pixel rtx_status (may be NULL).
 * Returns the first error status (0 if none). */
int rto_render(Scene* s, int x0, int y0, int x1, int y1, uint64_t seed, double* out,
               size_t stride, int32_t* status, uint64_t* counts) {
  Tr tr;
  tr_init(&tr, s, seed);
  int first = 0;
  for (int x = x0; x < x1; x++)
    for (int y = y0; y < y1; y++) {
      T t; memset(&t, 0, sizeof t);
      V c = render_at(&tr, x, y, &t);
      double* p = out + (size_t)(y - y0) * stride + (size_t)(x - x0) * 3;
      p[0] = c.x; p[1] = c.y; p[2] = c.z;
      if (status) status[(size_t)(y - y0) * (x1 - x0) + (x - x0)] = t.err;
      if (t.err && !first) {
        first = t.err;
        snprintf(s->errmsg, sizeof s->errmsg, "pixel (%d,%d): %s", x, y, t.msg);
      }
      if (counts) for (int k = 0; k < RTX_NCOUNT; k++) counts[k] += t.cnt[k];
    }
  tr_free(&tr);
  return first;
}

/* Render an arbitrary pixel list xy[2i], xy[2i+1] -> out[3i..3i+2]. */
int rto_render_pixels(Scene* s, int n, const int32_t* xy, uint64_t seed, double* out, int32_t* status,
                      uint64_t* counts) {
  Tr tr;
  tr_init(&tr, s, seed);
  int first = 0;
  for (int i = 0; i < n; i++) {
    T t; memset(&t, 0, sizeof t);
    V c = render_at(&tr, xy[2 * i], xy[2 * i + 1], &t);
    out[3 * i] = c.x; out[3 * i + 1] = c.y; out[3 * i + 2] = c.z;
    if (status) status[i] = t.err;
    if (t.err && !first) {
      first = t.err;
      snprintf(s->errmsg, sizeof s->errmsg, "pixel (%d,%d): %s", xy[2 * i], xy[2 * i + 1], t.msg);
    }
    if (counts) for (int k = 0; k < RTX_NCOUNT; k++) counts[k] += t.cnt[k];
  }
  tr_free(&tr);
  return first;
}

/* RayTracer#trace_sync for explicit rays (front, position) keyed by (x,y,sample). */
int rto_trace(Scene* s, int n, const double* rays, const int32_t* keys, uint64_t seed, double* out,
              int32_t* status) {
  Tr tr;
  tr_init(&tr, s, seed);
  int first = 0;
  for (int i = 0; i < n; i++) {
    T t; memset(&t, 0, sizeof t);
    tr.x = keys[3 * i]; tr.y = keys[3 * i + 1]; tr.sample = keys[3 * i + 2];
    Ray r = {vd(rays + 6 * i + 3), vd(rays + 6 * i)};
    V c = trace_sync(&tr, r, &t);
    out[3 * i] = c.x; out[3 * i + 1] = c.y; out[3 * i + 2] = c.z;
    if (status) status[i] = t.err;
    if (t.err && !first) first = t.err;
  }
  tr_free(&tr);
  return first;
}

/* Primary ray of Camera#lens_func (camera.rb:129-151) for cross-checks. */
void rto_lens(Scene* s, int x, int y, int j, uint64_t seed, double ray6[6]) {
  T t; memset(&t, 0, sizeof t);
  Ray r = lens(s, x, y, j, seed, &t);
  ray6[0] = r.d.x; ray6[1] = r.d.y; ray6[2] = r.d.z;
  ray6[3] = r.o.x; ray6[4] = r.o.y; ray6[5] = r.o.z;
}

/* Camera#render_fork + fork_jobs (camera.rb:41-68, fork_jobs.rb:1-33): nprocs
 * forked children, child i renders columns [floor(i/n*W), floor((i+1)/n*W))
 * (restricted to columns x % col_stride == 0, the bounded baseline sample) over
 * all rows, results exchanged through a shared mapping instead of JSON files.
 * out: full H x W x 3 frame (only sampled columns written). Returns 0 / -errno. */
int rto_render_fork(Scene* s, int nprocs, int col_stride, uint64_t seed, double* out) {
  const int W = s->cam.width, H = s->cam.height;
  size_t bytes = sizeof(double) * 3 * (size_t)W * H;
  double* shm = (double*)mmap(NULL, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (shm == MAP_FAILED) return -1;
  pid_t* pids = (pid_t*)calloc(nprocs, sizeof(pid_t));
  for (int i = 0; i < nprocs; i++) {
    pid_t pid = fork();
    if (pid == 0) {
      int sx = (int)((double)i / nprocs * W), ex = (int)((double)(i + 1) / nprocs * W);
      Tr tr;
      tr_init(&tr, s, seed);
      for (int x = sx; x < ex; x++) {
        if (x % col_stride) continue;
        for (int y = 0; y < H; y++) {
          T t; memset(&t, 0, sizeof t);
          V c = render_at(&tr, x, y, &t);
          double* p = shm + ((size_t)y * W + x) * 3;
          p[0] = c.x; p[1] = c.y; p[2] = c.z;
        }
      }
      _exit(0);
    }
    pids[i] = pid;
  }
  int rc = 0;
  for (int i = 0; i < nprocs; i++) {
    int st = 0;
    if (pids[i] <= 0 || waitpid(pids[i], &st, 0) < 0 || !WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = -2;
  }
  memcpy(out, shm, bytes);
  munmap(shm, bytes);
  free(pids);
  return rc;
}
