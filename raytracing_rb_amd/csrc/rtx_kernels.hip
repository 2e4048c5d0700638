// rtx_kernels.hip — the hot path of a1exwang/raytracing_rb on gfx950 (CDNA4).
//
//   Camera#render_at  (src/camera.rb:70-99)   adaptive sampling of one pixel
//   Camera#lens_func  (src/camera.rb:129-151) thin-lens primary ray
//   RayTracer#trace_sync / #rt_map (src/ray_tracer.rb:16-164, 292-298)
//   World#intersect / #lit_area / #local_lights / #high_lights (src/world.rb:37-98)
//   Sphere / Plane / Box / Texture (src/objects/*.rb)
//
// Design: one pixel per lane, binary64 everywhere, built with
// -ffp-contract=off so every operation rounds exactly as the Ruby + C-extension
// program does.  Each lane runs ONE flat loop over the work of its pixel —
// pop a pending ray / start the next camera sample / finish the pixel — so a
// lane whose sample tree is done immediately starts its next sample instead
// of idling until the wave's deepest tree finishes.  The ray tree is walked
// depth-first with the reference's LIFO order (children pushed reflection,
// refraction, path-tracing rays; last pushed is processed first) on a
// per-lane stack, and leaf colours are summed in emission order, which is the
// reference's FIFO drain order (ray_tracer.rb:31-45), so sums are bit-exact.
//
// The scene loops (World#intersect over every object, World#lit_area over
// every object per light) run in YAML order on a wave-uniform index, so the
// object records are wave-uniform loads (scalar/broadcast).  Spheres that the
// exact test would reject are skipped by a division-free conservative
// pre-test whose margins are proven safe in DESIGN.md ("exact culls"); it
// changes no bit of any result.
#include <hip/hip_runtime.h>

#include "rtx_launch.h"
#include "rtx_scene.h"
#include "rtx_vec3.h"

namespace rtx {

constexpr double PI = 3.141592653589793;   // Math::PI == M_PI
constexpr double EPS = 1e-5;               // Alex::EPSILON (src/libs/algebra.rb:2)

struct Ray {
  V3 o, d;                          // Alex::Ray#position, #front
};

struct Item {                       // one queue entry of RayTracer (ray_tracer.rb:21-30)
  Ray ray;
  V3 att;
  uint64_t path;                    // RNG ray-path id (DESIGN.md "RNG")
  int32_t depth;
  int32_t pad;
};

// Per-ray constants shared by every object test of the ray.
struct RayC {
  V3 o, d;
  V3 dn;        // front.normalize (recomputed by the reference per call; same bits)
  double r2;    // front.r2 = r*r
  double dd;    // d.d, cull only
  double so;    // |o|_1, cull only
};

enum { C_RAYS = 0, C_SPHERE_TESTS, C_SPHERE_HITS, C_PLANE_TESTS, C_BOX_TESTS, C_SHADE_HITS,
       C_COVER_SPHERE, C_COVER_PLANE, C_COVER_BOX, C_HIGHLIGHT_TESTS, C_PRIMARY, C_N };

__device__ __forceinline__ RayC make_rayc(V3 o, V3 d) {
  RayC c;
  c.o = o;
  c.d = d;
  double r = vr(d);
  c.r2 = r * r;
  c.dn = r == 0 ? d : v3(d.x / r, d.y / r, d.z / r);
  c.dd = vsq(d);
  c.so = fabs(o.x) + fabs(o.y) + fabs(o.z);
  return c;
}

// ----------------------------------------------------------------- spheres
// Exact Sphere#intersect (sphere.rb:60-85) preceded by the conservative cull.
// Returns true and the hit point if the reference returns non-nil.
__device__ __forceinline__ bool sphere_hit(const double* __restrict__ g, const RayC& rc, V3& hit,
                                           bool& in, double& tq) {
  const V3 C = v3(g[0], g[1], g[2]);
  const double R = g[3];
  const V3 oc = vsub(C, rc.o);                    // (center - ray.position)
  const double q = vdot(oc, rc.d);                // .dot(ray.front)
  const double s = vsq(oc);                       // == |position - center|^2, same bits
  // cull 1: the ray's line misses the sphere by a margin (exact culls)
  const double S = rc.so + g[5];
  if (s * rc.dd - q * q > rc.dd * (g[4] + 1e-10 * (S * S))) return false;
  // cull 2: sphere behind an origin that is outside it
  if (q < -1e-200 && s > g[4] * (1.0 + 1e-9)) return false;
  const double t = q / rc.r2;
  const V3 np = vadd(rc.o, vsc(rc.d, t));
  const double nd = vr(vsub(np, C));
  if (!(nd <= R)) return false;                   // inner?(nearest_point)
  const double h = sqrt(R * R - nd * nd);         // radius**2 - nearest_dis**2
  const V3 vec = vsc(rc.dn, h);
  const bool from_inner = sqrt(s) <= R;           // inner?(ray.position)
  in = !from_inner;
  hit = in ? vsub(np, vec) : vadd(np, vec);
  if (!from_inner && t < 0) return false;
  tq = t;
  return true;
}

// ----------------------------------------------------------------- planes
// Plane#intersect (plane.rb:38-51).  p = plane record (PLANE_GEO doubles).
__device__ __forceinline__ bool plane_hit(const double* __restrict__ p, const RayC& rc, V3& hit) {
  const V3 F = v3(p[3], p[4], p[5]);
  const double den = vdot(F, rc.d);
  if (den == 0) return false;
  const double t = vdot(vsub(v3(p[0], p[1], p[2]), rc.o), F) / den;
  hit = vadd(rc.o, vsc(rc.d, t));
  if (t < 0) return false;
  return true;
}

__device__ __forceinline__ void plane_uv(const double* __restrict__ p, V3 pos, double& u, double& v) {
  const V3 a = vsub(pos, v3(p[0], p[1], p[2]));   // plane.rb:81-85
  u = vdot(a, v3(p[6], p[7], p[8])) / p[12];
  v = vdot(a, v3(p[9], p[10], p[11])) / p[13];
}

// Box#intersect (box.rb:79-97): nearest face hit inside its u,v square.
__device__ __forceinline__ bool box_hit(const double* __restrict__ b, const RayC& rc, V3& hit, int& face) {
  double nearest = __builtin_inf();
  bool found = false;
  for (int i = 0; i < 6; i++) {
    const double* p = b + i * PLANE_GEO;
    V3 h;
    if (plane_hit(p, rc, h)) {
      double u, v;
      plane_uv(p, h, u, v);
      if (-0.5 <= u && u <= 0.5 && -0.5 <= v && v <= 0.5) {
        const double d = vr(vsub(h, rc.o));
        if (d < nearest) {
          nearest = d;
          hit = h;
          face = i;
          found = true;
        }
      }
    }
  }
  return found;
}

// ----------------------------------------------------------------- errors
__device__ __forceinline__ void seterr(uint32_t& err, uint32_t code) {
  if (!err) err = code;
}

// ----------------------------------------------------------------- lit_area
// World#lit_area (world.rb:62-69) for target T and light L: 1 - sum of
// cover_area over every object in YAML order, clamped at 0.  Objects whose
// cover is zero are skipped (subtracting 0 is exact).
template <bool COUNT>
__device__ double lit_area(const SceneDev& S, V3 T, V3 L, double radius, uint32_t& err,
                           unsigned long long* cnt) {
  const RayC rc = make_rayc(T, vsub(L, T));      // Ray(light - target, target)
  const V3 TL = vsub(T, L);
  double total = 1.0;
  if (COUNT) {
    cnt[C_COVER_SPHERE] += S.n_sphere;
    cnt[C_COVER_PLANE] += S.n_plane;
    cnt[C_COVER_BOX] += S.n_box;
  }
  for (int i = 0; i < S.n_obj; i++) {
    const ObjInfo oi = S.info[i];
    const double* __restrict__ g = S.geo + oi.geo;
    V3 hit;
    if (oi.type == OBJ_SPHERE) {
      bool in;
      double tq;
      if (!sphere_hit(g, rc, hit, in, tq)) continue;
      if (!(vdot(vsub(hit, L), TL) > 0)) continue;             // factor == 0
      // Sphere#cover_area penumbra (sphere.rb:31-56), factor == 1
      const V3 C = v3(g[0], g[1], g[2]);
      const double R = g[3];
      const V3 lt = rc.d;
      const double t = vdot(vsub(C, T), lt) / vr2(lt);
      const V3 x1 = vadd(T, vsc(lt, t));
      const double r1 = radius * (vr(vsub(x1, T)) / vr(lt));
      const double d = vr(vsub(x1, C));
      if (d >= r1 + R) continue;
      const double s1 = PI * r1 * r1;
      double cover;
      if (d > fabs(R - r1)) {
        double c1 = (r1 * r1 + d * d - R * R) / (2.0 * r1 * d);
        double c2 = (R * R + d * d - r1 * r1) / (2.0 * R * d);
        if (c1 > 1.0) c1 = 1.0;
        if (c2 > 1.0) c2 = 1.0;
        if (c1 < -1.0 || c2 < -1.0) seterr(err, ERR_DOMAIN);   // Math::DomainError
        const double th1 = acos(c1), th2 = acos(c2);
        const double ds = ((th1 - sin(th1)) * r1 * r1 + (th2 - sin(th2)) * R * R) / 2.0;
        cover = 1.0 * ds / s1;
      } else if (r1 > R) {
        cover = 1.0 * PI * R * R / s1;
      } else {
        cover = 1.0;
      }
      total -= cover;
    } else if (oi.type == OBJ_PLANE) {
      if (plane_hit(g, rc, hit) && vdot(vsub(hit, L), TL) > 0) total -= 1.0;
    } else {
      int face;
      if (box_hit(g, rc, hit, face) && vdot(vsub(hit, L), TL) > 0) total -= 1.0;
    }
  }
  return total > 0 ? total : 0.0;
}

// ----------------------------------------------------------------- shading
__device__ __forceinline__ Ray reflection(const Ray& ray, V3 n, V3 hit, V3 delta, uint32_t& err) {
  // WorldObject#get_reflection_by_ray_and_n (world_object.rb:121-125)
  const double c = vcos(ray.d, vneg(n), err);
  Ray r;
  r.d = vnorm(vadd(vsc(vnorm(n, err), 2.0 * c * vr(ray.d)), ray.d), err);
  r.o = vadd(hit, delta);
  return r;
}

__device__ __forceinline__ bool refraction(const Ray& ray, V3 n, V3 hit, V3 refl, double rate, Ray& out,
                                           uint32_t& err) {
  // WorldObject#get_refraction_by_ray_and_n (world_object.rb:127-137)
  const double c = vcos(ray.d, n, err);
  const double sin_i = sqrt(1.0 - c * c);        // 1 - cos**2
  const double sin_r = sin_i / rate;
  if (sin_r >= 1) return false;                  // total internal reflection
  const double r = asin(sin_r);
  const V3 nn = vnorm(n, err);
  out.d = vadd(vsc(nn, -cos(r)), vsc(vnorm(vadd(refl, ray.d), err), sin_r));
  out.o = vsub(hit, vsc(nn, EPS));
  return true;
}

__device__ __forceinline__ V3 texcolor(const SceneDev& S, int tex, double hs, double vs, double uo,
                                       double vo, double uu, double vv, uint32_t& err) {
  // Texture#color (texture.rb:23-28): trunc, then Ruby's floor-mod.
  const TexDev t = S.tex[tex];
  const double qu = (uu + uo) / hs, qv = (vv + vo) / vs;
  if (!isfinite(qu) || !isfinite(qv)) {
    seterr(err, ERR_DOMAIN);                     // FloatDomainError in Float#to_i
    return v3(0.0, 0.0, 0.0);
  }
  long iu = (long)fmod(trunc(qu), (double)t.w);
  long iv = (long)fmod(trunc(qv), (double)t.h);
  if (iu < 0) iu += t.w;
  if (iv < 0) iv += t.h;
  const uint8_t* p = S.texels + t.off + ((size_t)iv * t.w + iu) * 3;
  return v3(p[0] / 256.0, p[1] / 256.0, p[2] / 256.0);
}

__device__ __forceinline__ V3 vertical_vector(V3 n, uint32_t& err) {   // world_object.rb:105-120
  if (vr(n) == 0) {
    seterr(err, ERR_ZERO_VEC);
    return v3(1.0, 0.0, 0.0);
  }
  if (n.x == 0) {
    if (n.y == 0) return v3(1.0, 0.0, 0.0);
    return v3(0.0, -n.z / n.y, 1.0);
  }
  return v3(-(n.y + n.z) / n.x, 1.0, 1.0);
}

struct Pixel {
  uint64_t seed;
  int32_t x, y, sample;
};

template <int MAXS>
struct Stack {
  Item a[MAXS];
  int n;
};

// Push a child unless rt_map would discard it on pop (ray_tracer.rb:52):
// skipping a dead item changes nothing (no leaf, no RNG draw).
template <int MAXS>
__device__ __forceinline__ void push_child(Stack<MAXS>& st, const Ray& r, V3 att, uint64_t path, int depth) {
  if (depth <= 0 || vr(att) < 0.0001) return;
  if (st.n < MAXS) {
    Item& it = st.a[st.n++];
    it.ray = r;
    it.att = att;
    it.path = path;
    it.depth = depth;
  }
}

__device__ __forceinline__ void add_leaf(V3& sum, V3 c, uint32_t& err) {   // ray_tracer.rb:292-298
  sum = vadd(sum, c);
  if (!(sum.x <= 1 && sum.y <= 1 && sum.z <= 1)) seterr(err, ERR_COLOR_GT1);
}

// RayTracer#rt_map (ray_tracer.rb:50-164) for one live item: leaves go into
// `sum`, children onto the stack.
template <bool COUNT, int MAXS>
__device__ void rt_map(const SceneDev& S, const CameraDev& cam, const Pixel& px, const Item& it,
                       Stack<MAXS>& st, V3& sum, uint32_t& err, unsigned long long* cnt) {
  if (it.depth <= 0 || vr(it.att) < 0.0001) return;
  if (COUNT) {
    cnt[C_RAYS]++;
    cnt[C_HIGHLIGHT_TESTS] += S.n_light;
  }
  const Ray& ray = it.ray;
  // ---- World#high_lights (world.rb:83-98); the `&& lit_area(...)` is always
  // truthy in Ruby and is not evaluated.
  uint32_t fired = 0;
  int nfired = 0;
  for (int l = 0; l < S.n_light; l++) {
    const LightDev& L = S.light[l];
    const V3 a = vsub(v3p(L.pos), ray.o);
    const double dot = vdot(ray.d, a);
    const double r1 = vsq(ray.d), r2 = vsq(a);
    if (r1 == 0 || r2 == 0) {
      seterr(err, ERR_ZERO_VEC);
      continue;
    }
    bool fire;
    const double g = dot * dot, h = r1 * r2;
    if (L.hl_mode == 2) {
      fire = false;
    } else if (L.hl_mode == 0 && g > L.cos_hi2 * h) {
      fire = true;                                  // |cos| surely above cos(angle)
    } else if (L.hl_mode == 0 && g < L.cos_lo2 * h) {
      fire = false;                                 // |cos| surely below cos(angle)
    } else {
      double c = sqrt(g / r1 / r2);                 // Vec3#cos exactly
      if (c > 1) c = 1;
      if (c < -1) c = -1;
      fire = acos(c) < L.hl_angle_rad;
    }
    if (fire) {
      fired |= 1u << l;
      nfired++;
    }
  }
  if (nfired) {
    for (int l = 0; l < S.n_light; l++) {
      if (!(fired >> l & 1)) continue;
      const LightDev& L = S.light[l];
      add_leaf(sum, vdiv(vmul(it.att, vsc(v3p(L.color), L.hl_rate)), (double)nfired), err);
    }
    return;
  }
  // ---- World#intersect (world.rb:37-59): nearest hit, YAML order, strict <.
  const RayC rc = make_rayc(ray.o, ray.d);
  double best = S.max_distance;
  int besti = -1;
  if (COUNT) {
    cnt[C_SPHERE_TESTS] += S.n_sphere;
    cnt[C_PLANE_TESTS] += S.n_plane;
    cnt[C_BOX_TESTS] += S.n_box;
  }
  for (int i = 0; i < S.n_obj; i++) {
    const ObjInfo oi = S.info[i];
    const double* __restrict__ g = S.geo + oi.geo;
    V3 hit;
    bool ok;
    if (oi.type == OBJ_SPHERE) {
      bool in;
      double tq;
      ok = sphere_hit(g, rc, hit, in, tq);
      if (COUNT && ok) cnt[C_SPHERE_HITS]++;
    } else if (oi.type == OBJ_PLANE) {
      ok = plane_hit(g, rc, hit);
    } else {
      int face;
      ok = box_hit(g, rc, hit, face);
    }
    if (ok) {
      const double d = vr(vsub(rc.o, hit));         // Ray#distance
      if (d < best) {
        best = d;
        besti = i;
      }
    }
  }
  if (besti < 0) return;                            // "light_dead": contributes nothing
  if (COUNT) cnt[C_SHADE_HITS]++;
  // ---- re-evaluate the winner fully (same operations => same bits)
  const ObjInfo oi = S.info[besti];
  const double* __restrict__ g = S.geo + oi.geo;
  const Material& m = S.mat[besti];
  V3 hit, delta, n;
  Ray refl, refr;
  bool has_refr;
  const double* plane = nullptr;
  if (oi.type == OBJ_SPHERE) {                      // sphere.rb:60-101
    bool in;
    double tq;
    sphere_hit(g, rc, hit, in, tq);
    const V3 C = v3(g[0], g[1], g[2]);
    delta = vsc(vsc(vsub(hit, C), EPS), in ? 1.0 : -1.0);
    n = in ? vsub(hit, C) : vsub(C, hit);
    refl = reflection(ray, n, hit, delta, err);
    has_refr = refraction(ray, n, hit, refl.d, in ? m.rr : 1.0 / m.rr, refr, err);
  } else {                                          // plane.rb:38-67, box.rb:100-105
    if (oi.type == OBJ_PLANE) {
      plane = g;
      plane_hit(g, rc, hit);
    } else {
      int face = 0;
      box_hit(g, rc, hit, face);
      plane = g + face * PLANE_GEO;
    }
    const V3 F = v3(plane[3], plane[4], plane[5]);
    const double fd = vdot(F, ray.d);
    const double nfd = -fd;
    delta = vsc(vsc(F, EPS), nfd > 0 ? 1.0 : (nfd < 0 ? -1.0 : 0.0));   // (-f.d <=> 0).to_f
    n = fd > 0 ? vneg(F) : F;
    refl = reflection(ray, n, hit, delta, err);
    has_refr = m.has_rr ? refraction(ray, n, hit, refl.d, m.rr, refr, err) : false;
  }
  const uint64_t R = (uint64_t)cam.pt + 3;
  push_child<MAXS>(st, refl, vmul(it.att, v3p(m.refl_att)), it.path * R + 1, it.depth - 1);
  if (has_refr) push_child<MAXS>(st, refr, vmul(it.att, v3p(m.refr_att)), it.path * R + 2, it.depth - 1);
  // ---- World#local_lights (world.rb:72-80) at hit + delta, fused with the
  // light loop of WorldObject#local_lighting (world_object.rb:51-74): same
  // light order, same sums.
  const V3 T = vadd(hit, delta);
  V3 lc = v3(0.0, 0.0, 0.0);
  int nl = 0;
  for (int l = 0; l < S.n_light; l++) {
    const LightDev& L = S.light[l];
    const double area = lit_area<COUNT>(S, T, v3p(L.pos), L.radius, err, cnt);
    if (area > 0) {
      nl++;
      const double p = S.sse_is_two ? area * area : pow(area, S.sse);
      const V3 lcol = vsc(v3p(L.color), p / (double)S.n_light);
      const V3 nn = vnorm(n, err);
      const V3 ll = vnorm(vsub(v3p(L.pos), hit), err);
      double ldn = vdot(ll, nn);
      if (ldn > 1) ldn = 1.0;
      else if (ldn < 0) ldn = 0.0;
      lc = vadd(lc, vsc(lcol, ldn));
    }
  }
  if (nl == 0) {
    // WorldObject#path_tracing (world_object.rb:76-90) from hit + delta
    const int pt = cam.pt;
    const V3 att = vdiv(v3p(m.diffuse), (double)pt);
    const V3 front = vnorm(n, err);
    const V3 left = vnorm(vertical_vector(n, err), err);
    const V3 up = vcross(front, left);
    for (int k = 0; k < pt; k++) {
      const double theta = rand01(px.seed, px.x, px.y, px.sample, it.path, 2 * k) * PI / 2.0;
      const double phi = rand01(px.seed, px.x, px.y, px.sample, it.path, 2 * k + 1) * PI * 2.0;
      Ray r;
      r.o = T;
      r.d = vadd(vsc(front, sin(theta)), vsc(vadd(vsc(left, cos(phi)), vsc(up, sin(phi))), cos(theta)));
      push_child<MAXS>(st, r, vmul(it.att, att), it.path * R + 3 + (uint64_t)k, it.depth - 1);
    }
    return;
  }
  lc = vdiv(lc, (double)nl);
  V3 color;
  if (oi.type == OBJ_BOX) {
    color = vadd(vmul(lc, v3p(m.diffuse)), v3p(m.ambient));
  } else {
    V3 filter = v3(1.0, 1.0, 1.0);
    if (m.tex >= 0) {
      if (oi.type == OBJ_SPHERE) {                  // Sphere#get_uv (sphere.rb:111-120)
        const V3 vec = vsub(hit, v3(g[0], g[1], g[2]));
        const double R0 = g[3];
        const double x = vdot(vec, v3p(m.gw_n)) / R0;
        const double y = vdot(vec, v3p(m.east_n)) / R0;
        const double z = vdot(vec, v3p(m.north_n)) / R0;
        const double mm2 = x * x + y * y + z * z + 2.0 * x + 1.0;
        if (mm2 < 0) seterr(err, ERR_DOMAIN);
        const double mm = sqrt(mm2);
        filter = vmul(texcolor(S, m.tex, m.hs, m.vs, m.u_off, m.v_off, (y / mm + 1.0) / 2.0,
                               (-z / mm + 1.0) / 2.0, err), filter);
      } else {
        double u, v;
        plane_uv(plane, hit, u, v);
        filter = vmul(texcolor(S, m.tex, m.hs, m.vs, 0.0, 0.0, u, v, err), filter);
      }
    }
    color = vadd(vmul(vmul(lc, v3p(m.diffuse)), filter), v3p(m.ambient));
  }
  add_leaf(sum, vmul(it.att, color), err);
}

// Camera#lens_func (camera.rb:129-151) with the per-camera constants hoisted.
__device__ __forceinline__ Ray lens(const CameraDev& c, int x, int y, int j, uint64_t seed) {
  const V3 rp = vadd(vadd(v3p(c.retina_center), vsc(v3p(c.left), 2.0 * ((double)x / c.width - 0.5) * c.retina_width)),
                     vsc(v3p(c.up_n), 2.0 * ((double)y / c.height - 0.5) * c.retina_height));
  const double theta = rand01(seed, x, y, j, 0, 0);
  const V3 rv = vsc(vadd(vsc(v3p(c.left_n), cos(theta)), vsc(v3p(c.up_n), sin(theta))), c.aperture_radius);
  const V3 pos = v3p(c.pos);
  const V3 ap = vadd(pos, rv);
  const V3 rd = vsub(pos, rp);                                  // Ray(position - retina, retina)
  const double t = vdot(vsub(v3p(c.pofp), rp), v3p(c.front)) / vdot(v3p(c.front), rd);
  const V3 target = vadd(rp, vsc(rd, t));
  Ray r;
  r.o = ap;
  r.d = vsub(target, ap);
  return r;
}

__device__ __forceinline__ void record_error(ErrState* e, uint32_t code, int x, int y, int W) {
  atomicOr(&e->flags, 1u << code);
  atomicMin(&e->first[code], (unsigned long long)y * (unsigned long long)W + (unsigned long long)x);
}

__device__ __forceinline__ int row_to_y(const KParams& p, int row) {
  if (p.tile_rows == 0) return p.y0 + row;
  const int k = row / p.tile_rows;
  return (k * p.nranks + p.rank) * p.tile_rows + (row - k * p.tile_rows);
}

// One lane per pixel; a wave covers an 8x8 pixel tile, a 256-thread block 4 tiles.
template <bool COUNT, int MAXS, int MAXPRE, int WPS>
__global__ __launch_bounds__(256, WPS) void k_render(KParams p) {
  const int lane = threadIdx.x & 63;
  const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int tiles_x = (p.nx + 7) >> 3;
  const int px_ = (tile % tiles_x) * 8 + (lane & 7);
  const int row = (tile / tiles_x) * 8 + (lane >> 3);
  if (px_ >= p.nx || row >= p.nrows) return;
  const int y = row_to_y(p, row);
  if (y >= p.cam->height) return;
  const int x = p.x0 + px_;
  const SceneDev& S = *p.scene;
  const CameraDev& cam = *p.cam;

  unsigned long long cnt[C_N];
  if (COUNT)
    for (int k = 0; k < C_N; k++) cnt[k] = 0;

  Pixel pix;
  pix.seed = p.seed;
  pix.x = x;
  pix.y = y;
  Stack<MAXS> st;
  st.n = 0;
  V3 smp[MAXPRE];
  uint32_t err = 0;
  const int pre = cam.pre;
  int ntot = pre;
  bool extra = false;
  V3 avg = v3(0.0, 0.0, 0.0), cv = v3(0.0, 0.0, 0.0), sum = v3(0.0, 0.0, 0.0);
  int j = 0;
  // Camera#render_at (camera.rb:70-99) as one flat loop over all its rays.
  Item cur;
  cur.ray = lens(cam, x, y, 0, p.seed);
  cur.att = v3(1.0, 1.0, 1.0);
  cur.path = 1;
  cur.depth = cam.depth;
  pix.sample = 0;
  if (COUNT) cnt[C_PRIMARY]++;
  bool have = true;
  while (true) {
    if (!have) {
      if (st.n > 0) {
        cur = st.a[--st.n];
      } else {
        // sample j is complete
        if (j < pre) {
          smp[j] = sum;
          avg = vadd(avg, sum);
        } else {
          cv = vadd(cv, sum);
        }
        j++;
        if (j == pre) {
          avg = vdiv(avg, (double)pre);
          double variance = 0.0;
          for (int k = 0; k < pre; k++) {
            const V3 dd = vsub(smp[k], avg);
            double mx = dd.x;
            if (dd.y > mx) mx = dd.y;
            if (dd.z > mx) mx = dd.z;
            variance += mx * mx;               // .max ** 2
          }
          variance /= (double)pre;
          if (variance >= cam.variant_threshold) {
            extra = true;
            ntot = cam.max_samples;
          }
        }
        if (j >= ntot) break;
        sum = v3(0.0, 0.0, 0.0);
        cur.ray = lens(cam, x, y, j, p.seed);
        cur.att = v3(1.0, 1.0, 1.0);
        cur.path = 1;
        cur.depth = cam.depth;
        pix.sample = j;
        if (COUNT) cnt[C_PRIMARY]++;
      }
    }
    have = false;
    rt_map<COUNT, MAXS>(S, cam, pix, cur, st, sum, err, cnt);
  }
  if (extra) avg = vdiv(vadd(vsc(avg, (double)pre), cv), (double)cam.max_samples);
  double* o = p.out + (size_t)row * p.stride + (size_t)px_ * 3;
  o[0] = avg.x;
  o[1] = avg.y;
  o[2] = avg.z;
  if (err) record_error(p.err, err, x, y, cam.width);
  if (COUNT)
    for (int k = 0; k < C_N; k++) atomicAdd(&p.counts[k], cnt[k]);
}

// RayTracer#trace_sync(x, y, ray) for explicit rays: rays[i] = (front, position).
template <int MAXS>
__global__ __launch_bounds__(256) void k_trace(KParams p, const double* __restrict__ rays,
                                               const int32_t* __restrict__ keys, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Pixel pix;
  pix.seed = p.seed;
  pix.x = keys[3 * i];
  pix.y = keys[3 * i + 1];
  pix.sample = keys[3 * i + 2];
  Stack<MAXS> st;
  st.n = 0;
  uint32_t err = 0;
  V3 sum = v3(0.0, 0.0, 0.0);
  Item cur;
  cur.ray.d = v3p(rays + 6 * i);
  cur.ray.o = v3p(rays + 6 * i + 3);
  cur.att = v3(1.0, 1.0, 1.0);
  cur.path = 1;
  cur.depth = p.cam->depth;
  while (true) {
    rt_map<false, MAXS>(*p.scene, *p.cam, pix, cur, st, sum, err, nullptr);
    if (st.n == 0) break;
    cur = st.a[--st.n];
  }
  p.out[3 * i] = sum.x;
  p.out[3 * i + 1] = sum.y;
  p.out[3 * i + 2] = sum.z;
  if (err) record_error(p.err, err, i, 0, 0x7fffffff);
}

// Camera#array_to_color (camera.rb:153-156) + PNG::Canvas#point over black.
__global__ void k_quantize(const double* __restrict__ rgb, int w, int h, size_t stride, int blend,
                           uint8_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= w * h) return;
  const int y = i / w, x = i - y * w;
  const double* c = rgb + (size_t)y * stride + (size_t)x * 3;
  uint8_t* o = out + (size_t)i * 4;
  for (int k = 0; k < 3; k++) {
    double v = c[k] * 256.0;
    if (!(v < 255.0)) v = 255.0;                  // [x, 255].min
    int b = v > 0 ? (int)v : 0;                   // "%c" truncation
    if (blend) b = (b * 255) >> 8;                // Color#blend over Black, alpha 255
    o[k] = (uint8_t)b;
  }
  o[3] = 255;
}

// ----------------------------------------------------------------- launchers
int stack_bucket(int need) {
  if (need <= 8) return 8;
  if (need <= 16) return 16;
  if (need <= 32) return 32;
  if (need <= 64) return 64;
  return -1;
}

hipError_t launch_render(const KParams& p, bool count, int maxs, int wps, hipStream_t s) {
  const int tiles = ((p.nx + 7) / 8) * ((p.nrows + 7) / 8);
  const dim3 grid((tiles + 3) / 4), block(256);
  if (tiles == 0) return hipSuccess;
#define RTX_L(C, M, W)                                                   \
  if (count == C && maxs == M && wps == W) {                             \
    hipLaunchKernelGGL((k_render<C, M, 16, W>), grid, block, 0, s, p);  \
    return hipGetLastError();                                            \
  }
  RTX_L(false, 8, 2) RTX_L(false, 16, 2) RTX_L(false, 32, 2) RTX_L(false, 64, 2)
  RTX_L(false, 16, 1) RTX_L(false, 16, 3) RTX_L(false, 16, 4)
  RTX_L(true, 8, 2) RTX_L(true, 16, 2) RTX_L(true, 32, 2) RTX_L(true, 64, 2)
#undef RTX_L
  return hipErrorInvalidValue;
}

hipError_t launch_trace(const KParams& p, const double* rays, const int32_t* keys, int n, int maxs,
                        hipStream_t s) {
  const dim3 grid((n + 255) / 256), block(256);
  if (n == 0) return hipSuccess;
  switch (maxs) {
    case 8: hipLaunchKernelGGL((k_trace<8>), grid, block, 0, s, p, rays, keys, n); break;
    case 16: hipLaunchKernelGGL((k_trace<16>), grid, block, 0, s, p, rays, keys, n); break;
    case 32: hipLaunchKernelGGL((k_trace<32>), grid, block, 0, s, p, rays, keys, n); break;
    case 64: hipLaunchKernelGGL((k_trace<64>), grid, block, 0, s, p, rays, keys, n); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_quantize(const double* rgb, int w, int h, size_t stride, int blend, uint8_t* out,
                           hipStream_t s) {
  const int n = w * h;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_quantize, dim3((n + 255) / 256), dim3(256), 0, s, rgb, w, h, stride, blend, out);
  return hipGetLastError();
}

}  // namespace rtx
