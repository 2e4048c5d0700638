// rtx_kernels.hip — the hot path of a1exwang/raytracing_rb on gfx950 (CDNA4).
//
//   Camera#render_at  (src/camera.rb:70-99)   adaptive sampling of one pixel
//   Camera#lens_func  (src/camera.rb:129-151) thin-lens primary ray
//   RayTracer#trace_sync / #rt_map (src/ray_tracer.rb:16-164, 292-298)
//   World#intersect / #lit_area / #local_lights / #high_lights (src/world.rb:37-98)
//   Sphere / Plane / Box / Texture (src/objects/{sphere,plane,box,texture}.rb)
//
// Design: one pixel per lane, binary64 for every value the
// reference computes, built with -ffp-contract=off so each operation rounds
// exactly as the Ruby + C-extension program does.
//
// Each lane runs a small state machine.  Every loop iteration executes ONE
// "query" — an ordered walk over all objects of the scene with one ray — for
// every active lane at once: either the nearest-hit walk of World#intersect
// (EXTEND) or the cover-area walk of World#lit_area for one light (SHADOW).
// Both kinds run in the same object loop, so lanes at different stages of
// their ray trees stay converged in the expensive part.  Between queries a
// lane does its divergent-but-short work: pop the next ray of its tree (LIFO,
// as RayTracer#trace_sync), start the next camera sample, the highlight test,
// shading and child-ray generation.  The last child generated is kept in
// registers (it is the next one the LIFO would pop); only its older siblings
// go to the per-lane stack.  Leaf colours are summed in emission order —
// the reference's FIFO drain order (ray_tracer.rb:31-45) — so sums are exact.
//
// Spheres are first tested with a float32 conservative pre-test from a
// 16-byte record staged in LDS; only spheres it cannot rule out run the exact
// binary64 Sphere#intersect.  The pre-test margins are proven in DESIGN.md
// ("exact culls"): it never rejects a sphere the exact test would accept,
// so it changes no bit of any result.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rtx_launch.h"
#include "rtx_scene.h"
#include "rtx_vec3.h"

namespace rtx {

constexpr double PI = 3.141592653589793;   // Math::PI == M_PI
constexpr double EPS = 1e-5;               // Alex::EPSILON (src/libs/algebra.rb:2)
constexpr float CULL_M = 2e-5f;            // pre-test margin (exact culls)

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

enum { C_RAYS = 0, C_SPHERE_TESTS, C_SPHERE_HITS, C_PLANE_TESTS, C_BOX_TESTS, C_SHADE_HITS,
       C_COVER_SPHERE, C_COVER_PLANE, C_COVER_BOX, C_HIGHLIGHT_TESTS, C_PRIMARY, C_N };

enum { M_NEED = 0, M_EXTEND = 1, M_SHADOW = 2, M_DONE = 3, M_FETCH = 4 };

// Out-of-line the rarely-executed shading blocks (1) or inline everything (0).
#ifndef RTX_OUTLINE_SHADING
#define RTX_OUTLINE_SHADING 0
#endif
#if RTX_OUTLINE_SHADING
#define RTX_SHADE_FN __device__ __noinline__
#else
#define RTX_SHADE_FN __device__ __forceinline__
#endif

// The scene is read-only for the whole launch: reading it through the constant
// address space (4) lets wave-uniform indices become scalar loads (s_load) into
// SGPRs instead of per-lane vector loads.
#define RTX_CONST __attribute__((address_space(4)))
template <typename T>
__device__ __forceinline__ const RTX_CONST T* cptr(const T* p) {
  return (const RTX_CONST T*)(p);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
enum { SRC_PIXELS = 0, SRC_RAYS = 1, SRC_EXTRA = 2, SRC_LIST = 3 };
#ifndef RTX_CLAIM_MAX
#define RTX_CLAIM_MAX 64     // cap on the items a wave claims beyond its lanes' need (with expensive tiles first + Morton items: 32: C2 8.68 ms, 64: 8.30 ms, 96: 9.13 ms, 128: 9.58 ms — expensive tiles pile up in one wave)
#endif

// Diagnostic build only (-DRTX_STAMPS=1): per-wave shader-clock time spent in
// each phase of the lane state machine, summed into rtx_stamps[] (read with
// rtxdbg_read_stamps).  The shipped library is built without it.
#ifndef RTX_CLAIM_DIV
#define RTX_CLAIM_DIV 2      // a claim's extra items: at most remaining / (RTX_CLAIM_DIV x waves) (C2: 2: 8.27 ms, 4: 8.35-8.48 ms, 8: 8.37 ms)
#endif
#ifndef RTX_CLAIM_ALIGN
#define RTX_CLAIM_ALIGN 1    // claims rounded up to a multiple of this (every claimed range then starts aligned; 64: C2 9.2 ms, worse)
#endif
#ifndef RTX_PROBE_W
#define RTX_PROBE_W 0        // k_tile_cost hit weights: 0 (1, +1 reflective, +3 refractive), 1 (1, +1/+2 by reflectance, +6 refractive)
#endif
#ifndef RTX_ITEM_ORDER
#define RTX_ITEM_ORDER 1     // SRC_PIXELS items within a tile: 1 (pixel Morton, sample; C2 8.75 -> 8.65 ms, C4 505 -> 495 ms), 0 (sample, pixel row-major)
#endif
#ifndef RTX_DIAG_NOEXACT
#define RTX_DIAG_NOEXACT 0
#endif
#ifndef RTX_STAMPS
#define RTX_STAMPS 0
#endif
#ifndef RTX_LVL_WPS
#define RTX_LVL_WPS 2        // waves per SIMD k_level is compiled for
#endif
#ifndef RTX_LV_CLAIM_AHEAD
#define RTX_LV_CLAIM_AHEAD 0 // k_level claims its next 64-ray chunk while working on the current one (C2 6.26 vs 6.22 ms: off)
#endif
__device__ unsigned long long rtx_stamps[16];
__device__ __forceinline__ unsigned long long wall() {   // 100 MHz constant clock, same on every XCD
#if RTX_STAMPS
  return __builtin_amdgcn_s_memrealtime();
#else
  return 0;
#endif
}
__device__ __forceinline__ unsigned long long stamp() {
#if RTX_STAMPS
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
#else
  return 0;
#endif
}

// sin and cos of one angle: separate ocml calls (measured 4 % faster on C2 than
// ocml's sincos; both give the same bits).  -DRTX_SEPARATE_SINCOS=0 for sincos.
#ifndef RTX_SEPARATE_SINCOS
#define RTX_SEPARATE_SINCOS 1
#endif
// Transcendentals are real calls by default: inlined into the state machine,
// their 64-bit polynomial coefficients are hoisted to the kernel entry and
// spilled, and every sin/cos/acos then waits on a chain of serialized scratch
// reloads (seen in the gfx950 ISA).  -DRTX_INLINE_MATH=1 inlines them again.
#ifndef RTX_INLINE_MATH
#define RTX_INLINE_MATH 0
#endif
#if RTX_INLINE_MATH
#define RTX_MATH_FN __device__ __forceinline__
#else
#define RTX_MATH_FN __device__ __noinline__
#endif
RTX_MATH_FN double rx_sin(double x) { return sin(x); }
RTX_MATH_FN double rx_cos(double x) { return cos(x); }
RTX_MATH_FN double rx_asin(double x) { return asin(x); }
RTX_MATH_FN double rx_acos(double x) { return acos(x); }
RTX_MATH_FN double rx_pow(double x, double y) { return pow(x, y); }
RTX_MATH_FN void rx_sincos(double x, double* s, double* c) { sincos(x, s, c); }

#if RTX_SEPARATE_SINCOS
#define RTX_SINCOS(x, s, c) (*(s) = rx_sin(x), *(c) = rx_cos(x))
#else
#define RTX_SINCOS(x, s, c) rx_sincos((x), (s), (c))
#endif

// A lane's first raise (low byte) plus GT1_PENDING: rt_reduce's "color greater
// than 1" is raised by the FIFO drain after the whole tree (ray_tracer.rb:39-45),
// so it is held back and applies only if no rt_map of the tree raised (end_tree).
constexpr uint32_t GT1_PENDING = 0x80000000u;
__device__ __forceinline__ void seterr(uint32_t& err, uint32_t code) {
  if (!(err & 0xffu)) err = (err & GT1_PENDING) | code;
}
__device__ __forceinline__ uint32_t end_tree(uint32_t err) {
  const uint32_t code = err & 0xffu;
  return code ? code : ((err & GT1_PENDING) ? (uint32_t)ERR_COLOR_GT1 : 0u);
}

// ----------------------------------------------------------------- spheres
// Exact Sphere#intersect (sphere.rb:60-85); r2 = front.r2, dn = front.normalize.
__device__ __forceinline__ bool sphere_exact(V3 C, double R, V3 o, V3 d, V3 dn, double r2, V3& hit, bool& in) {
  const V3 oc = vsub(C, o);                       // center - ray.position
  const double q = vdot(oc, d);
  const double t = q / r2;
  const double s = vsq(oc);                       // |position - center|^2 (same bits)
  // The reference returns nil when the origin is outside and t < 0 (sphere.rb:80).
  // s > R*R*(1 + 1e-12) proves |o - C|.r > R without the sqrt, so
  // this exit is taken only where the full evaluation below would return nil.
  if (t < 0 && s > R * R * (1.0 + 1e-12)) return false;
  const V3 np = vadd(o, vsc(d, t));
  const double nd = vr(vsub(np, C));
  if (!(nd <= R)) return false;                   // inner?(nearest_point)
  const double h = sqrt(R * R - nd * nd);         // radius**2 - nearest_dis**2
  const V3 vec = vsc(dn, h);
  const bool from_inner = sqrt(s) <= R;           // inner?(ray.position)
  in = !from_inner;
  hit = in ? vsub(np, vec) : vadd(np, vec);
  if (!from_inner && t < 0) return false;
  return true;
}

// ----------------------------------------------------------------- planes
// Plane#intersect (plane.rb:38-51).  p = plane record (PLANE_GEO doubles).
template <typename P>
__device__ __forceinline__ bool plane_hit(P p, V3 o, V3 d, V3& hit) {
  const V3 F = v3(p[3], p[4], p[5]);
  const double den = vdot(F, d);
  if (den == 0) return false;
  const double t = vdot(vsub(v3(p[0], p[1], p[2]), o), F) / den;
  hit = vadd(o, vsc(d, t));
  if (t < 0) return false;
  return true;
}

template <typename P>
__device__ __forceinline__ void plane_uv(P p, V3 pos, double& u, double& v) {
  const V3 a = vsub(pos, v3(p[0], p[1], p[2]));   // plane.rb:81-85
  u = vdot(a, v3(p[6], p[7], p[8])) / p[12];
  v = vdot(a, v3(p[9], p[10], p[11])) / p[13];
}

// Box#intersect (box.rb:79-97): nearest face hit inside its u,v square.
template <typename P>
__device__ __forceinline__ bool box_hit(P b, V3 o, V3 d, V3& hit, int& face) {
  double nearest = __builtin_inf();
  bool found = false;
  for (int i = 0; i < 6; i++) {
    const P p = b + i * PLANE_GEO;
    V3 h;
    if (plane_hit(p, o, d, h)) {
      double u, v;
      plane_uv(p, h, u, v);
      if (-0.5 <= u && u <= 0.5 && -0.5 <= v && v <= 0.5) {
        const double dd = vr(vsub(h, o));
        if (dd < nearest) {
          nearest = dd;
          hit = h;
          face = i;
          found = true;
        }
      }
    }
  }
  return found;
}

// Sphere#cover_area's penumbra (sphere.rb:31-56) once the binary factor is 1.
RTX_SHADE_FN double penumbra(V3 C, double R, V3 T, V3 lt, double radius, uint32_t& err) {
  const double t = vdot(vsub(C, T), lt) / vr2(lt);
  const V3 x1 = vadd(T, vsc(lt, t));
  const double r1 = radius * (vr(vsub(x1, T)) / vr(lt));
  const double d = vr(vsub(x1, C));
  if (d >= r1 + R) return 0.0;
  const double s1 = PI * r1 * r1;
  if (d > fabs(R - r1)) {
    double c1 = (r1 * r1 + d * d - R * R) / (2.0 * r1 * d);
    double c2 = (R * R + d * d - r1 * r1) / (2.0 * R * d);
    if (c1 > 1.0) c1 = 1.0;
    if (c2 > 1.0) c2 = 1.0;
    if (c1 < -1.0 || c2 < -1.0) seterr(err, ERR_DOMAIN);     // Math::DomainError
    const double th1 = rx_acos(c1), th2 = rx_acos(c2);
    const double ds = ((th1 - rx_sin(th1)) * r1 * r1 + (th2 - rx_sin(th2)) * R * R) / 2.0;
    return 1.0 * ds / s1;
  }
  if (r1 > R) return 1.0 * PI * R * R / s1;
  return 1.0;
}

// ----------------------------------------------------------------- the query
// One ordered walk over every object with ray (o, d), for every active lane.
//   EXTEND: World#intersect — nearest hit (strict <, YAML order) -> best/besti.
//   SHADOW: World#lit_area for light L (o = target T, d = L - T) -> total
//           (1 - ordered sum of cover areas; zero covers skipped: exact).
template <bool COUNT, typename SPH>
__device__ __forceinline__ void query(const SceneDev& S, SPH sph, bool ext, V3 o, V3 d,
                                      V3 L, double radius, double& best, int& besti, V3& bhit, bool& bin,
                                      double& total, uint32_t& err, unsigned long long* cnt) {
  const double r = vr(d);
  const double r2 = r * r;                        // front.r2
  // front.normalize is needed only by a sphere that passes the pre-test:
  // computed on first use (same bits wherever it is computed).
#ifndef RTX_LAZY_DN
#define RTX_LAZY_DN 0
#endif
  V3 dn = d;
  bool have_dn = false;
  if (!RTX_LAZY_DN) {
    if (r != 0) dn = v3(d.x / r, d.y / r, d.z / r);
    have_dn = true;
  }
  // float32 pre-test constants (exact culls)
  const float ox = (float)o.x, oy = (float)o.y, oz = (float)o.z;
  const float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
  const float dd = __builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz));
  const float Sx = fabsf(ox) + fabsf(oy) + fabsf(oz) + S.sph_scale;
  const float ms2 = CULL_M * Sx * Sx;
  const float kline = dd * ms2;
  const float qneg = -CULL_M * Sx * sqrtf(dd);
  if (COUNT) {
    if (ext) {
      cnt[C_SPHERE_TESTS] += S.n_sphere;
      cnt[C_PLANE_TESTS] += S.n_plane;
      cnt[C_BOX_TESTS] += S.n_box;
    } else {
      cnt[C_COVER_SPHERE] += S.n_sphere;
      cnt[C_COVER_PLANE] += S.n_plane;
      cnt[C_COVER_BOX] += S.n_box;
    }
  }
  const RTX_CONST Run* runs = cptr(S.runs);
  const RTX_CONST Sphere64* sph64 = cptr(S.sph64);
  const int n_runs = uni(S.n_runs);
  for (int ri = 0; ri < n_runs; ri++) {
    Run run;
    run.type = uni(runs[ri].type);
    run.obj0 = uni(runs[ri].obj0);
    run.count = uni(runs[ri].count);
    run.rec0 = uni(runs[ri].rec0);
    if (run.type == OBJ_SPHERE) {
      // Pre-test 4 spheres at a time (4 LDS reads in flight), then run the
      // exact test, in order, for those this lane cannot rule out.
      for (int k0 = 0; k0 < run.count; k0 += 4) {
        // The record table is padded to a multiple of 4 (rtx_capi.cpp), so
        // the group loads are unconditional; records past the run are masked.
        float4 c[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {                // {cx, cy, cz, R^2}, wave-uniform
          const int b = 4 * (run.rec0 + k0 + u);
          c[u].x = sph[b];
          c[u].y = sph[b + 1];
          c[u].z = sph[b + 2];
          c[u].w = sph[b + 3];
        }
        uint32_t keep = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const float ocx = c[u].x - ox, ocy = c[u].y - oy, ocz = c[u].z - oz;
          const float s = __builtin_fmaf(ocx, ocx, __builtin_fmaf(ocy, ocy, ocz * ocz));
          const float q = __builtin_fmaf(ocx, dx, __builtin_fmaf(ocy, dy, ocz * dz));
          const bool miss_line = __builtin_fmaf(s, dd, -q * q) > __builtin_fmaf(dd, c[u].w, kline);
          const bool behind = q < qneg && s > c[u].w + ms2;
          keep |= (miss_line || behind) ? 0u : (1u << u);
        }
        if (k0 + 4 > run.count) keep &= (1u << (run.count - k0)) - 1u;
#if RTX_STAMPS == 2
        if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) {
          for (int u = 0; u < 4; u++) atomicAdd(&rtx_stamps[6], __ballot(keep >> u & 1) ? 1ull : 0ull);
        }
        atomicAdd(&rtx_stamps[7], (unsigned long long)__builtin_popcount(keep));
#endif
#if RTX_DIAG_NOEXACT
        keep = 0;                                    // diagnostic only: wrong results
#endif
        if (!keep) continue;
#pragma unroll
        for (int u = 0; u < 4; u++) {
          if (!(keep >> u & 1)) continue;
          const int k = k0 + u;
          const RTX_CONST Sphere64& sp = sph64[run.rec0 + k];
          const V3 C = v3(sp.c[0], sp.c[1], sp.c[2]);
          const double sr = sp.r;
          if (!have_dn) {
            if (r != 0) dn = v3(d.x / r, d.y / r, d.z / r);
            have_dn = true;
          }
          V3 hit;
          bool in;
          if (!sphere_exact(C, sr, o, d, dn, r2, hit, in)) continue;
          if (ext) {
            if (COUNT) cnt[C_SPHERE_HITS]++;
            const double dist = vr(vsub(o, hit));    // Ray#distance
            if (dist < best) {
              best = dist;
              besti = run.obj0 + k;
              bhit = hit;                              // kept for shading (same bits as a re-evaluation)
              bin = in;
            }
          } else if (vdot(vsub(hit, L), vsub(o, L)) > 0) {   // cover factor 1
            total -= penumbra(C, sr, o, d, radius, err);
          }
        }
      }
    } else if (run.type == OBJ_PLANE) {
      for (int k = 0; k < run.count; k++) {
        V3 hit;
        if (!plane_hit(cptr(S.planes) + (size_t)(run.rec0 + k) * PLANE_GEO, o, d, hit)) continue;
        if (ext) {
          const double dist = vr(vsub(o, hit));
          if (dist < best) {
            best = dist;
            besti = run.obj0 + k;
            bhit = hit;
            bin = true;
          }
        } else if (vdot(vsub(hit, L), vsub(o, L)) > 0) {
          total -= 1.0;
        }
      }
    } else {
      for (int k = 0; k < run.count; k++) {
        V3 hit;
        int face;
        if (!box_hit(cptr(S.boxes) + (size_t)(run.rec0 + k) * BOX_GEO, o, d, hit, face)) continue;
        if (ext) {
          const double dist = vr(vsub(o, hit));
          if (dist < best) {
            best = dist;
            besti = run.obj0 + k;
          }
        } else if (vdot(vsub(hit, L), vsub(o, L)) > 0) {
          total -= 1.0;
        }
      }
    }
  }
}

// ----------------------------------------------------------------- the query, hierarchical
// The same query answered through the four-wide box hierarchy (rtx_scene.h).
// Every lane traverses on its own (per-lane stack in LDS, nearest child first,
// "while-while": lanes descend through inner nodes together, then process
// their leaves together).  A lane skips a child box when a float32 slab test
// of the box dilated by m*S (the margin of DESIGN.md §2.1) proves that every
// sphere below it
//   * misses the ray's line, or lies wholly behind the origin (nil), or
//   * EXTEND: is farther than the lane's current best hit (loses the strict <
//     of world.rb:48-50 even on a tie), or
//   * SHADOW: lies wholly beyond the light (cover factor 0, sphere.rb:30).
// Order independence makes the result bit-identical to the ordered walk:
//   * EXTEND keeps the lexicographic minimum of (distance, object index) below
//     max_distance, which is exactly what the ordered strict-< scan returns;
//   * SHADOW collects the non-zero covers in a per-lane list sorted by object
//     index and subtracts them in that order (world.rb:64-67).  A lane whose
//     list overflows COVER_K repeats the ordered linear walk.
// Planes and boxes are few: they are walked first (tightening `best`).
//
// Slab-test rounding: each computed slab bound errs by a few float32 ulps of
// (|box coordinate| + |o| + m*S) / |d_axis| <= 1e-6 * S / |d_axis|, far inside
// the dilation m*S / |d_axis| (m = 2e-5), so the computed interval contains
// the exact interval of the undilated box; direction components below
// 1e-20 |d|_1 are replaced by that value (a deviation of < 1e-15 over any
// distance the scene spans) so every reciprocal is finite.
__device__ __forceinline__ bool lex_better(double dist, int obj, double best, int besti) {
  return dist < best || (dist == best && besti >= 0 && obj < besti);
}

template <int BS>
__device__ __forceinline__ void push_cover(int* ci, double* cv, int& n, bool& ovf, int obj, double val) {
  if (n >= COVER_K) {
    ovf = true;
    return;
  }
  int k = n;                                        // insertion sort by object index
  while (k > 0) {
    const int pi = ci[(k - 1) * BS];
    if (pi < obj) break;
    ci[k * BS] = pi;
    cv[k * BS] = cv[(k - 1) * BS];
    k--;
  }
  ci[k * BS] = obj;
  cv[k * BS] = val;
  n++;
}

// Resumable: a lane whose walk is still running when fewer than `postpone`
// lanes of its wave are is postponed (returns false) with its walk in
// ref / sp (+ the LDS stack) / ncov / ovf (+ the LDS cover list) and best /
// besti / bhit / bin, and continues where it stopped at the next call with
// resume = true; meanwhile the wave's other lanes shade and start new
// queries instead of idling.  Every lane visits the same nodes and leaves in
// the same order either way, so the result is unchanged.
template <int BS, bool PP, typename NP, typename LP>
__device__ __forceinline__ bool query_bvh(const SceneDev& S, NP nodes, LP leaf4, int* stk, int* ci, double* cv,
                                          bool ext, V3 o, V3 d, V3 L, double radius, double& best, int& besti,
                                          V3& bhit, bool& bin, double& total, uint32_t& err, int& ref, int& sp,
                                          int& ncov, bool& ovf, bool resume, int postpone) {
  const double r = vr(d);
  const double r2 = r * r;                        // front.r2
  V3 dn = d;
  if (r != 0) dn = v3(d.x / r, d.y / r, d.z / r); // front.normalize (same bits as the walk)
  const float ox = (float)o.x, oy = (float)o.y, oz = (float)o.z;
  const float dx = (float)d.x, dy = (float)d.y, dz = (float)d.z;
  const float dd = __builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz));
  const float Sx = fabsf(ox) + fabsf(oy) + fabsf(oz) + S.sph_scale;
  const float ms2 = CULL_M * Sx * Sx;
  const float mS = CULL_M * Sx;
  const float kline = dd * ms2;
  const float qneg = -CULL_M * Sx * sqrtf(dd);
  // slab set-up: reciprocal direction and the dilated origin terms
  const float l1 = fabsf(dx) + fabsf(dy) + fabsf(dz);
  const float tiny = 1e-20f * l1;
  const float ex = fabsf(dx) < tiny ? copysignf(tiny, dx) : dx;
  const float ey = fabsf(dy) < tiny ? copysignf(tiny, dy) : dy;
  const float ez = fabsf(dz) < tiny ? copysignf(tiny, dz) : dz;
  const float ix = 1.0f / ex, iy = 1.0f / ey, iz = 1.0f / ez;
  const float ax = (ox + mS) * ix, ay = (oy + mS) * iy, az = (oz + mS) * iz;   // lo - mS side
  const float bx = (ox - mS) * ix, by = (oy - mS) * iy, bz = (oz - mS) * iz;   // hi + mS side
  // A non-finite or zero ray makes no cull (comparisons would be unordered).
  const bool fin = __builtin_isfinite(dd) && __builtin_isfinite(Sx) && l1 > 0.0f && __builtin_isfinite(ix) &&
                   __builtin_isfinite(iy) && __builtin_isfinite(iz);
  if (!fin) {
    // no float32 cull is valid for this ray: the ordered linear walk (same result)
    if (!ext) total = 1.0;
    query<false>(S, cptr(S.sph32), ext, o, d, L, radius, best, besti, bhit, bin, total, err, nullptr);
    return true;
  }
  const float rf = (float)r;
  // far bound on the ray parameter: EXTEND the current best hit, SHADOW the light
  float thi = ext ? (float)(best / r * (1.0 + 1e-6)) : 1.0f + 1e-5f + mS / rf;
  if (!resume) {
    ncov = 0;
    ovf = false;
    ref = S.bvh_root;
    sp = 0;
  }

  // planes and boxes first, in run order (their order does not matter either)
  const RTX_CONST Run* runs = cptr(S.runs);
  const int n_runs = resume ? 0 : uni(S.n_runs);
  for (int ri = 0; ri < n_runs; ri++) {
    const int type = uni(runs[ri].type);
    if (type == OBJ_SPHERE) continue;
    const int obj0 = uni(runs[ri].obj0), count = uni(runs[ri].count), rec0 = uni(runs[ri].rec0);
    for (int k = 0; k < count; k++) {
      V3 hit;
      bool h;
      if (type == OBJ_PLANE) {
        h = plane_hit(cptr(S.planes) + (size_t)(rec0 + k) * PLANE_GEO, o, d, hit);
      } else {
        int face;
        h = box_hit(cptr(S.boxes) + (size_t)(rec0 + k) * BOX_GEO, o, d, hit, face);
      }
      if (!h) continue;
      if (ext) {
        const double dist = vr(vsub(o, hit));
        if (lex_better(dist, obj0 + k, best, besti)) {
          best = dist;
          besti = obj0 + k;
          bhit = hit;
          bin = true;
          thi = (float)(best / r * (1.0 + 1e-6));
        }
      } else if (vdot(vsub(hit, L), vsub(o, L)) > 0) {
        push_cover<BS>(ci, cv, ncov, ovf, obj0 + k, 1.0);
      }
    }
  }

  while (ref != BVH_NONE) {
    // ---- inner nodes: slab-test the four child boxes, descend into the nearest
    while (ref >= 0 && ref != BVH_NONE) {
      float key[4];
      int ch[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        ch[k] = nodes[ref].child[k];
        const float t0x = __builtin_fmaf(nodes[ref].lo[0][k], ix, -ax);
        const float t1x = __builtin_fmaf(nodes[ref].hi[0][k], ix, -bx);
        const float t0y = __builtin_fmaf(nodes[ref].lo[1][k], iy, -ay);
        const float t1y = __builtin_fmaf(nodes[ref].hi[1][k], iy, -by);
        const float t0z = __builtin_fmaf(nodes[ref].lo[2][k], iz, -az);
        const float t1z = __builtin_fmaf(nodes[ref].hi[2][k], iz, -bz);
        const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
        const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
        // empty slots hold a box at (3e38, 3e38, 3e38): never wanted by a finite ray
        key[k] = (tn <= tf && tf >= 0.0f && tn <= thi) ? tn : __builtin_inff();
      }
#define RTX_CS(a, b)         \
  if (key[b] < key[a]) {     \
    const float tk = key[a]; \
    key[a] = key[b];         \
    key[b] = tk;             \
    const int tc = ch[a];    \
    ch[a] = ch[b];           \
    ch[b] = tc;              \
  }
      RTX_CS(0, 1) RTX_CS(2, 3) RTX_CS(0, 2) RTX_CS(1, 3) RTX_CS(1, 2)
#undef RTX_CS
#pragma unroll
      for (int k = 3; k >= 1; k--)
        if (key[k] < __builtin_inff()) stk[(sp++) * BS] = ch[k];
      if (key[0] < __builtin_inff()) ref = ch[0];
      else ref = sp > 0 ? stk[(--sp) * BS] : BVH_NONE;
    }
    if (ref == BVH_NONE) break;
    // ---- leaf: pre-test its spheres, exact test for those not ruled out
    {
      const int v = ~ref;
      const int slot0 = (v >> 2) * BVH_LEAF;
      const int cnt = (v & 3) + 1;
      float4 c[4];
#pragma unroll
      for (int u = 0; u < 4; u++) c[u] = leaf4[slot0 + u];
      uint32_t keep = 0;
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const float ocx = c[u].x - ox, ocy = c[u].y - oy, ocz = c[u].z - oz;
        const float s = __builtin_fmaf(ocx, ocx, __builtin_fmaf(ocy, ocy, ocz * ocz));
        const float q = __builtin_fmaf(ocx, dx, __builtin_fmaf(ocy, dy, ocz * dz));
        const bool miss_line = __builtin_fmaf(s, dd, -q * q) > __builtin_fmaf(dd, c[u].w, kline);
        const bool behind = q < qneg && s > c[u].w + ms2;
        keep |= (miss_line || behind) ? 0u : (1u << u);
      }
      keep &= (1u << cnt) - 1u;
      while (keep) {
        const int u = __builtin_ctz(keep);
        keep &= keep - 1;
        const Sphere64 sp64 = S.bvh_sph64[slot0 + u];
        const V3 C = v3(sp64.c[0], sp64.c[1], sp64.c[2]);
        V3 hit;
        bool in;
        if (!sphere_exact(C, sp64.r, o, d, dn, r2, hit, in)) continue;
        const int obj = S.bvh_obj[slot0 + u];
        if (ext) {
          const double dist = vr(vsub(o, hit));      // Ray#distance
          if (lex_better(dist, obj, best, besti)) {
            best = dist;
            besti = obj;
            bhit = hit;
            bin = in;
            thi = (float)(best / r * (1.0 + 1e-6));
          }
        } else if (vdot(vsub(hit, L), vsub(o, L)) > 0) {   // cover factor 1
          const double cov = penumbra(C, sp64.r, o, d, radius, err);
          if (cov != 0.0) push_cover<BS>(ci, cv, ncov, ovf, obj, cov);
        }
      }
    }
    ref = sp > 0 ? stk[(--sp) * BS] : BVH_NONE;
    if (PP && __popcll(__ballot(ref != BVH_NONE)) < postpone && ref != BVH_NONE) return false;
  }
  if (!ext) {
    total = 1.0;
    if (ovf) {
      // more than COVER_K non-zero covers: the ordered linear walk (rare)
      query<false>(S, cptr(S.sph32), false, o, d, L, radius, best, besti, bhit, bin, total, err, nullptr);
    } else {
      for (int k = 0; k < ncov; k++) total -= cv[k * BS];
    }
  }
  return true;
}

// ----------------------------------------------------------------- shading
// WorldObject#get_reflection_by_ray_and_n (world_object.rb:121-125).
// nn = n.normalize, c = ray.front.cos(-n) (== ray.front.cos(n): |cos| of a
// negated vector has the same bits), both computed once per hit.
__device__ __forceinline__ Ray reflection(const Ray& ray, V3 nn, double c, V3 hit, V3 delta, uint32_t& err) {
  Ray r;
  r.d = vnorm(vadd(vsc(nn, 2.0 * c * vr(ray.d)), ray.d), err);
  r.o = vadd(hit, delta);
  return r;
}

// WorldObject#get_refraction_by_ray_and_n (world_object.rb:127-137).
__device__ __forceinline__ bool refraction(const Ray& ray, V3 nn, double c, V3 hit, V3 refl, double rate,
                                           Ray& out, uint32_t& err) {
  const double sin_i = sqrt(1.0 - c * c);        // 1 - cos**2
  const double sin_r = sin_i / rate;
  if (sin_r >= 1) return false;                  // total internal reflection
  const double r = rx_asin(sin_r);
  out.d = vadd(vsc(nn, -rx_cos(r)), vsc(vnorm(vadd(refl, ray.d), err), sin_r));
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

// Geometry of the winning hit: position, delta, normal n and the :in flag of
// intersect_parameters (sphere.rb:60-101, plane.rb:38-67, box.rb:100-105).
// Re-evaluated with the same operations as in the walk, hence the same bits.
// Geometry of the winning hit: delta, normal n and the :in flag of
// intersect_parameters (sphere.rb:60-101, plane.rb:38-67, box.rb:100-105).
// Spheres and planes: `hit` and `in` are the walk's own evaluation of the
// winner (kept when it became the nearest; same bits a re-evaluation gives).
// Boxes re-evaluate to find the face.
RTX_SHADE_FN void hit_info(const SceneDev& S, int obj, const Ray& ray, V3& hit, V3& delta, V3& n, bool& in) {
  const Material& m = S.mat[obj];
  if (m.type == OBJ_SPHERE) {
    const Sphere64 sp = S.sph64[m.rec];
    const V3 C = v3p(sp.c);
    delta = vsc(vsc(vsub(hit, C), EPS), in ? 1.0 : -1.0);
    n = in ? vsub(hit, C) : vsub(C, hit);
    return;
  }
  in = true;
  const double* plane;
  if (m.type == OBJ_PLANE) {
    plane = S.planes + (size_t)m.rec * PLANE_GEO;
  } else {
    int face = 0;
    box_hit(S.boxes + (size_t)m.rec * BOX_GEO, ray.o, ray.d, hit, face);
    plane = S.boxes + (size_t)m.rec * BOX_GEO + face * PLANE_GEO;
  }
  const V3 F = v3(plane[3], plane[4], plane[5]);
  const double fd = vdot(F, ray.d);
  const double nfd = -fd;
  delta = vsc(vsc(F, EPS), nfd > 0 ? 1.0 : (nfd < 0 ? -1.0 : 0.0));   // (-f.d <=> 0).to_f
  n = fd > 0 ? vneg(F) : F;
}

// Per-lane LIFO of pending rays (RayTracer#trace_sync's Array, ray_tracer.rb:21-30).
// The bottom `slots` entries live in LDS (11 eight-byte words per entry, laid
// out word-major across the workgroup's lanes so a wave's accesses are
// conflict-free); deeper entries go to the lane's own contiguous region of a
// global buffer (12 doubles per entry: one push or pop touches two 64-B lines,
// where a private-array entry, swizzled across the wave, touched 21).
constexpr int ITEM_WORDS = 11;
constexpr int GITEM_DOUBLES = 12;
template <int MAXS>
struct Stack {
  int n;
  double* lds;     // this lane's word 0 of entry 0; word w of entry e at lds[(e * ITEM_WORDS + w) * bs]
  double* g;       // this lane's global region: entry e at g[e * GITEM_DOUBLES]
  int bs;
  int slots;

  __device__ __forceinline__ void push(const Item& it) {
    if (n < slots) {
      double* q = lds + (size_t)n * ITEM_WORDS * bs;
      q[0] = it.ray.o.x;
      q[bs] = it.ray.o.y;
      q[2 * bs] = it.ray.o.z;
      q[3 * bs] = it.ray.d.x;
      q[4 * bs] = it.ray.d.y;
      q[5 * bs] = it.ray.d.z;
      q[6 * bs] = it.att.x;
      q[7 * bs] = it.att.y;
      q[8 * bs] = it.att.z;
      q[9 * bs] = __builtin_bit_cast(double, it.path);
      q[10 * bs] = __builtin_bit_cast(double, (int64_t)it.depth);
    } else {
      double2* q = reinterpret_cast<double2*>(g + (size_t)(n - slots) * GITEM_DOUBLES);
      q[0] = make_double2(it.ray.o.x, it.ray.o.y);
      q[1] = make_double2(it.ray.o.z, it.ray.d.x);
      q[2] = make_double2(it.ray.d.y, it.ray.d.z);
      q[3] = make_double2(it.att.x, it.att.y);
      q[4] = make_double2(it.att.z, __builtin_bit_cast(double, it.path));
      q[5] = make_double2(__builtin_bit_cast(double, (int64_t)it.depth), 0.0);
    }
    n++;
  }
  __device__ __forceinline__ void pop(Item& it) {
    n--;
    if (n < slots) {
      const double* q = lds + (size_t)n * ITEM_WORDS * bs;
      it.ray.o = v3(q[0], q[bs], q[2 * bs]);
      it.ray.d = v3(q[3 * bs], q[4 * bs], q[5 * bs]);
      it.att = v3(q[6 * bs], q[7 * bs], q[8 * bs]);
      it.path = __builtin_bit_cast(uint64_t, q[9 * bs]);
      it.depth = (int32_t)__builtin_bit_cast(int64_t, q[10 * bs]);
    } else {
      const double2* q = reinterpret_cast<const double2*>(g + (size_t)(n - slots) * GITEM_DOUBLES);
      const double2 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5];
      it.ray.o = v3(a.x, a.y, b.x);
      it.ray.d = v3(b.y, c.x, c.y);
      it.att = v3(d.x, d.y, e.x);
      it.path = __builtin_bit_cast(uint64_t, e.y);
      it.depth = (int32_t)__builtin_bit_cast(int64_t, f.x);
    }
  }
};

__device__ __forceinline__ void add_leaf(V3& sum, V3 c, uint32_t& err) {   // ray_tracer.rb:292-298
  sum = vadd(sum, c);
  if (!(sum.x <= 1 && sum.y <= 1 && sum.z <= 1)) err |= GT1_PENDING;
}

// Children are generated in the reference's push order; the most recent live
// one is held in `pend` (it is what Array#pop returns next) and only older
// siblings are written to the stack.  A child rt_map would discard on pop
// (ray_tracer.rb:52) is dropped here: no leaf, no RNG draw, no effect.
template <int MAXS>
__device__ __forceinline__ void emit(Stack<MAXS>& st, Item& pend, bool& has, uint32_t& err, const Ray& r,
                                     V3 att, uint64_t path, int depth) {
  if (depth <= 0 || vr(att) < 0.0001) return;
  if (has) {
    if (st.n < MAXS) st.push(pend);
    else seterr(err, ERR_DOMAIN);                // cannot happen: stack sized on the host
  }
  pend.ray = r;
  pend.att = att;
  pend.path = path;
  pend.depth = depth;
  has = true;
}

// The rest of rt_map once every light's lit area is known (ray_tracer.rb:80-158):
// reflection / refraction children, then path-tracing children (no lit light)
// or the local-lighting leaf.  Returns true with the next ray in `cur`.
template <int MAXS>
RTX_SHADE_FN bool shade_finish(const SceneDev& S, const CameraDev& cam, uint64_t seed, int x, int y,
                                          int sample, int obj, bool in, V3 hit, V3 delta, V3 n, V3 nn, V3 lc,
                                          int nl,
                                          Item& cur, Stack<MAXS>& st, V3& sum, uint32_t& err) {
  const Material& m = S.mat[obj];
  Item pend;
  bool has = false;
  const uint64_t R = (uint64_t)cam.pt + 3;
  const double c = vcos(cur.ray.d, n, err);
  const Ray refl = reflection(cur.ray, nn, c, hit, delta, err);
  emit<MAXS>(st, pend, has, err, refl, vmul(cur.att, v3p(m.refl_att)), cur.path * R + 1, cur.depth - 1);
  Ray refr;
  bool has_refr = false;
  if (m.type == OBJ_SPHERE)                                  // sphere.rb:92-94: rate inverted leaving
    has_refr = refraction(cur.ray, nn, c, hit, refl.d, in ? m.rr : 1.0 / m.rr, refr, err);
  else if (m.has_rr)                                         // plane.rb:57-61: same rate both ways
    has_refr = refraction(cur.ray, nn, c, hit, refl.d, m.rr, refr, err);
  if (has_refr)
    emit<MAXS>(st, pend, has, err, refr, vmul(cur.att, v3p(m.refr_att)), cur.path * R + 2, cur.depth - 1);
  if (nl == 0) {
    // WorldObject#path_tracing (world_object.rb:76-90) from hit + delta
    const int pt = cam.pt;
    const V3 att = vmul(cur.att, vdiv(v3p(m.diffuse), (double)pt));
    const V3 front = nn;
    const V3 left = vnorm(vertical_vector(n, err), err);
    const V3 up = vcross(front, left);
    Ray r;
    r.o = vadd(hit, delta);
    for (int k = 0; k < pt; k++) {
      const double theta = rand01(seed, x, y, sample, cur.path, 2 * k) * PI / 2.0;
      const double phi = rand01(seed, x, y, sample, cur.path, 2 * k + 1) * PI * 2.0;
      double sth, cth, sph, cph;
      RTX_SINCOS(theta, &sth, &cth);
      RTX_SINCOS(phi, &sph, &cph);
      r.d = vadd(vsc(front, sth), vsc(vadd(vsc(left, cph), vsc(up, sph)), cth));
      emit<MAXS>(st, pend, has, err, r, att, cur.path * R + 3 + (uint64_t)k, cur.depth - 1);
    }
  } else {
    lc = vdiv(lc, (double)nl);
    V3 color;
    if (m.type == OBJ_BOX) {
      color = vadd(vmul(lc, v3p(m.diffuse)), v3p(m.ambient));
    } else {
      V3 filter = v3(1.0, 1.0, 1.0);
      if (m.tex >= 0) {
        if (m.type == OBJ_SPHERE) {                   // Sphere#get_uv (sphere.rb:111-120)
          const Sphere64 sp = S.sph64[m.rec];
          const V3 vec = vsub(hit, v3p(sp.c));
          const double x0 = vdot(vec, v3p(m.gw_n)) / sp.r;
          const double y0 = vdot(vec, v3p(m.east_n)) / sp.r;
          const double z0 = vdot(vec, v3p(m.north_n)) / sp.r;
          const double mm2 = x0 * x0 + y0 * y0 + z0 * z0 + 2.0 * x0 + 1.0;
          if (mm2 < 0) seterr(err, ERR_DOMAIN);
          const double mm = sqrt(mm2);
          filter = vmul(texcolor(S, m.tex, m.hs, m.vs, m.u_off, m.v_off, (y0 / mm + 1.0) / 2.0,
                                 (-z0 / mm + 1.0) / 2.0, err), filter);
        } else {
          double u, v;
          plane_uv(S.planes + (size_t)m.rec * PLANE_GEO, hit, u, v);
          filter = vmul(texcolor(S, m.tex, m.hs, m.vs, 0.0, 0.0, u, v, err), filter);
        }
      }
      color = vadd(vmul(vmul(lc, v3p(m.diffuse)), filter), v3p(m.ambient));
    }
    add_leaf(sum, vmul(cur.att, color), err);
  }
  if (has) cur = pend;
  return has;
}

// Camera#lens_func (camera.rb:129-151).  Everything but the aperture point is
// independent of the sample: the focal-plane target of pixel (x, y) is
// computed once per pixel (lens_target), the sample's ray per draw (lens_ray).
__device__ __forceinline__ V3 lens_target(const CameraDev& c, int x, int y) {
  const V3 rp = vadd(vadd(v3p(c.retina_center), vsc(v3p(c.left), 2.0 * ((double)x / c.width - 0.5) * c.retina_width)),
                     vsc(v3p(c.up_n), 2.0 * ((double)y / c.height - 0.5) * c.retina_height));
  const V3 rd = vsub(v3p(c.pos), rp);                           // Ray(position - retina, retina)
  const double t = vdot(vsub(v3p(c.pofp), rp), v3p(c.front)) / vdot(v3p(c.front), rd);
  return vadd(rp, vsc(rd, t));                                  // intersect_plane (:123-127)
}

__device__ __forceinline__ Ray lens_ray(const CameraDev& c, V3 target, int x, int y, int j, uint64_t seed) {
  const double theta = rand01(seed, x, y, j, 0, 0);
  double st, ct;
  RTX_SINCOS(theta, &st, &ct);
  const V3 rv = vsc(vadd(vsc(v3p(c.left_n), ct), vsc(v3p(c.up_n), st)), c.aperture_radius);
  Ray r;
  r.o = vadd(v3p(c.pos), rv);
  r.d = vsub(target, r.o);
  return r;
}

// World#high_lights (world.rb:83-98) for `ray`: every fired light's leaf goes
// to `leaf(V3)` in light order.  Returns true if any light fired (the ray then
// stops, ray_tracer.rb:77).  The `&& lit_area(...)` is always truthy in Ruby and
// is not evaluated.
template <typename Leaf>
__device__ __forceinline__ bool highlight_leaves(const SceneDev& S, const Item& it, Leaf&& leaf, uint32_t& err) {
  uint32_t fired = 0;
  int nfired = 0;
  const RTX_CONST LightDev* lights = cptr(S.light);
  for (int l = 0; l < S.n_light; l++) {
    const RTX_CONST LightDev& L = lights[l];
    const V3 a = vsub(v3(L.pos[0], L.pos[1], L.pos[2]), it.ray.o);
    const double dot = vdot(it.ray.d, a);
    const double r1 = vsq(it.ray.d), r2 = vsq(a);
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
      fire = rx_acos(c) < L.hl_angle_rad;
    }
    if (fire) {
      fired |= 1u << l;
      nfired++;
    }
  }
  if (!nfired) return false;
  for (int l = 0; l < S.n_light; l++) {
    if (!(fired >> l & 1)) continue;
    const RTX_CONST LightDev& L = lights[l];
    leaf(vdiv(vmul(it.att, vsc(v3(L.color[0], L.color[1], L.color[2]), L.hl_rate)), (double)nfired));
  }
  return true;
}

// The same into a running sum.  REDUCE: leaves go through rt_reduce
// (trace_sync); path_trace adds them with a plain `ret +=` (ray_tracer.rb:210),
// no "color greater than 1" check.
template <bool REDUCE = true>
__device__ __forceinline__ bool highlights(const SceneDev& S, const Item& it, V3& sum, uint32_t& err) {
  return highlight_leaves(S, it, [&](V3 c) {
    if (REDUCE) add_leaf(sum, c, err);
    else sum = vadd(sum, c);
  }, err);
}

// `key` orders the raise sites as the reference meets them: x * height + y for
// pixels (render_sync runs x in the outer loop, y in the inner one,
// camera.rb:102-103), the ray index for rtx_trace.
__device__ __forceinline__ void record_error(ErrState* e, uint32_t code, unsigned long long key) {
  atomicOr(&e->flags, 1u << code);
  atomicMin(&e->first[code], key);
}
__device__ __forceinline__ unsigned long long px_key(int x, int y, int H) {
  return (unsigned long long)x * (unsigned long long)H + (unsigned long long)y;
}

__device__ __forceinline__ int row_to_y(const KParams& p, int row) {
  if (p.tile_rows == 0) return p.y0 + row;
  const int k = row / p.tile_rows;
  return (k * p.nranks + p.rank) * p.tile_rows + (row - k * p.tile_rows);
}

// Level-0 item k of a bounce-level batch (KParams lv_*): pass 0, the pre
// samples of the batch's tiles in (tile, pixel in Morton order, sample) order;
// pass 1, the extra samples of the batch's extra-list entries.
struct ItemPos {
  int px, row, sample;
  bool valid;                      // inside the region (8x8 tiles are padded)
};
__device__ __forceinline__ ItemPos decode_item(const KParams& p, int k) {
  ItemPos ip;
  if (p.lv_pass == 0) {
    const int tiles_x = (p.nx + 7) >> 3;
    const int per = 64 * p.pre;
    const int slot = k / per, r = k - slot * per;
    const int tile = p.lv_t0 + slot;
    const int l = r / p.pre;
    ip.sample = r - l * p.pre;
    ip.px = (tile % tiles_x) * 8 + ((l & 1) | ((l >> 1) & 2) | ((l >> 2) & 4));
    ip.row = (tile / tiles_x) * 8 + (((l >> 1) & 1) | ((l >> 2) & 2) | ((l >> 3) & 4));
    ip.valid = ip.px < p.nx && ip.row < p.nrows && row_to_y(p, ip.row) < p.cam->height;
  } else {
    const int n_extra = p.max_samples - p.pre;
    const int e = k / n_extra;
    const int idx = p.extra_list[p.lv_e0 + e];
    ip.sample = p.pre + (k - e * n_extra);
    ip.px = idx % p.nx;
    ip.row = idx / p.nx;
    ip.valid = true;
  }
  return ip;
}

// SRC_PIXELS: work item = one of Camera#render_at's pre_sample_times samples
// of one pixel (a wave's first fetch covers an 8x8 tile for one sample index);
// the sample's colour and first raise go to p.samples, and k_finalize does the
// mean / variance / extra-sample decision.  SRC_EXTRA: the extra samples of the
// pixels k_finalize listed.  SRC_RAYS: one lane per explicit ray running
// RayTracer#trace_sync (rtx_trace).  SPH: where the sphere walk reads its
// records (SphMode, rtx_launch.h).  BS: threads per workgroup.
template <bool COUNT, int MAXS, int WPS, int SPH, int SRC, int BS, bool PP>
__global__ __launch_bounds__(BS, WPS) void k_render(KParams p) {
  const double* __restrict__ rays = p.rays;
  const int32_t* __restrict__ keys = p.keys;
  const int nrays = p.nrays;
  static_assert(!COUNT || SPH == SPH_LIN_LDS || SPH == SPH_LIN_SCALAR, "counting launches walk linearly");
  const SceneDev& S = p.scene;                // kernel argument: scalar loads
  const CameraDev& cam = *p.cam;
  if (SRC == SRC_LIST && p.lv_ctl->redo_n == 0) return;   // nothing to re-render (the usual case)
  // Dynamic LDS: the sphere records of the walk (SPH_LIN_LDS: float32 pre-test
  // records; SPH_BVH_LDS: hierarchy nodes at 0, leaf records at lds_leaf),
  // then (BVH modes) the per-wave traversal stacks and per-lane cover lists.
  extern __shared__ float4 lds_sph[];
  char* lds = reinterpret_cast<char*>(lds_sph);
  if (SPH == SPH_LIN_LDS) {
    for (int i = threadIdx.x; i < S.n_sphere + 4; i += BS)
      lds_sph[i] = reinterpret_cast<const float4*>(S.sph32)[i];
    __syncthreads();
  } else if (SPH == SPH_BVH_LDS) {
    const int nn = S.n_nodes * (int)(sizeof(Bvh4Node) / 16);
    for (int i = threadIdx.x; i < nn; i += BS) lds_sph[i] = reinterpret_cast<const float4*>(S.bvh)[i];
    float4* leaf = reinterpret_cast<float4*>(lds + p.lds_leaf);
    for (int i = threadIdx.x; i < S.n_slots; i += BS) leaf[i] = reinterpret_cast<const float4*>(S.bvh_sph32)[i];
    __syncthreads();
  }
  const float* sph_lds = reinterpret_cast<const float*>(lds_sph);
  const RTX_CONST float* sph_k = cptr(S.sph32);
  int* stk = reinterpret_cast<int*>(lds + p.lds_stack) + threadIdx.x;
  int* cov_i = reinterpret_cast<int*>(lds + p.lds_cov) + threadIdx.x;
  double* cov_v = reinterpret_cast<double*>(lds + p.lds_cov + COVER_K * BS * 4) + threadIdx.x;

  // Persistent lanes: every lane takes work items (SRC_PIXELS: (pixel, sample)
  // in 8x8-tile order; SRC_EXTRA: (listed pixel, extra sample); SRC_RAYS: rays)
  // from one counter per launch and takes the next one as soon as its current
  // item is finished, so no lane idles until the pool is empty.  Items are one
  // ray tree each: the longest item, which bounds the launch's tail, is one
  // sample, not a whole pixel.  A wave's lanes that need work are served by one
  // atomic (ballot + prefix count).
  const int tiles_x = (p.nx + 7) >> 3;
  const int pre = p.pre, n_extra = p.max_samples - p.pre;
  const int ms = p.max_samples > p.pre ? p.max_samples : p.pre;   // sample records per pixel
  const int nwork = SRC == SRC_PIXELS ? tiles_x * ((p.nrows + 7) >> 3) * 64 * pre
                    : SRC == SRC_EXTRA ? *p.extra_count * n_extra
                    : SRC == SRC_LIST ? (int)p.lv_ctl->redo_n : nrays;
  int x = 0, y = 0, row = 0, px_ = 0, item_ = 0;
  V3 tgt = v3(0.0, 0.0, 0.0);

  unsigned long long cnt[C_N];
  if (COUNT)
    for (int k = 0; k < C_N; k++) cnt[k] = 0;

  Stack<MAXS> st;
  st.n = 0;
  st.bs = BS;
  st.slots = p.stk_slots;
  st.lds = reinterpret_cast<double*>(lds + p.lds_items) + threadIdx.x;
  st.g = p.stk_glb + ((size_t)blockIdx.x * BS + threadIdx.x) * (MAXS * GITEM_DOUBLES);
  uint32_t err = 0;
  V3 sum = v3(0.0, 0.0, 0.0), avg = sum;
  bool started = false;              // the current item's tree has begun
  int wbase = 0, wlim = 0;           // the wave's claimed, not yet assigned items (wave-uniform)
  const int nwaves = (int)gridDim.x * (BS / 64);
  int sample = 0;                    // camera sample of the item = RNG key of its tree
  Item cur;
  bool have = false;                 // `cur` holds a ray not yet processed
  int mode = M_FETCH;
  // shading state of the ray being shaded
  int besti = -1, li = 0, nl = 0;
  bool hin = true;
  double best = 0.0, total = 0.0;
  V3 hit = avg, delta = avg, n = avg, nn = avg, lc = avg;
  V3 qo = avg, qd = avg, qL = avg;
  double qrad = 0.0;
  int q_ref = BVH_NONE, q_sp = 0, q_ncov = 0;   // a postponed hierarchy walk (query_bvh)
  bool q_ovf = false, q_resume = false;

  unsigned long long tA = 0, tB = 0, tC = 0, tD = 0, tR = 0, iters = 0, t0 = 0, t1;
  const unsigned long long w_start = wall();
  unsigned long long w_dry = 0;                // when this lane found the work pool empty
  unsigned long long w_item = 0, w_maxitem = 0; // start of the current item, longest item
  while (true) {
    if (RTX_STAMPS) t0 = stamp();
    // ---- A: find this lane's next query (divergent, short)
    while (true) {
      while (mode == M_NEED) {
        if (have) {
          have = false;
        } else if (st.n > 0) {
          st.pop(cur);
        } else {
          // the current tree is complete: the item's result
          if (started) {
            err = end_tree(err);
            if (SRC == SRC_RAYS) {
              p.out[3 * row] = sum.x;
              p.out[3 * row + 1] = sum.y;
              p.out[3 * row + 2] = sum.z;
              if (err) record_error(p.err, err, (unsigned long long)row);
            } else {                            // one camera sample: colour + first raise
              double2* q = SRC == SRC_LIST
                               ? reinterpret_cast<double2*>(p.lv_redo_smp + (size_t)item_ * 4)
                               : reinterpret_cast<double2*>(p.samples + ((size_t)row * p.nx + px_) * ms * 4 +
                                                            (size_t)sample * 4);
              q[0] = make_double2(sum.x, sum.y);
              q[1] = make_double2(sum.z, __builtin_bit_cast(double, (uint64_t)err));
            }
            mode = M_FETCH;
            break;
          }
          started = true;
          sum = v3(0.0, 0.0, 0.0);
          if (SRC != SRC_RAYS) {
            cur.ray = lens_ray(cam, tgt, x, y, sample, p.seed);
            if (COUNT) cnt[C_PRIMARY]++;
          } else {
            cur.ray.d = v3p(rays + 6 * row);
            cur.ray.o = v3p(rays + 6 * row + 3);
            sample = keys[3 * row + 2];
          }
          cur.att = v3(1.0, 1.0, 1.0);
          cur.path = 1;
          cur.depth = cam.depth;
        }
        // rt_map prologue (ray_tracer.rb:52-75)
        if (cur.depth <= 0 || vr(cur.att) < 0.0001) continue;
        if (COUNT) {
          cnt[C_RAYS]++;
          cnt[C_HIGHLIGHT_TESTS] += S.n_light;
        }
        if (highlights(S, cur, sum, err)) continue;
        mode = M_EXTEND;
        qo = cur.ray.o;
        qd = cur.ray.d;
        best = S.max_distance;
        besti = -1;
      }
      // ---- refill: lanes whose item is finished take the next ones, first
      // from the wave's claimed range [wbase, wlim), then from a new claim
      const uint64_t f = __ballot(mode == M_FETCH);
      if (!f) break;
      const int need = __popcll(f), left = wlim - wbase;
      int base = wbase;                        // items of rank >= left come from `fresh`
      int fresh = 0;
      if (left < need) {
        // guided self-scheduling: besides what the lanes need now, claim up to
        // 1/(RTX_CLAIM_DIV x waves) of what the last claim saw remaining (at
        // most RTX_CLAIM_MAX), so a
        // wave pays the atomic's round trip once per several refills and the
        // items held privately stay a small share of the pool at every point
        int extra = (nwork - wlim) / (RTX_CLAIM_DIV * nwaves);
        extra = extra < 0 ? 0 : (extra > RTX_CLAIM_MAX ? RTX_CLAIM_MAX : extra);
        int claim = need - left + extra;
        if (RTX_CLAIM_ALIGN > 1) claim = (claim + RTX_CLAIM_ALIGN - 1) / RTX_CLAIM_ALIGN * RTX_CLAIM_ALIGN;
        const int src = __builtin_ctzll(f);
        const unsigned long long t_r = RTX_STAMPS == 1 ? stamp() : 0;
        if ((int)__lane_id() == src) fresh = atomicAdd(p.work, claim);
        fresh = __builtin_amdgcn_readlane(fresh, src);
        if (RTX_STAMPS == 1) tR += stamp() - t_r;
        wbase = fresh + (need - left);
        wlim = fresh + claim;
      } else {
        wbase += need;
      }
      if (mode == M_FETCH) {
        const int r = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(f >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)f, 0u));
        const int k = r < left ? base + r : fresh + (r - left);
        if (k >= nwork) {
          mode = M_DONE;
          if (RTX_STAMPS) w_dry = wall();
        } else if (SRC != SRC_RAYS) {
          if (RTX_STAMPS) {
            const unsigned long long w = wall();
            if (w_item && w - w_item > w_maxitem) w_maxitem = w - w_item;
            w_item = w;
          }
          if (SRC == SRC_PIXELS) {
            const int slot = k / (64 * pre), r = k - slot * (64 * pre);
            const int tile = p.tile_order ? p.tile_order[slot] : slot;   // expensive tiles first
#if RTX_ITEM_ORDER == 1
            // (pixel in Morton order, sample): a wave's 64 items are the
            // pre_sample_times samples of a compact block of pixels
            const int l = r / pre;
            sample = r - l * pre;
            px_ = (tile % tiles_x) * 8 + ((l & 1) | ((l >> 1) & 2) | ((l >> 2) & 4));
            row = (tile / tiles_x) * 8 + (((l >> 1) & 1) | ((l >> 2) & 2) | ((l >> 3) & 4));
#else
            const int l = r & 63;
            sample = r >> 6;
            px_ = (tile % tiles_x) * 8 + (l & 7);
            row = (tile / tiles_x) * 8 + (l >> 3);
#endif
          } else if (SRC == SRC_LIST) {       // a bounce-level item re-rendered here
            item_ = k;
            const ItemPos ip = decode_item(p, p.lv_redo_list[k]);
            sample = ip.sample;
            px_ = ip.px;
            row = ip.row;
          } else {
            const int e = k / n_extra;
            const int idx = p.extra_list[e];
            sample = pre + (k - e * n_extra);
            px_ = idx % p.nx;
            row = idx / p.nx;
          }
          if (px_ < p.nx && row < p.nrows) {
            y = row_to_y(p, row);
            if (y < cam.height) {
              x = p.x0 + px_;
              tgt = lens_target(cam, x, y);
              started = false;
              err = 0;
              mode = M_NEED;
            }
          }
        } else {
          row = k;
          x = keys[3 * row];
          y = keys[3 * row + 1];
          started = false;
          err = 0;
          mode = M_NEED;
        }
      }
    }
    if (RTX_STAMPS) {
      t1 = stamp();
      tA += t1 - t0;
      t0 = t1;
      iters++;
    }
    if (mode == M_DONE) break;

    // ---- B: the object walk, shared by EXTEND and SHADOW lanes
    if (SPH == SPH_LIN_LDS)
      query<COUNT>(S, sph_lds, mode == M_EXTEND, qo, qd, qL, qrad, best, besti, hit, hin, total, err, cnt);
    else if (SPH == SPH_LIN_SCALAR)
      query<COUNT>(S, sph_k, mode == M_EXTEND, qo, qd, qL, qrad, best, besti, hit, hin, total, err, cnt);
    else if (SPH == SPH_BVH_LDS)
      q_resume = !query_bvh<BS, PP>(S, reinterpret_cast<const Bvh4Node*>(lds),
                                reinterpret_cast<const float4*>(lds + p.lds_leaf), stk, cov_i, cov_v,
                                mode == M_EXTEND, qo, qd, qL, qrad, best, besti, hit, hin, total, err, q_ref, q_sp,
                                q_ncov, q_ovf, q_resume, p.postpone);
    else
      q_resume = !query_bvh<BS, PP>(S, S.bvh, reinterpret_cast<const float4*>(S.bvh_sph32), stk, cov_i, cov_v,
                                mode == M_EXTEND, qo, qd, qL, qrad, best, besti, hit, hin, total, err, q_ref, q_sp,
                                q_ncov, q_ovf, q_resume, p.postpone);
    if (RTX_STAMPS) {
      t1 = stamp();
      tB += t1 - t0;
      t0 = t1;
    }
    if (PP && q_resume) continue;            // walk postponed: resumed at the next B

    // ---- C: consume the query result
    if (mode == M_EXTEND) {
      if (besti < 0) {                       // "light_dead": nothing hit
        mode = M_NEED;
        continue;
      }
      if (COUNT) cnt[C_SHADE_HITS]++;
      hit_info(S, besti, cur.ray, hit, delta, n, hin);
      nn = vnorm(n, err);                    // n.normalize, shared by every use below
      li = 0;
      nl = 0;
      lc = v3(0.0, 0.0, 0.0);
    } else {
      // World#local_lights (world.rb:72-80) fused with the light loop of
      // WorldObject#local_lighting (world_object.rb:51-74): same order, same sums.
      const double area = total > 0 ? total : 0.0;
      if (area > 0) {
        const LightDev& L = S.light[li];
        nl++;
        const double pw = S.sse_is_two ? area * area : rx_pow(area, S.sse);
        const V3 lcol = vsc(v3p(L.color), pw / (double)S.n_light);
        const V3 ll = vnorm(vsub(v3p(L.pos), hit), err);
        double ldn = vdot(ll, nn);
        if (ldn > 1) ldn = 1.0;
        else if (ldn < 0) ldn = 0.0;
        lc = vadd(lc, vsc(lcol, ldn));
      }
      li++;
    }
    if (li < S.n_light) {                    // next light: a SHADOW query from hit + delta
      const LightDev& L = S.light[li];
      mode = M_SHADOW;
      qo = vadd(hit, delta);
      qL = v3p(L.pos);
      qd = vsub(qL, qo);                     // Ray(light - target, target)
      qrad = L.radius;
      total = 1.0;
      if (RTX_STAMPS) {
        t1 = stamp();
        tC += t1 - t0;
      }
      continue;
    }
    if (RTX_STAMPS) {
      t1 = stamp();
      tC += t1 - t0;
      t0 = t1;
    }
    have = shade_finish<MAXS>(S, cam, p.seed, x, y, sample, besti, hin, hit, delta, n, nn, lc, nl, cur, st, sum,
                              err);
    mode = M_NEED;
    if (RTX_STAMPS) tD += stamp() - t0;
  }
  if (RTX_STAMPS) {                            // lane utilisation: busy wall time vs the kernel's span
    const unsigned long long w_end = wall();
    atomicMin(&rtx_stamps[8], w_start);
    atomicMax(&rtx_stamps[9], w_end);
    atomicAdd(&rtx_stamps[10], w_dry - w_start);
    atomicAdd(&rtx_stamps[11], 1ull);
    atomicAdd(&rtx_stamps[12], w_end - w_start);
    atomicMin(&rtx_stamps[13], w_dry);
    atomicMax(&rtx_stamps[14], w_dry);
    if (w_item && w_dry - w_item > w_maxitem) w_maxitem = w_dry - w_item;
    atomicMax(&rtx_stamps[15], w_maxitem);
  }
  if (RTX_STAMPS && (threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) {
    atomicAdd(&rtx_stamps[0], tA);
    atomicAdd(&rtx_stamps[1], tB);
    atomicAdd(&rtx_stamps[2], tC);
    atomicAdd(&rtx_stamps[3], tD);
    atomicAdd(&rtx_stamps[4], iters);
    atomicAdd(&rtx_stamps[5], 1ull);
    if (RTX_STAMPS == 1) atomicAdd(&rtx_stamps[6], tR);
  }

  if (COUNT)
    for (int k = 0; k < C_N; k++) atomicAdd(&p.counts[k], cnt[k]);
}

// RayTracer#path_trace_sync / #path_trace (ray_tracer.rb:181-289) for explicit
// rays, one lane per ray.  Dead code in the reference (never called), kept for
// API fidelity with its exact behaviour:
//   * trace_depth <= 0 (attenuation starts at 1): black (:197-201);
//   * a light in the highlight cone: the sum of att * color / n (:206-214);
//   * no object hit: black (:284-288);
//   * a hit: intersect_parameters runs (its normalize / asin raises come
//     first), then roulette_random sums the never-assigned *_probability
//     accessors (world_object.rb:12): `0 + nil` raises TypeError (:167).
// The Monte-Carlo children are therefore unreachable.  The walk is the
// ordered linear one (same first-index nearest hit as every other walk).
__global__ __launch_bounds__(256) void k_path_trace(KParams p) {
  const int i = blockIdx.x * 256 + (int)threadIdx.x;
  if (i >= p.nrays) return;
  const SceneDev& S = p.scene;
  Item it;
  it.ray.d = v3p(p.rays + 6 * (size_t)i);
  it.ray.o = v3p(p.rays + 6 * (size_t)i + 3);
  it.att = v3(1.0, 1.0, 1.0);
  it.path = 1;
  it.depth = p.cam->depth;
  uint32_t err = 0;
  V3 sum = v3(0.0, 0.0, 0.0);
  if (it.depth > 0 && !(vr(it.att) < 0.0001) && !highlights<false>(S, it, sum, err)) {
    double best = S.max_distance, total = 0.0;
    int besti = -1;
    V3 hit = sum;
    bool hin = true;
    query<false>(S, cptr(S.sph32), true, it.ray.o, it.ray.d, hit, 0.0, best, besti, hit, hin, total, err, nullptr);
    if (besti >= 0) {
      V3 delta, n;
      hit_info(S, besti, it.ray, hit, delta, n, hin);
      const V3 nn = vnorm(n, err);
      const double c = vcos(it.ray.d, n, err);
      const Ray refl = reflection(it.ray, nn, c, hit, delta, err);
      const Material& m = S.mat[besti];
      Ray refr;
      if (m.type == OBJ_SPHERE) refraction(it.ray, nn, c, hit, refl.d, hin ? m.rr : 1.0 / m.rr, refr, err);
      else if (m.has_rr) refraction(it.ray, nn, c, hit, refl.d, m.rr, refr, err);
      seterr(err, ERR_TYPE);
    }
  }
  p.out[3 * (size_t)i] = sum.x;
  p.out[3 * (size_t)i + 1] = sum.y;
  p.out[3 * (size_t)i + 2] = sum.z;
  if (err) record_error(p.err, err, (unsigned long long)i);
}

// Camera#render_at's reduction (camera.rb:70-99) over the sample records of
// k_render.  phase 0, every pixel of the region: mean of the pre_sample_times
// colours (in sample order), the variance test, then either the pixel's result
// or (variance >= threshold and max_sample_times > pre_sample_times) an entry in
// p.extra_list for the SRC_EXTRA launch.  phase 1, every listed pixel: the
// extra samples' sum in order and (avg * pre + cv) / max.  The first raise of a
// pixel is the one of its lowest erring sample, as in the sequential loop.
__global__ __launch_bounds__(256) void k_finalize(KParams p, int phase) {
  const int i = blockIdx.x * 256 + (int)threadIdx.x;
  int idx;
  if (phase == 0) {
    if (i >= p.nx * p.nrows) return;
    idx = i;
  } else {
    if (i >= *p.extra_count) return;
    idx = p.extra_list[i];
  }
  const int px_ = idx % p.nx, row = idx / p.nx;
  const int y = row_to_y(p, row);
  const CameraDev& cam = *p.cam;
  if (y >= cam.height) return;                       // packed rows past the image bottom
  const int x = p.x0 + px_;
  const int pre = p.pre, ms = p.max_samples > p.pre ? p.max_samples : p.pre;
  const double* q = p.samples + (size_t)idx * ms * 4;
  uint32_t err = 0;
  V3 avg = v3(0.0, 0.0, 0.0);
  if (phase == 0 && pre == 4) {                      // the common 4x case: all 8 loads in flight at once
    const double2* q2 = reinterpret_cast<const double2*>(q);
    double2 a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = q2[k];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      avg = vadd(avg, v3(a[2 * j].x, a[2 * j].y, a[2 * j + 1].x));
      if (!err) err = (uint32_t)__builtin_bit_cast(uint64_t, a[2 * j + 1].y);
    }
  } else {
    for (int j = 0; j < pre; j++) {
      avg = vadd(avg, v3(q[4 * j], q[4 * j + 1], q[4 * j + 2]));
      if (!err) err = (uint32_t)__builtin_bit_cast(uint64_t, q[4 * j + 3]);
    }
  }
  avg = vdiv(avg, (double)pre);
  if (phase == 0) {
    double variance = 0.0;                           // camera.rb:80-85
    for (int j = 0; j < pre; j++) {
      const V3 dd = vsub(v3(q[4 * j], q[4 * j + 1], q[4 * j + 2]), avg);
      double mx = dd.x;
      if (dd.y > mx) mx = dd.y;
      if (dd.z > mx) mx = dd.z;
      variance += mx * mx;                           // .max ** 2
    }
    variance /= (double)pre;
    if (variance >= cam.variant_threshold) {
      if (p.max_samples > pre) {                     // more samples: the SRC_EXTRA launch
        p.extra_list[atomicAdd(p.extra_count, 1)] = idx;
        if (err) record_error(p.err, err, px_key(x, y, cam.height));
        return;
      }
      avg = vdiv(vadd(vsc(avg, (double)pre), v3(0.0, 0.0, 0.0)), (double)p.max_samples);
    }
  } else {
    V3 cv = v3(0.0, 0.0, 0.0);
    for (int j = pre; j < p.max_samples; j++) {
      cv = vadd(cv, v3(q[4 * j], q[4 * j + 1], q[4 * j + 2]));
      if (!err) err = (uint32_t)__builtin_bit_cast(uint64_t, q[4 * j + 3]);
    }
    avg = vdiv(vadd(vsc(avg, (double)pre), cv), (double)p.max_samples);
  }
  double* o = p.out + (size_t)row * p.stride + (size_t)px_ * 3;
  o[0] = avg.x;
  o[1] = avg.y;
  o[2] = avg.z;
  if (err) record_error(p.err, err, px_key(x, y, cam.height));
}

// ================================================================= bounce levels
// The bounce-level engine (option "engine" = 1).  Instead of
// one lane walking one sample's whole ray tree (the lanes engine above), every
// ray of tree level d is one work item of the level-d launch: the camera
// samples at level 0, their live children at level 1, and so on.  A wave's 64
// lanes therefore run the same step of rt_map (ray_tracer.rb:50-164) on 64
// rays at once, and no sample's tree can hold a launch open: a launch's
// longest item is one ray.
//
// Order.  trace_sync pops rays LIFO and drains the leaves FIFO afterwards
// (ray_tracer.rb:31-45): leaves are summed in pre-order of the tree, children
// visited in reverse push order (refraction after its pt siblings, reflection
// last).  Each ray writes a tree record {first raise, leaf count, child mask,
// first child, leaves} at its level; its live children go, contiguous and in
// slot order, to the next level at an offset found by a wave prefix count
// (ballot / mbcnt / shfl) plus one atomic per wave.  k_tree_finalize walks each
// sample's tree in the reference's order and sums the leaves in it: the same
// additions in the same order as the sequential program, so the same bits.
//
// Raises.  rt_map's raises happen while the tree is walked, the "color greater
// than 1" of rt_reduce only in the drain after it (:39-45): a record keeps the
// first raise of its ray in rt_map's order (highlights; reflection and
// refraction; local_lights' lit_area; path tracing / local_lighting), the walk
// takes the first in tree order, and a >1 partial sum counts only without one.
//
// Capacity.  Children beyond the staging buffer or tree records beyond the
// record arena are not written; their camera sample is listed (lv_redo_list)
// and re-rendered whole by the lanes engine (SRC_LIST), exact either way.
constexpr int RAY_DOUBLES = 12;          // staging ray record: o, d, att, path, root item, pad (96 B)

int levels_rec_bytes(int n_light) {
  const int nl = n_light > 1 ? n_light : 1;
  return (8 + 24 * nl + 15) & ~15;       // {meta, first child} + one leaf per fired light
}

__device__ __forceinline__ uint32_t lv_count(const KParams& p, int d) {
  const uint32_t c = p.lv_ctl->count[d];
  return d == 0 ? c : (c < p.lv_scap ? c : p.lv_scap);
}

__device__ __forceinline__ void lv_redo(const KParams& p, int root) {
  if (atomicCAS(&p.lv_redo_of[root], -1, -2) == -1) {
    const uint32_t e = atomicAdd(&p.lv_ctl->redo_n, 1u);
    p.lv_redo_list[e] = root;
    p.lv_redo_of[root] = (int)e;
  }
}

// root: the level-0 item of the ray's tree; (x, y, sample): its RNG key.
__device__ __forceinline__ void lv_store_ray(double* dst, const Ray& r, V3 att, uint64_t path, int root, int x, int y,
                                             int sample) {
  double2* q = reinterpret_cast<double2*>(dst);
  q[0] = make_double2(r.o.x, r.o.y);
  q[1] = make_double2(r.o.z, r.d.x);
  q[2] = make_double2(r.d.y, r.d.z);
  q[3] = make_double2(att.x, att.y);
  q[4] = make_double2(att.z, __builtin_bit_cast(double, path));
  q[5] = make_double2(__builtin_bit_cast(double, (uint64_t)(uint32_t)root | (uint64_t)(uint32_t)sample << 32),
                      __builtin_bit_cast(double, (uint64_t)(uint32_t)x | (uint64_t)(uint32_t)y << 32));
}

// Launch `level` (0 .. trace_depth-1) of one batch.  Persistent: every wave
// claims 64-ray chunks until the level's count is exhausted.
template <int SPH, int BS>
__global__ __launch_bounds__(BS, RTX_LVL_WPS) void k_level(KParams p, int level) {
  const SceneDev& S = p.scene;
  const CameraDev& cam = *p.cam;
  extern __shared__ float4 lds_sph[];
  char* lds = reinterpret_cast<char*>(lds_sph);
  const uint32_t n = lv_count(p, level);
  if (n == 0) return;                         // uniform: before any barrier
  if (SPH == SPH_LIN_LDS) {
    for (int i = threadIdx.x; i < S.n_sphere + 4; i += BS)
      lds_sph[i] = reinterpret_cast<const float4*>(S.sph32)[i];
    __syncthreads();
  } else if (SPH == SPH_BVH_LDS) {
    const int nn = S.n_nodes * (int)(sizeof(Bvh4Node) / 16);
    for (int i = threadIdx.x; i < nn; i += BS) lds_sph[i] = reinterpret_cast<const float4*>(S.bvh)[i];
    float4* leaf = reinterpret_cast<float4*>(lds + p.lds_leaf);
    for (int i = threadIdx.x; i < S.n_slots; i += BS) leaf[i] = reinterpret_cast<const float4*>(S.bvh_sph32)[i];
    __syncthreads();
  }
  const float* sph_lds = reinterpret_cast<const float*>(lds_sph);
  const RTX_CONST float* sph_k = cptr(S.sph32);
  int* stk = reinterpret_cast<int*>(lds + p.lds_stack) + threadIdx.x;
  int* cov_i = reinterpret_cast<int*>(lds + p.lds_cov) + threadIdx.x;
  double* cov_v = reinterpret_cast<double*>(lds + p.lds_cov + COVER_K * BS * 4) + threadIdx.x;

  uint32_t base = 0;                          // this level's first record in lv_rec
  for (int e = 0; e < level; e++) base += lv_count(p, e);
  const double* __restrict__ in = p.lv_stage[level & 1];
  double* __restrict__ outs = p.lv_stage[(level + 1) & 1];
  const int depth = cam.depth - level;        // trace_depth of this level's rays
  const int pt = cam.pt;
  const uint64_t R = (uint64_t)pt + 3;
  const int lane = (int)__lane_id();

  // walk dispatch (the same query code as the lanes engine; every lane of a
  // level launch runs the same query kind at the same time)
  auto walk = [&](bool ext, V3 o, V3 d, V3 L, double rad, double& best, int& besti, V3& hit, bool& hin,
                  double& total, uint32_t& err) {
    if (SPH == SPH_LIN_LDS)
      query<false>(S, sph_lds, ext, o, d, L, rad, best, besti, hit, hin, total, err, nullptr);
    else if (SPH == SPH_LIN_SCALAR)
      query<false>(S, sph_k, ext, o, d, L, rad, best, besti, hit, hin, total, err, nullptr);
    else {
      int q_ref = BVH_NONE, q_sp = 0, q_ncov = 0;
      bool q_ovf = false;
      if (SPH == SPH_BVH_LDS)
        query_bvh<BS, false>(S, reinterpret_cast<const Bvh4Node*>(lds), reinterpret_cast<const float4*>(lds + p.lds_leaf),
                             stk, cov_i, cov_v, ext, o, d, L, rad, best, besti, hit, hin, total, err, q_ref, q_sp,
                             q_ncov, q_ovf, false, 0);
      else
        query_bvh<BS, false>(S, S.bvh, reinterpret_cast<const float4*>(S.bvh_sph32), stk, cov_i, cov_v, ext, o, d, L,
                             rad, best, besti, hit, hin, total, err, q_ref, q_sp, q_ncov, q_ovf, false, 0);
    }
  };

  unsigned long long tS[6] = {0, 0, 0, 0, 0, 0}, t0 = 0, t1, nchunks = 0;   // RTX_STAMPS diagnostic build only
#define RTX_LV_STAMP(k)  \
  if (RTX_STAMPS) {      \
    t1 = stamp();        \
    tS[k] += t1 - t0;    \
    t0 = t1;             \
  }
  // Chunk claims: one atomic per 64 rays (RTX_LV_CLAIM_AHEAD issues the next
  // claim when a chunk starts instead; measured no faster).
  int next = 0;
  if (RTX_LV_CLAIM_AHEAD) {
    if (lane == 0) next = (int)atomicAdd(&p.lv_ctl->claim[level], 1u);
  }
  while (true) {
    if (RTX_STAMPS) {
      t0 = stamp();
      nchunks++;
    }
    int chunk = 0;
    if (RTX_LV_CLAIM_AHEAD) {
      chunk = __shfl(next, 0);
      if ((uint32_t)chunk * 64u >= n) break;
      if (lane == 0) next = (int)atomicAdd(&p.lv_ctl->claim[level], 1u);
    } else {
      if (lane == 0) chunk = (int)atomicAdd(&p.lv_ctl->claim[level], 1u);
      chunk = __shfl(chunk, 0);
      if ((uint32_t)chunk * 64u >= n) break;
    }
    const uint32_t i = (uint32_t)chunk * 64u + (uint32_t)lane;
    bool active = i < n;

    // ---- the ray: a camera sample (level 0) or a staged child
    Item cur;
    int root = 0, x = 0, y = 0, sample = 0;
    bool alive = false;
    if (active) {
      if (level == 0) {
        root = (int)i;
      } else {
        const double2* q = reinterpret_cast<const double2*>(in + (size_t)i * RAY_DOUBLES);
        const double2 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5];
        cur.ray.o = v3(a.x, a.y, b.x);
        cur.ray.d = v3(b.y, c.x, c.y);
        cur.att = v3(d.x, d.y, e.x);
        cur.path = __builtin_bit_cast(uint64_t, e.y);
        const uint64_t rs = __builtin_bit_cast(uint64_t, f.x), xy = __builtin_bit_cast(uint64_t, f.y);
        root = (int)(uint32_t)rs;
        sample = (int)(rs >> 32);
        x = (int)(uint32_t)xy;
        y = (int)(xy >> 32);
      }
      if (level == 0) {
        p.lv_redo_of[i] = -1;                 // no overflow yet (lv_redo)
        const ItemPos ip = decode_item(p, root);
        x = p.x0 + ip.px;
        y = row_to_y(p, ip.row);
        sample = ip.sample;
        if (ip.valid) {
          cur.ray = lens_ray(cam, lens_target(cam, x, y), x, y, sample, p.seed);
          cur.att = v3(1.0, 1.0, 1.0);
          cur.path = 1;
          alive = !(depth <= 0 || vr(cur.att) < 0.0001);   // rt_map's cutoff (ray_tracer.rb:52)
        } else {
          active = false;                     // padding of an 8x8 tile: no record
        }
      } else {
        alive = true;                         // children are staged only past the cutoff
      }
      if (active && base + i >= p.lv_lcap) { // no room for this ray's record
        lv_redo(p, root);
        active = alive = false;
      }
    }
    char* rec = p.lv_rec + (size_t)(base + i) * p.lv_rec_bytes;
    double* leafp = reinterpret_cast<double*>(rec + 8);

    // ---- rt_map: highlights (ray_tracer.rb:60-75), raises in rt_map's order:
    // errA highlights, errS intersect_parameters (reflection / refraction),
    // errL local_lights' lit_area, errP path_tracing / local_lighting
    uint32_t errA = 0, errS = 0, errL = 0, errP = 0;
    int nleaf = 0;
    bool fired = false;
    if (alive)
      fired = highlight_leaves(S, cur, [&](V3 c) {
        leafp[3 * nleaf] = c.x;
        leafp[3 * nleaf + 1] = c.y;
        leafp[3 * nleaf + 2] = c.z;
        nleaf++;
      }, errA);

    RTX_LV_STAMP(0)
    // ---- World#intersect (world.rb:37-59)
    const bool ext = alive && !fired;
    double best = S.max_distance, total = 0.0;
    int besti = -1;
    V3 hit = v3(0.0, 0.0, 0.0);
    bool hin = true;
    if (ext) walk(true, cur.ray.o, cur.ray.d, hit, 0.0, best, besti, hit, hin, total, errL);
    const bool shade = ext && besti >= 0;
    RTX_LV_STAMP(1)

    V3 delta = hit, nrm = hit, nn = hit;
    double c = 0.0;
    if (shade) {
      hit_info(S, besti, cur.ray, hit, delta, nrm, hin);
      nn = vnorm(nrm, errS);                  // n.normalize (world_object.rb:123)
      c = vcos(cur.ray.d, nrm, errS);         // ray.front.cos(-n): same bits as cos(n)
    }
    const V3 qo = vadd(hit, delta);           // the shadow rays' target point (world.rb:76)

    RTX_LV_STAMP(2)
    // ---- World#local_lights (world.rb:72-80) fused with local_lighting's
    // light loop (world_object.rb:51-74): one SHADOW walk per light.  (Holding
    // delta / n / n.normalize across the walks measured faster than
    // recomputing them after: 6.22 vs 6.40 ms on C2.)
    V3 lc = v3(0.0, 0.0, 0.0);
    int nl = 0;
    for (int li = 0; li < S.n_light; li++) {
      if (!shade) continue;
      const LightDev& L = S.light[li];
      const V3 qL = v3p(L.pos);
      double tot = 1.0;
      double b2 = 0.0;
      int bi2 = -1;
      V3 h2 = qo;
      bool in2 = true;
      walk(false, qo, vsub(qL, qo), qL, L.radius, b2, bi2, h2, in2, tot, errL);
      const double area = tot > 0 ? tot : 0.0;
      if (area > 0) {
        nl++;
        const double pw = S.sse_is_two ? area * area : rx_pow(area, S.sse);
        const V3 lcol = vsc(v3p(L.color), pw / (double)S.n_light);
        const V3 ll = vnorm(vsub(v3p(L.pos), hit), errP);
        double ldn = vdot(ll, nn);
        if (ldn > 1) ldn = 1.0;
        else if (ldn < 0) ldn = 0.0;
        lc = vadd(lc, vsc(lcol, ldn));
      }
    }
    RTX_LV_STAMP(3)
    // ---- which children pass rt_map's cutoff (ray_tracer.rb:52) at depth - 1
    uint32_t mask = 0;
    double rate = 0.0;
    bool may_refract = false;
    const Material* m = shade ? &S.mat[besti] : S.mat;
    if (shade) {
      const int cd = depth - 1;
      if (cd > 0 && !(vr(vmul(cur.att, v3p(m->refl_att))) < 0.0001)) mask |= 1u;
      if (m->type == OBJ_SPHERE) {            // sphere.rb:92-94: rate inverted leaving
        may_refract = true;
        rate = hin ? m->rr : 1.0 / m->rr;
      } else if (m->has_rr) {                 // plane.rb:57-61: the same rate both ways
        may_refract = true;
        rate = m->rr;
      }
      if (may_refract && !(sqrt(1.0 - c * c) / rate >= 1) && cd > 0 &&
          !(vr(vmul(cur.att, v3p(m->refr_att))) < 0.0001))
        mask |= 2u;                           // refraction exists (no TIR) and is alive
      if (nl == 0 && cd > 0 && !(vr(vmul(cur.att, vdiv(v3p(m->diffuse), (double)pt))) < 0.0001))
        mask |= ((1u << pt) - 1u) << 2;       // every path-tracing child (same attenuation)
    }

    // ---- room in the next level: wave prefix count of the live children + one atomic
    const int cnt = __popc(mask);
    int incl = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(incl, off);
      if (lane >= off) incl += t;
    }
    const int wtotal = __shfl(incl, 63);
    uint32_t wbase = 0;
    if (wtotal > 0) {
      if (lane == 0) wbase = atomicAdd(&p.lv_ctl->count[level + 1], (uint32_t)wtotal);
      wbase = __shfl(wbase, 0);
    }
    const uint32_t child0 = wbase + (uint32_t)(incl - cnt);
    RTX_LV_STAMP(4)

    // ---- children in the reference's push order (ray_tracer.rb:84-143), then the leaf
    if (shade) {
      uint32_t slot = child0;
      auto put = [&](const Ray& r, V3 att, uint64_t path) {
        if (slot < p.lv_scap) lv_store_ray(outs + (size_t)slot * RAY_DOUBLES, r, att, path, root, x, y, sample);
        else {
          lv_redo(p, root);
          atomicAdd(&p.lv_ctl->dropped, 1u);
        }
        slot++;
      };
      const Ray refl = reflection(cur.ray, nn, c, hit, delta, errS);
      if (mask & 1u) put(refl, vmul(cur.att, v3p(m->refl_att)), cur.path * R + 1);
      if (may_refract) {
        Ray refr;
        if (refraction(cur.ray, nn, c, hit, refl.d, rate, refr, errS) && (mask & 2u))
          put(refr, vmul(cur.att, v3p(m->refr_att)), cur.path * R + 2);
      }
      if (nl == 0) {
        // WorldObject#path_tracing (world_object.rb:76-90) from hit + delta
        const V3 att = vmul(cur.att, vdiv(v3p(m->diffuse), (double)pt));
        const V3 left = vnorm(vertical_vector(nrm, errP), errP);
        const V3 up = vcross(nn, left);
        Ray r;
        r.o = vadd(hit, delta);
        for (int k = 0; k < pt; k++) {
          const double theta = rand01(p.seed, x, y, sample, cur.path, 2 * k) * PI / 2.0;
          const double phi = rand01(p.seed, x, y, sample, cur.path, 2 * k + 1) * PI * 2.0;
          double sth, cth, sph, cph;
          RTX_SINCOS(theta, &sth, &cth);
          RTX_SINCOS(phi, &sph, &cph);
          r.d = vadd(vsc(nn, sth), vsc(vadd(vsc(left, cph), vsc(up, sph)), cth));
          if (mask >> (2 + k) & 1u) put(r, att, cur.path * R + 3 + (uint64_t)k);
        }
      } else {
        // WorldObject#local_lighting's colour (world_object.rb:51-74), texture filter
        lc = vdiv(lc, (double)nl);
        V3 color;
        if (m->type == OBJ_BOX) {
          color = vadd(vmul(lc, v3p(m->diffuse)), v3p(m->ambient));
        } else {
          V3 filter = v3(1.0, 1.0, 1.0);
          if (m->tex >= 0) {
            if (m->type == OBJ_SPHERE) {             // Sphere#get_uv (sphere.rb:111-120)
              const Sphere64 sp = S.sph64[m->rec];
              const V3 vec = vsub(hit, v3p(sp.c));
              const double x0 = vdot(vec, v3p(m->gw_n)) / sp.r;
              const double y0 = vdot(vec, v3p(m->east_n)) / sp.r;
              const double z0 = vdot(vec, v3p(m->north_n)) / sp.r;
              const double mm2 = x0 * x0 + y0 * y0 + z0 * z0 + 2.0 * x0 + 1.0;
              if (mm2 < 0) seterr(errP, ERR_DOMAIN);
              const double mm = sqrt(mm2);
              filter = vmul(texcolor(S, m->tex, m->hs, m->vs, m->u_off, m->v_off, (y0 / mm + 1.0) / 2.0,
                                     (-z0 / mm + 1.0) / 2.0, errP), filter);
            } else {
              double u, v;
              plane_uv(S.planes + (size_t)m->rec * PLANE_GEO, hit, u, v);
              filter = vmul(texcolor(S, m->tex, m->hs, m->vs, 0.0, 0.0, u, v, errP), filter);
            }
          }
          color = vadd(vmul(vmul(lc, v3p(m->diffuse)), filter), v3p(m->ambient));
        }
        const V3 leaf = vmul(cur.att, color);
        leafp[0] = leaf.x;
        leafp[1] = leaf.y;
        leafp[2] = leaf.z;
        nleaf = 1;
      }
    }
    if (active) {
      uint32_t err = errA;
      if (!err) err = errS;
      if (!err) err = errL;
      if (!err) err = errP;
      uint2* hdr = reinterpret_cast<uint2*>(rec);
      *hdr = make_uint2((err & 0xffu) | ((uint32_t)nleaf << 8) | (mask << 16), child0);
    }
    RTX_LV_STAMP(5)
  }
#undef RTX_LV_STAMP
  if (RTX_STAMPS && lane == 0) {
    for (int k = 0; k < 6; k++) atomicAdd(&rtx_stamps[k], tS[k]);
    atomicAdd(&rtx_stamps[6], nchunks);
    atomicAdd(&rtx_stamps[7], 1ull);
  }
}

// Sum of one camera sample's tree (level-0 item `root`) in trace_sync's
// order: pre-order, children in reverse slot order; `base` = first record of
// every level.  Returns the first raise (rt_map's first, else rt_reduce's).
// The walk keeps one pending child range per level below the root in
// lo[k * st] / hi[k * st], k < sd (LDS, word-major over the block's threads,
// or a private array with st = 1).
__device__ __forceinline__ V3 lv_tree_sum(const KParams& p, const uint32_t* base, int root, int nlev,
                                          uint32_t* lo, uint32_t* hi, int st, int sd, uint32_t& err_out) {
  int sp = 0;
  V3 sum = v3(0.0, 0.0, 0.0);
  uint32_t err = 0, pf = 0;
  bool gt1 = false;
  int lev = 0;
  uint32_t q = (uint32_t)root;
  while (true) {
    const char* rec = p.lv_rec + (size_t)(base[lev] + q) * p.lv_rec_bytes;
    const uint2 hdr = *reinterpret_cast<const uint2*>(rec);
    const double* lf = reinterpret_cast<const double*>(rec + 8);
    const double2 l01 = *reinterpret_cast<const double2*>(lf);   // the first leaf, with the header's sector
    const double l2 = lf[2];
    if (!err) err = hdr.x & 0xffu;
    const int nleaf = (int)(hdr.x >> 8 & 0xffu);
    if (nleaf > 0) {                           // rt_reduce (ray_tracer.rb:292-298), in emission order
      sum = vadd(sum, v3(l01.x, l01.y, l2));
      if (!(sum.x <= 1 && sum.y <= 1 && sum.z <= 1)) gt1 = true;
      for (int k = 1; k < nleaf; k++) {
        sum = vadd(sum, v3(lf[3 * k], lf[3 * k + 1], lf[3 * k + 2]));
        if (!(sum.x <= 1 && sum.y <= 1 && sum.z <= 1)) gt1 = true;
      }
    }
    const uint32_t nch = (uint32_t)__popc(hdr.x >> 16);
    if (nch && lev + 1 < nlev && sp < sd) {
      lo[sp * st] = hdr.y;
      hi[sp * st] = hdr.y + nch;
      sp++;
      // the children's records (contiguous, slot order) are fetched now, all
      // at once: the walk's dependent chain becomes the tree's depth, not
      // its size (the loads' values are consumed only at the end)
      const char* c0 = p.lv_rec + (size_t)(base[lev + 1] + hdr.y) * p.lv_rec_bytes;
      pf += *reinterpret_cast<const uint32_t*>(c0) +
            *reinterpret_cast<const uint32_t*>(c0 + (size_t)(nch - 1) * p.lv_rec_bytes);
    }
    // next: the last unvisited child of the deepest pending range (LIFO pop)
    while (sp > 0 && hi[(sp - 1) * st] == lo[(sp - 1) * st]) sp--;
    if (sp == 0) break;
    q = --hi[(sp - 1) * st];
    lev = sp;
  }
  asm volatile("" : : "v"(pf));               // the prefetches' values, consumed
  err_out = err ? err : (gt1 ? (uint32_t)ERR_COLOR_GT1 : 0u);
  return sum;
}

// Block 0 also adds the batch's level statistics to lv_acc (rtx_level_stats):
// every level launch of the batch has ended.
__device__ __forceinline__ void lv_bases(const KParams& p, int nlev, uint32_t* base) {
  if (threadIdx.x == 0) {
    uint32_t b = 0;
    for (int d = 0; d <= nlev && d <= LV_MAXL; d++) {
      base[d] = b;
      b += lv_count(p, d);
    }
  }
  if (blockIdx.x == 0 && p.lv_acc) {
    const int t = (int)threadIdx.x;
    if (t == 0) p.lv_acc[0] += p.lv_ctl->redo_n;
    if (t == 1) p.lv_acc[1] += p.lv_ctl->dropped;
    if (t < LV_MAXL + 1) p.lv_acc[2 + t] += p.lv_ctl->count[t];
  }
  __syncthreads();
}

// One camera sample's colour and first raise: its tree, or the lanes engine's
// record when the sample overflowed the level buffers.
__device__ __forceinline__ V3 lv_sample(const KParams& p, const uint32_t* base, int item, int nlev, uint32_t* lo,
                                        uint32_t* hi, int st, int sd, uint32_t& e) {
  const int r = p.lv_redo_of[item];
  if (r >= 0) {
    const double* q = p.lv_redo_smp + (size_t)r * 4;
    e = (uint32_t)__builtin_bit_cast(uint64_t, q[3]);
    return v3(q[0], q[1], q[2]);
  }
  return lv_tree_sum(p, base, item, nlev, lo, hi, st, sd, e);
}

// Camera#render_at's reduction (camera.rb:70-99) of pass 0: one 256-thread
// block per 8x8 tile of the batch.  The block's threads sum the tile's
// 64 x pre sample trees (item order (pixel, sample): a wave's trees are
// neighbours), park colour and raise in LDS, then 64 threads do the pixels:
// mean in sample order, the variance test, then the pixel or (max_sample_times
// > pre) an extra-list entry with the pre mean parked in the output.
// Dynamic LDS: SD * 2 words of walk stack per thread, then 64 * pre samples.
template <int SD>
__global__ __launch_bounds__(256) void k_tree_finalize(KParams p, int nlev) {
  __shared__ uint32_t base[LV_MAXL + 1];
  extern __shared__ uint32_t lds_fin[];
  lv_bases(p, nlev, base);
  const int pre = p.pre;
  const int slot = blockIdx.x;                 // tile of the batch
  uint32_t* lo = lds_fin + threadIdx.x;
  uint32_t* hi = lo + SD * 256;
  double* scol = reinterpret_cast<double*>(lds_fin + 2 * SD * 256);   // 64 * pre * 3
  uint32_t* serr = reinterpret_cast<uint32_t*>(scol + 64 * pre * 3);
  uint32_t lo_p[SD > 16 ? LV_MAXL : 1], hi_p[SD > 16 ? LV_MAXL : 1];  // deep trees: private stack
  const int n_items = 64 * pre;
  const int item0 = slot * n_items;
  for (int it = (int)threadIdx.x; it < n_items; it += 256) {
    const ItemPos ip = decode_item(p, item0 + it);
    if (!ip.valid) continue;
    uint32_t e = 0;
    const V3 c = SD > 16 ? lv_sample(p, base, item0 + it, nlev, lo_p, hi_p, 1, LV_MAXL, e)
                         : lv_sample(p, base, item0 + it, nlev, lo, hi, 256, SD, e);
    scol[3 * it] = c.x;
    scol[3 * it + 1] = c.y;
    scol[3 * it + 2] = c.z;
    serr[it] = e;
  }
  __syncthreads();
  const int l = (int)threadIdx.x;
  if (l >= 64) return;
  const int tiles_x = (p.nx + 7) >> 3;
  const int tile = p.lv_t0 + slot;
  const int px_ = (tile % tiles_x) * 8 + ((l & 1) | ((l >> 1) & 2) | ((l >> 2) & 4));
  const int row = (tile / tiles_x) * 8 + (((l >> 1) & 1) | ((l >> 2) & 2) | ((l >> 3) & 4));
  if (px_ >= p.nx || row >= p.nrows) return;
  const int y = row_to_y(p, row);
  const CameraDev& cam = *p.cam;
  if (y >= cam.height) return;
  const int x = p.x0 + px_;
  const double* sc = scol + 3 * l * pre;
  uint32_t err = 0;
  V3 avg = v3(0.0, 0.0, 0.0);
  for (int j = 0; j < pre; j++) {
    avg = vadd(avg, v3(sc[3 * j], sc[3 * j + 1], sc[3 * j + 2]));
    if (!err) err = serr[l * pre + j];
  }
  avg = vdiv(avg, (double)pre);
  double variance = 0.0;                       // camera.rb:80-85
  for (int j = 0; j < pre; j++) {
    const V3 dd = vsub(v3(sc[3 * j], sc[3 * j + 1], sc[3 * j + 2]), avg);
    double mx = dd.x;
    if (dd.y > mx) mx = dd.y;
    if (dd.z > mx) mx = dd.z;
    variance += mx * mx;                       // .max ** 2
  }
  variance /= (double)pre;
  double* o = p.out + (size_t)row * p.stride + (size_t)px_ * 3;
  if (variance >= cam.variant_threshold) {
    if (p.max_samples > pre) {                 // extra samples: pass 1 finishes this pixel
      p.extra_list[atomicAdd(p.extra_count, 1)] = row * p.nx + px_;
      o[0] = avg.x;
      o[1] = avg.y;
      o[2] = avg.z;
      if (err) record_error(p.err, err, px_key(x, y, cam.height));
      return;
    }
    avg = vdiv(vadd(vsc(avg, (double)pre), v3(0.0, 0.0, 0.0)), (double)p.max_samples);
  }
  o[0] = avg.x;
  o[1] = avg.y;
  o[2] = avg.z;
  if (err) record_error(p.err, err, px_key(x, y, cam.height));
}

// Pass 1: one thread per extra-list entry of the batch: (pre mean * pre +
// the extra samples in order) / max_sample_times.
template <int SD>
__global__ __launch_bounds__(256) void k_tree_finalize_extra(KParams p, int nlev) {
  __shared__ uint32_t base[LV_MAXL + 1];
  extern __shared__ uint32_t lds_fin[];
  lv_bases(p, nlev, base);
  uint32_t* lo = lds_fin + threadIdx.x;
  uint32_t* hi = lo + SD * 256;
  uint32_t lo_p[SD > 16 ? LV_MAXL : 1], hi_p[SD > 16 ? LV_MAXL : 1];
  const int t = blockIdx.x * 256 + (int)threadIdx.x;
  if (t >= p.lv_entries || p.lv_e0 + t >= *p.extra_count) return;
  const int idx = p.extra_list[p.lv_e0 + t];
  const int px_ = idx % p.nx, row = idx / p.nx;
  const int y = row_to_y(p, row);
  const CameraDev& cam = *p.cam;
  if (y >= cam.height) return;
  const int x = p.x0 + px_;
  const int pre = p.pre, n_extra = p.max_samples - pre;
  double* o = p.out + (size_t)row * p.stride + (size_t)px_ * 3;
  const V3 avg = v3(o[0], o[1], o[2]);         // the pre mean parked by pass 0
  V3 cv = v3(0.0, 0.0, 0.0);
  uint32_t err = 0;
  for (int j = 0; j < n_extra; j++) {
    uint32_t e = 0;
    const int item = t * n_extra + j;
    cv = vadd(cv, SD > 16 ? lv_sample(p, base, item, nlev, lo_p, hi_p, 1, LV_MAXL, e)
                          : lv_sample(p, base, item, nlev, lo, hi, 256, SD, e));
    if (!err) err = e;
  }
  const V3 r = vdiv(vadd(vsc(avg, (double)pre), cv), (double)p.max_samples);
  o[0] = r.x;
  o[1] = r.y;
  o[2] = r.z;
  if (err) record_error(p.err, err, px_key(x, y, cam.height));
}

// Per batch: the control block, count[0] = the batch's level-0 items (pass 1:
// from the device-side extra count), the lanes engine's work counter (the
// re-render launch); the call's first batch also the extra-list count and the
// level statistics.  (Every level-0 lane sets its item's redo slot to -1.)
__global__ __launch_bounds__(256) void k_level_begin(KParams p, int n0_max, int first) {
  const int t = blockIdx.x * 256 + (int)threadIdx.x;
  if (t == 0) *p.work = 0;
  if (first) {
    if (t == 0) *p.extra_count = 0;
    if (p.lv_acc && t < LV_MAXL + 3) p.lv_acc[t] = 0;
  }
  if (t < 2 * (LV_MAXL + 1) + 2) {
    uint32_t v = 0;
    if (t == 0) {
      if (p.lv_pass == 0) {
        v = (uint32_t)n0_max;
      } else {
        const int left = *p.extra_count - p.lv_e0;
        const int ent = left < 0 ? 0 : (left < p.lv_entries ? left : p.lv_entries);
        v = (uint32_t)(ent * (p.max_samples - p.pre));
      }
    }
    reinterpret_cast<uint32_t*>(p.lv_ctl)[t] = v;
  }
}

// ----------------------------------------------------------------- tile order
// Expensive tiles first (longest-processing-time order).  The frame's tail is
// the lanes that are still inside a deep glass/mirror ray tree when the work
// pool runs dry; handing those trees out first leaves cheap items for the end.
// The order of work items changes no bit: every item writes its own record.
//
// k_tile_cost: one lane per probe, 4 probes per tile (the quadrant centres,
// sample 0's lens ray), each an ordered nearest-hit walk.  A probe weighs
// 1 for a hit, +1 for a reflective and +3 for a refractive material (the
// children of ray_tracer.rb:84-112 that pass the cutoff of :61); a tile's
// class is the sum, clamped to TILE_CLASSES - 1.  (Following the mirror
// bounce as well measured no better on C2.)
constexpr int TILE_CLASSES = 16;
constexpr int TILE_SORT_LDS = 64 * 1024;          // k_tile_sort stages up to this many classes in LDS
__global__ __launch_bounds__(256) void k_tile_cost(KParams p, int32_t* cls) {
  const int i = blockIdx.x * 256 + (int)threadIdx.x;
  const int tiles_x = (p.nx + 7) >> 3;
  const int tiles = tiles_x * ((p.nrows + 7) >> 3);
  const int tile = i >> 2, q = i & 3;
  int w = 0;
  if (tile < tiles) {
    const int px_ = (tile % tiles_x) * 8 + 2 + 3 * (q & 1);
    const int row = (tile / tiles_x) * 8 + 2 + 3 * (q >> 1);
    const CameraDev& cam = *p.cam;
    const int y = row_to_y(p, row);
    if (px_ < p.nx && row < p.nrows && y < cam.height) {
      const SceneDev& S = p.scene;
      const int x = p.x0 + px_;
      const Ray r = lens_ray(cam, lens_target(cam, x, y), x, y, 0, p.seed);
      double best = S.max_distance, total = 0.0;
      int besti = -1;
      bool hin = true;
      uint32_t err = 0;                              // a probe raises nothing
      V3 hit = v3(0.0, 0.0, 0.0);
      query<false>(S, cptr(S.sph32), true, r.o, r.d, hit, 0.0, best, besti, hit, hin, total, err, nullptr);
      if (besti >= 0) {
        const Material& m = S.mat[besti];
#if RTX_PROBE_W == 1
        const double ra = vr(v3p(m.refl_att));
        w = 1 + (ra >= 0.0001 ? (ra >= 0.5 ? 2 : 1) : 0) + (m.has_rr && vr(v3p(m.refr_att)) >= 0.0001 ? 6 : 0);
#elif RTX_PROBE_W == 2
        w = 1 + (vr(v3p(m.refl_att)) >= 0.0001 ? 1 : 0) + (m.has_rr && vr(v3p(m.refr_att)) >= 0.0001 ? 2 : 0);
#elif RTX_PROBE_W == 3
        w = (m.has_rr && vr(v3p(m.refr_att)) >= 0.0001) ? 2 : 1;
#else
        w = 1 + (vr(v3p(m.refl_att)) >= 0.0001 ? 1 : 0) + (m.has_rr && vr(v3p(m.refr_att)) >= 0.0001 ? 3 : 0);
#endif
      }
    }
  }
  w += __shfl_xor(w, 1);
  w += __shfl_xor(w, 2);
  if (q == 0 && tile < tiles) cls[tile] = w < TILE_CLASSES ? w : TILE_CLASSES - 1;
}

// k_tile_sort: one workgroup; a stable counting sort of the tiles by class,
// most expensive class first, into p.tile_order (deterministic: thread t owns
// a contiguous chunk of tiles; offsets are scanned in (class desc, t) order).
// Strided ownership (coalesced reads, 30 vs 59 us) scattered the tiles of a
// class over the frame and measured 9.36 vs 8.59 ms per C2 k_render.
__global__ __launch_bounds__(1024) void k_tile_sort(KParams p, const int32_t* cls, int32_t* order) {
  const int tiles = ((p.nx + 7) >> 3) * ((p.nrows + 7) >> 3);
  const int t = (int)threadIdx.x;
#ifndef RTX_TILE_SORT_STRIDED
#define RTX_TILE_SORT_STRIDED 0
#endif
  const int chunk = RTX_TILE_SORT_STRIDED ? 1024 : (tiles + 1023) >> 10;   // step between a thread's tiles
  const int t0 = RTX_TILE_SORT_STRIDED ? t : t * chunk;
  const int t1 = RTX_TILE_SORT_STRIDED ? tiles : min(tiles, t0 + chunk);
  const int st = RTX_TILE_SORT_STRIDED ? 1024 : 1;
  __shared__ int cnt[TILE_CLASSES * 1024];        // [class desc][thread]
  __shared__ int part[1024];
  __shared__ uint8_t cl8[TILE_SORT_LDS];        // the classes, staged with coalesced reads when they fit
  const bool staged = tiles <= TILE_SORT_LDS;
  if (staged)
    for (int k = t; k < tiles; k += 1024) cl8[k] = (uint8_t)cls[k];
  for (int c = 0; c < TILE_CLASSES; c++) cnt[c * 1024 + t] = 0;
  __syncthreads();
  for (int k = t0; k < t1; k += st) cnt[(TILE_CLASSES - 1 - (staged ? cl8[k] : cls[k])) * 1024 + t]++;
  __syncthreads();
  // exclusive scan of the 16384 counts: thread t scans entries [16t, 16t+16)
  int run = 0;
  for (int j = 0; j < TILE_CLASSES; j++) {
    const int v = cnt[t * TILE_CLASSES + j];
    cnt[t * TILE_CLASSES + j] = run;
    run += v;
  }
  part[t] = run;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {     // inclusive scan of the partial sums
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const int base = t > 0 ? part[t - 1] : 0;
  for (int j = 0; j < TILE_CLASSES; j++) cnt[t * TILE_CLASSES + j] += base;
  __syncthreads();
  for (int k = t0; k < t1; k += st) order[cnt[(TILE_CLASSES - 1 - (staged ? cl8[k] : cls[k])) * 1024 + t]++] = k;
}

// rtx_render_multi: the rank-major packed tiles gathered on one device ->
// the frame (camera.rb:42-51 merges the children's bands the same way).  One
// thread per double of the frame; packed row r of rank k is image row
// ((r / tile_rows) * n + k) * tile_rows + r % tile_rows.
__global__ void k_unpack(const double* __restrict__ gathered, int w, int h, int tile_rows, int n, int rows_per_rank,
                         double* __restrict__ out, size_t stride) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per_row = (long)w * 3;
  if (i >= (long)n * rows_per_rank * per_row) return;
  const int src_row = (int)(i / per_row);
  const int k = src_row / rows_per_rank, r = src_row - k * rows_per_rank;
  const int y = ((r / tile_rows) * n + k) * tile_rows + r % tile_rows;
  if (y >= h) return;
  out[(size_t)y * stride + (i - (long)src_row * per_row)] = gathered[i];
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
extern "C" int rtxdbg_read_stamps(unsigned long long* out, int reset) {   // diagnostic builds
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rtx_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {0, 0, 0, 0, 0, 0, 0, 0, ~0ull, 0, 0, 0, 0, ~0ull, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rtx_stamps), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}

int stack_bucket(int need) {
  if (need <= 8) return 8;
  if (need <= 16) return 16;
  if (need <= 32) return 32;
  if (need <= 64) return 64;
  return -1;
}

// LDS budgets.  Linear walk: 16 B per sphere in 256-thread workgroups, small
// enough for several workgroups per CU.  Hierarchy: nodes + leaf records in
// one 512-thread workgroup per CU (2 waves per SIMD, the register-limited
// occupancy), next to its stacks and cover lists.
constexpr size_t LDS_SPHERE_BYTES = 32 * 1024;
constexpr size_t LDS_TOTAL_BYTES = 160 * 1024;
constexpr size_t LDS_LIN_BLOCK_BYTES = 76 * 1024;   // two 256-thread workgroups per CU
#ifndef RTX_BS_BVH
#define RTX_BS_BVH 512
#endif
constexpr int BS_LIN = 256, BS_BVH = RTX_BS_BVH;
#ifndef RTX_WPS
#define RTX_WPS 2            // waves per SIMD the kernels are compiled for (256 VGPRs)
#endif

size_t bvh_lds_bytes(int n_nodes, int n_slots, int bvh_stack) {
  return (size_t)n_nodes * sizeof(Bvh4Node) + (size_t)n_slots * 16 + (size_t)bvh_stack * BS_BVH * 4 +
         (size_t)COVER_K * BS_BVH * 12 + 64;
}
size_t bvh_lds_budget() { return LDS_TOTAL_BYTES; }

int resolve_mode(const SceneDev& S, int mode) {
  if (mode == SPH_LIN_LDS && (size_t)(S.n_sphere + 4) * 16 > LDS_SPHERE_BYTES) return SPH_LIN_SCALAR;
  if (mode == SPH_BVH_LDS && bvh_lds_bytes(S.n_nodes, S.n_slots, S.bvh_stack) > LDS_TOTAL_BYTES)
    return SPH_BVH_GLOBAL;
  return mode;
}

// Fills the LDS layout of `p` for `mode` and returns the dynamic LDS bytes.
static size_t lds_layout(KParams& p, int mode, int bs) {
  const SceneDev& S = p.scene;
  size_t off = 0;
  if (mode == SPH_LIN_LDS) off = (size_t)(S.n_sphere + 4) * 16;
  if (mode == SPH_BVH_LDS) {
    off = (size_t)S.n_nodes * sizeof(Bvh4Node);
    p.lds_leaf = (int32_t)off;
    off += (size_t)S.n_slots * 16;
  }
  off = (off + 15) & ~(size_t)15;
  p.lds_stack = (int32_t)off;
  p.lds_cov = (int32_t)off;
  if (mode == SPH_BVH_LDS || mode == SPH_BVH_GLOBAL) {
    off += (size_t)S.bvh_stack * bs * 4;
    off = (off + 15) & ~(size_t)15;
    p.lds_cov = (int32_t)off;
    off += (size_t)COVER_K * bs * 12;
  }
  // the bottom of every lane's ray stack, as many entries as fit the budget
  off = (off + 15) & ~(size_t)15;
  p.lds_items = (int32_t)off;
  const size_t budget = (mode == SPH_BVH_LDS || mode == SPH_BVH_GLOBAL) ? LDS_TOTAL_BYTES : LDS_LIN_BLOCK_BYTES;
  const size_t per = (size_t)ITEM_WORDS * 8 * bs;
  int slots = budget > off ? (int)((budget - off) / per) : 0;
  if (slots > p.stk_slots_max) slots = p.stk_slots_max;
  p.stk_slots = slots;
  off += (size_t)slots * per;
  return off;
}

static thread_local KernelEvents* g_kev = nullptr;   // set by launch_render for its launches
static thread_local bool g_work_zeroed = false;      // launch_one: the work counter is already zero

// Persistent launch: as many workgroups as can be resident at once (the
// occupancy API; an over-estimate only leaves blocks that start after the
// pool is empty and exit at once), never more than the work needs.
template <bool COUNT, int MAXS, int SPH, int SRC, bool PP = false>
static hipError_t launch_one(KParams p, int nwork, hipStream_t s) {
  constexpr int BS = (SPH == SPH_BVH_LDS || SPH == SPH_BVH_GLOBAL) ? BS_BVH : BS_LIN;
  const size_t lds = lds_layout(p, SPH, BS);
  auto kern = k_render<COUNT, MAXS, RTX_WPS, SPH, SRC, BS, PP>;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  int dev = 0, cus = 0, per_cu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, BS, lds);
  if (e != hipSuccess) return e;
  if (per_cu < 1) per_cu = 1;
  const long need = ((long)nwork + BS - 1) / BS;
  long blocks = std::min<long>(need, (long)cus * per_cu);
  blocks = std::min<long>(blocks, (long)p.stk_glb_lanes / BS);   // lanes with a global ray-stack region
  if (blocks <= 0) return hipSuccess;
  if (!g_work_zeroed) e = hipMemsetAsync(p.work, 0, sizeof(int), s);
  if (e != hipSuccess) return e;
  KernelEvents* kev = g_kev && g_kev->n < g_kev->max ? g_kev : nullptr;
  if (kev) (void)hipEventRecord(kev->ev[2 * kev->n], s);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(BS), lds, s, p);
  e = hipGetLastError();
  if (kev) {
    (void)hipEventRecord(kev->ev[2 * kev->n + 1], s);
    kev->n++;
  }
  return e;
}

template <bool COUNT, int MAXS, int SRC>
static hipError_t launch_mode(const KParams& p, int mode, int nwork, hipStream_t s) {
  switch (mode) {
    case SPH_LIN_LDS: return launch_one<COUNT, MAXS, SPH_LIN_LDS, SRC>(p, nwork, s);
    case SPH_LIN_SCALAR: return launch_one<COUNT, MAXS, SPH_LIN_SCALAR, SRC>(p, nwork, s);
    case SPH_BVH_LDS:
      if (!COUNT && p.postpone > 0) return launch_one<false, MAXS, SPH_BVH_LDS, SRC, true>(p, nwork, s);
      if (!COUNT) return launch_one<false, MAXS, SPH_BVH_LDS, SRC>(p, nwork, s);
      break;
    case SPH_BVH_GLOBAL:
      if (!COUNT && p.postpone > 0) return launch_one<false, MAXS, SPH_BVH_GLOBAL, SRC, true>(p, nwork, s);
      if (!COUNT) return launch_one<false, MAXS, SPH_BVH_GLOBAL, SRC>(p, nwork, s);
      break;
  }
  return hipErrorInvalidValue;
}

template <int SRC>
static hipError_t launch_src(const KParams& p, int mode, bool count, int maxs, int nwork, hipStream_t s) {
#define RTX_L(M)                                                                                     \
  if (maxs == M)                                                                                     \
    return count ? launch_mode<true, M, SRC>(p, mode, nwork, s) : launch_mode<false, M, SRC>(p, mode, nwork, s);
  RTX_L(8) RTX_L(16) RTX_L(32) RTX_L(64)
#undef RTX_L
  return hipErrorInvalidValue;
}

// Camera#render_at over a region: the pre samples of every pixel, the
// reduction, then (only when max_sample_times > pre_sample_times) the extra
// samples of the pixels whose variance asked for them and their reduction.
// All on stream `s`; p.samples / extra_list / extra_count are the caller's.
struct KevScope {                   // g_kev for the duration of one launch_render
  explicit KevScope(KernelEvents* k) { g_kev = k; }
  ~KevScope() { g_kev = nullptr; }
};

hipError_t launch_render(KParams p, int mode, bool count, int maxs, hipStream_t s, KernelEvents* kev) {
  const int tiles = ((p.nx + 7) / 8) * ((p.nrows + 7) / 8);
  if (tiles == 0) return hipSuccess;
  KevScope kscope(count ? nullptr : kev);
  if (count) mode = (mode == SPH_LIN_LDS || mode == SPH_BVH_LDS) ? SPH_LIN_LDS : SPH_LIN_SCALAR;
  mode = resolve_mode(p.scene, mode);
  hipError_t e = hipMemsetAsync(p.extra_count, 0, sizeof(int32_t), s);
  if (e == hipSuccess && p.tile_order && !count) {   // expensive tiles first (k_tile_cost)
    hipLaunchKernelGGL(k_tile_cost, dim3((unsigned)((tiles * 4 + 255) / 256)), dim3(256), 0, s, p, p.tile_cls);
    hipLaunchKernelGGL(k_tile_sort, dim3(1), dim3(1024), 0, s, p, p.tile_cls, p.tile_order);
    e = hipGetLastError();
  } else {
    p.tile_order = nullptr;
  }
  if (e == hipSuccess) e = launch_src<SRC_PIXELS>(p, mode, count, maxs, tiles * 64 * p.pre, s);
  const int npx = p.nx * p.nrows;
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, s, p, 0);
    e = hipGetLastError();
  }
  if (e != hipSuccess || p.max_samples <= p.pre) return e;
  // extra samples: at most npx * (max - pre) items; the count is on the device
  e = launch_src<SRC_EXTRA>(p, mode, count, maxs, npx * (p.max_samples - p.pre), s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, s, p, 1);
    e = hipGetLastError();
  }
  return e;
}


// ----------------------------------------------------------------- bounce-level launchers
template <int SPH>
static hipError_t launch_level(const KParams& p, int level, long cap_items, hipStream_t s, KernelEvents* kev) {
  constexpr int BS = (SPH == SPH_BVH_LDS || SPH == SPH_BVH_GLOBAL) ? BS_BVH : BS_LIN;
  KParams q = p;
  q.stk_slots_max = 0;                         // no ray stack in this engine
  const size_t lds = lds_layout(q, SPH, BS);
  auto kern = k_level<SPH, BS>;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
  int dev = 0, cus = 0, per_cu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, BS, lds);
  if (e != hipSuccess) return e;
  if (per_cu < 1) per_cu = 1;
  long blocks = std::min<long>((cap_items + BS - 1) / BS, (long)cus * per_cu);
  if (blocks < 1) blocks = 1;
  const bool ev = kev && kev->n < kev->max;
  if (ev) (void)hipEventRecord(kev->ev[2 * kev->n], s);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(BS), lds, s, q, level);
  e = hipGetLastError();
  if (ev) {
    (void)hipEventRecord(kev->ev[2 * kev->n + 1], s);
    kev->n++;
  }
  return e;
}

static hipError_t launch_level_mode(const KParams& p, int mode, int level, long cap, hipStream_t s,
                                    KernelEvents* kev) {
  switch (mode) {
    case SPH_LIN_LDS: return launch_level<SPH_LIN_LDS>(p, level, cap, s, kev);
    case SPH_LIN_SCALAR: return launch_level<SPH_LIN_SCALAR>(p, level, cap, s, kev);
    case SPH_BVH_LDS: return launch_level<SPH_BVH_LDS>(p, level, cap, s, kev);
    case SPH_BVH_GLOBAL: return launch_level<SPH_BVH_GLOBAL>(p, level, cap, s, kev);
  }
  return hipErrorInvalidValue;
}

template <int SD>
static hipError_t launch_finalize_sd(const KParams& q, int nlev, int n, hipStream_t s) {
  const size_t stack = SD > 16 ? 0 : (size_t)SD * 2 * 256 * 4;
  if (q.lv_pass == 0) {                        // n = tiles of the batch
    const size_t lds = stack + (size_t)64 * q.pre * 28;
    hipLaunchKernelGGL(k_tree_finalize<SD>, dim3((unsigned)n), dim3(256), lds, s, q, nlev);
  } else {                                     // n = extra-list entries of the batch
    hipLaunchKernelGGL(k_tree_finalize_extra<SD>, dim3((unsigned)((n + 255) / 256)), dim3(256), stack, s, q, nlev);
  }
  return hipGetLastError();
}

static hipError_t launch_finalize(const KParams& q, int nlev, int n, hipStream_t s) {
  if (nlev <= 8) return launch_finalize_sd<8>(q, nlev, n, s);
  if (nlev <= 16) return launch_finalize_sd<16>(q, nlev, n, s);
  return launch_finalize_sd<64>(q, nlev, n, s);
}

// One batch: reset, the levels, the lanes-engine re-render of overflowed
// samples (exits at once when there are none), the tree reduction.
static hipError_t level_batch(KParams q, int mode, int maxs, int nlev, int n0_max, int fin_threads, hipStream_t s,
                              KernelEvents* kev, bool first) {
  hipLaunchKernelGGL(k_level_begin, dim3(1), dim3(256), 0, s, q, n0_max, first ? 1 : 0);
  hipError_t e = hipGetLastError();
  for (int d = 0; d < nlev && e == hipSuccess; d++)
    e = launch_level_mode(q, mode, d, d == 0 ? (long)n0_max : (long)q.lv_scap, s, kev);
  g_work_zeroed = true;                        // k_level_begin zeroed the re-render launch's counter
  if (e == hipSuccess) e = launch_src<SRC_LIST>(q, mode, false, maxs, n0_max, s);
  g_work_zeroed = false;
  if (e == hipSuccess && fin_threads > 0) e = launch_finalize(q, nlev, fin_threads, s);

  return e;
}

hipError_t launch_levels(KParams p, int mode, int maxs, int nlev, int batch_tiles, hipStream_t s,
                         KernelEvents* kev) {
  const int tiles = ((p.nx + 7) / 8) * ((p.nrows + 7) / 8);
  if (tiles == 0) return hipSuccess;
  mode = resolve_mode(p.scene, mode);
  batch_tiles = std::max(1, std::min(batch_tiles, tiles));
  const int per_tile = 64 * p.pre;
  p.tile_order = nullptr;
  hipError_t e = hipSuccess;                   // (the first batch's k_level_begin zeroes the extra count)
  for (int t0 = 0; t0 < tiles && e == hipSuccess; t0 += batch_tiles) {
    KParams q = p;
    q.lv_pass = 0;
    q.lv_t0 = t0;
    q.lv_tiles = std::min(batch_tiles, tiles - t0);
    q.lv_e0 = q.lv_entries = 0;
    e = level_batch(q, mode, maxs, nlev, q.lv_tiles * per_tile, q.lv_tiles, s, kev, t0 == 0);
  }
  if (e != hipSuccess || p.max_samples <= p.pre) return e;
  // extra samples of the pixels the variance test listed (count on the device)
  const int n_extra = p.max_samples - p.pre;
  const int entries = std::max(1, batch_tiles * per_tile / n_extra);
  const int npx = p.nx * p.nrows;
  for (int e0 = 0; e0 < npx && e == hipSuccess; e0 += entries) {
    KParams q = p;
    q.lv_pass = 1;
    q.lv_e0 = e0;
    q.lv_entries = std::min(entries, npx - e0);
    q.lv_t0 = q.lv_tiles = 0;
    e = level_batch(q, mode, maxs, nlev, q.lv_entries * n_extra, q.lv_entries, s, kev, false);
  }
  return e;
}

hipError_t launch_trace(KParams p, int mode, int maxs, hipStream_t s) {
  if (p.nrays == 0) return hipSuccess;
  mode = resolve_mode(p.scene, mode);
  switch (maxs) {
    case 8: return launch_mode<false, 8, SRC_RAYS>(p, mode, p.nrays, s);
    case 16: return launch_mode<false, 16, SRC_RAYS>(p, mode, p.nrays, s);
    case 32: return launch_mode<false, 32, SRC_RAYS>(p, mode, p.nrays, s);
    case 64: return launch_mode<false, 64, SRC_RAYS>(p, mode, p.nrays, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_path_trace(KParams p, hipStream_t s) {
  if (p.nrays <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_path_trace, dim3((unsigned)((p.nrays + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_unpack(const double* gathered, int w, int h, int tile_rows, int n, int rows_per_rank,
                         double* out, size_t stride, hipStream_t s) {
  const long total = (long)n * rows_per_rank * w * 3;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, gathered, w, h, tile_rows, n,
                     rows_per_rank, out, stride);
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
