// rtx_device.h — device code shared by the two kernel translation units:
// rtx_kernels.hip (lanes engine, finalize, tile order, quantize) and
// rtx_levels.hip (bounce-level engine).  Scene walks, shading, Vec3, RNG,
// the work-item decoding, and the LDS layout of a walk workgroup.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "rtx_launch.h"
#include "rtx_scene.h"
#include "rtx_vec3.h"

namespace rtx {

constexpr double PI = 3.141592653589793;   // Math::PI == M_PI
constexpr double EPS = 1e-5;               // Alex::EPSILON (src/libs/algebra.rb:2)
typedef float F2 __attribute__((ext_vector_type(2)));   // packed FP32 pair (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32)

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
static __device__ unsigned long long rtx_stamps[16];   // one per translation unit (no -fgpu-rdc)
#ifndef RTX_WALKSTATS
#define RTX_WALKSTATS 0      // diagnostic build only: lane occupancy of the hierarchy walk's loops
#endif
// [0] wave iterations of the inner-node loop, [1] lanes in them, [2] leaf
// visits (wave), [3] lanes in them; [4..7] the same for SHADOW walks
static __device__ unsigned long long rtx_walkstats[8];
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

// ----------------------------------------------------------------- World#lit_area's raises
// Sphere#cover_area (sphere.rb:28-57) runs its penumbra arithmetic for every
// sphere, whatever its binary factor, and Math.acos raises Math::DomainError
// for a cos_theta below -1 (only the upper clamp exists, :43-44).  Inside the
// branch d > |R - r1| neither can be below -1 in exact arithmetic:
//   cos_theta1 + 1 = (r1 + d - R)(r1 + d + R) / (2 r1 d),
//   cos_theta2 + 1 = (R + d - r1)(R + d + r1) / (2 R d);
// rounded, either can when d is within a few ulps of |R - r1| (DESIGN.md §2.4;
// tools/raise_search.py finds such configurations).  The shading walks skip
// the penumbra of spheres whose factor is 0, so these raises need their own
// check: World#high_lights' lit_area (world.rb:92-93) by its own walk
// (lit_area_raises), World#local_lights' (world.rb:76) inside the shadow walk
// (option exact_raises = 1: xr_setup / xr_band below; off by default, §2.4).
//
// penumbra_raises: the reference's own operations up to the two acos
// arguments (the bits of penumbra() and of rt_oracle.c's cover_area).
__device__ __forceinline__ bool penumbra_raises(V3 C, double R, V3 T, V3 lt, double radius) {
  const double t = vdot(vsub(C, T), lt) / vr2(lt);
  const V3 x1 = vadd(T, vsc(lt, t));
  const double r1 = radius * (vr(vsub(x1, T)) / vr(lt));
  const double d = vr(vsub(x1, C));
  if (d >= r1 + R) return false;                 // :38-39 (a NaN goes on, as in Ruby, and never raises)
  if (!(d > fabs(R - r1))) return false;         // :42
  const double c1 = (r1 * r1 + d * d - R * R) / (2.0 * r1 * d);
  const double c2 = (R * R + d * d - r1 * r1) / (2.0 * R * d);
  return c1 < -1.0 || c2 < -1.0;                 // ([x, 1.0].min < -1 iff x < -1)
}

// Option exact_raises inside the shadow walk of World#lit_area(T, L, radius)
// (DESIGN.md §2.4).  A sphere whose cover_area raises although its binary
// factor is 0 touches the surface of the double cone rho = radius |t| around
// the line Q(t) = T + t (L - T) (t = 1 at the light) in the cross-section
// through its own center: the cone's circle there (r1 = radius |t|) and the
// sphere's are internally tangent, d = |R - r1| (sphere.rb:42), up to a few
// binary64 ulps.  So
//   * at a leaf, a sphere can raise only if its distance rho from the line
//     lies within mg of |R - r1| (xr_band, on the pre-test's own float32
//     quantities: l = rho^2 |d|^2 up to 14 ulps of |oc|^2 |d|^2, q = (C - T).d,
//     r1 = radius |q| / |d|^2); those go to the binary64 test (penumbra_raises);
//   * a box that holds one meets the cone: a point P of the spheres' box within
//     radius |t| (+ mg) of Q(t) has, on each axis, |t| (|d_a| - radius) <= the
//     box's far side from T along that nappe's direction + mg, which bounds t
//     to [-tb, tf] (xr_setup), so the walk slab-tests the child boxes dilated by
//     radius max(tb, tf) + mg over t in [-tb, tf]; the segment's own boxes (t in
//     [0, 1], dilated by m S <= mg) are among them, so the covers' walk is
//     unchanged.
// The box dilation mg = 2e-5 S (1 + radius / |d|) is ten times the float32
// error of T, d and the box bounds (as the covers' m S, §2.2).  The band's own
// half-width is 32 float32 ulps of S (1 + radius / |d|): the float32 geometry
// (T, d, the centers and radii rounded, S >= |T|_1, |C|_1 + R) moves rho, R and
// r1 by less than 10 ulps of S (1 + radius / |d|) from the binary64 values whose
// tangency raises (to within a few binary64 ulps), and the rounding of l and of
// the squared bounds is covered separately (4e-6 (sq + hi^2) |d|^2 >= 14 ulps of
// sq |d|^2); 16-bit leaf records add their decoding error (q_err) to both.
// A ray for which these bounds are not finite walks every sphere in order and
// tests each one in binary64.
struct XrRay {
  float k;       // radius / |d|^2: r1 = k |q|
  float mb;      // the band's half-width (with the 16-bit records' decoding error)
  bool all;      // no valid float32 bound: every sphere goes to the binary64 test
};

__device__ __forceinline__ XrRay xr_ray(float Sx, float dd, double radius, float qerr) {
  XrRay x;
  // hardware reciprocal / rsqrt (1 ulp): the bounds carry far more margin
  const float rad = (float)radius, kn = rad * __builtin_amdgcn_rsqf(dd);
  x.k = rad * __builtin_amdgcn_rcpf(dd);
  x.mb = 32.0f * 5.9604645e-8f * Sx * (1.0f + kn) + (2.0f + kn) * qerr;
  x.all = !(__builtin_isfinite(x.k) && __builtin_isfinite(x.mb) && dd > 0.0f);
  return x;
}

// rho = |R - r1| within mb, for one sphere: l = |oc|^2 |d|^2 - (oc.d)^2 and sq =
// |oc|^2 as the pre-test computed them, R its radius.
__device__ __forceinline__ bool xr_band(const XrRay& x, float dd, float l, float q, float sq, float R) {
  const float t = fabsf(R - x.k * fabsf(q));
  const float lo = fmaxf(t - x.mb, 0.0f), hi = t + x.mb;
  const float e = 4e-6f * (sq + hi * hi) * dd;   // l's rounding (<= 14 ulps of sq dd) and the bounds'
  return x.all || (l >= lo * lo * dd - e && l <= hi * hi * dd + e);
}

// ----------------------------------------------------------------- the query
// One ordered walk over every object with ray (o, d), for every active lane.
//   EXTEND: World#intersect — nearest hit (strict <, YAML order) -> best/besti.
//   SHADOW: World#lit_area for light L (o = target T, d = L - T) -> total
//           (1 - ordered sum of cover areas; zero covers skipped: exact).
template <bool COUNT, typename SPH>
__device__ __forceinline__ void query(const SceneDev& S, SPH sph, bool ext, V3 o, V3 d,
                                      V3 L, double radius, double& best, int& besti, V3& bhit, bool& bin,
                                      double& total, uint32_t& err, unsigned long long* cnt, bool xr = false) {
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
  xr = xr && !ext;                                // exact_raises: the shadow walk's band check
  const XrRay xrr = xr_ray(Sx, dd, radius, 0.0f);
  const bool xall = xrr.all || !(__builtin_isfinite(Sx) && __builtin_isfinite(kline));
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
        uint32_t keep = 0, xkeep = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const float ocx = c[u].x - ox, ocy = c[u].y - oy, ocz = c[u].z - oz;
          const float s = __builtin_fmaf(ocx, ocx, __builtin_fmaf(ocy, ocy, ocz * ocz));
          const float q = __builtin_fmaf(ocx, dx, __builtin_fmaf(ocy, dy, ocz * dz));
          const float l = __builtin_fmaf(s, dd, -q * q);
          const bool miss_line = l > __builtin_fmaf(dd, c[u].w, kline);
          const bool behind = q < qneg && s > c[u].w + ms2;
          keep |= (miss_line || behind) ? 0u : (1u << u);
          if (xr && (xall || xr_band(xrr, dd, l, q, s, __builtin_amdgcn_sqrtf(c[u].w)))) xkeep |= 1u << u;
        }
        if (k0 + 4 > run.count) {
          keep &= (1u << (run.count - k0)) - 1u;
          xkeep &= (1u << (run.count - k0)) - 1u;
        }
        // exact_raises: the binary64 test of every sphere the band keeps (its cover_area's
        // acos arguments, whatever its factor; a factor-1 cover checks again below)
        while (xkeep && !(err & 0xffu)) {
          const int u = __builtin_ctz(xkeep);
          xkeep &= xkeep - 1;
          const RTX_CONST Sphere64& sp = sph64[run.rec0 + k0 + u];
          if (penumbra_raises(v3(sp.c[0], sp.c[1], sp.c[2]), sp.r, o, d, radius)) seterr(err, ERR_DOMAIN);
        }
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
  if (n >= COVER_K) {                               // full: keep the COVER_K smallest object indices
    ovf = true;
    if (!(obj < ci[(COVER_K - 1) * BS])) return;
    n = COVER_K - 1;                                // (the largest drops out)
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

// The float32 set-up of a walk's culls (§2.1 pre-test, §2.2 slab test), shared
// by the hierarchy walk and the flat leaf scan.
struct SlabRay {
  float ox, oy, oz, dx, dy, dz, dd, Sx, ms2, mS, kline, qneg;
  F2 pix, piy, piz, pax, pay, paz;   // packed operands of the slab test: {lo, hi} * {i, i} + {-a, -b} per axis
  bool fin;                          // false: a non-finite or zero ray, no float32 cull is valid
};

__device__ __forceinline__ SlabRay slab_setup(const SceneDev& S, V3 o, V3 d) {
  SlabRay s;
  s.ox = (float)o.x, s.oy = (float)o.y, s.oz = (float)o.z;
  s.dx = (float)d.x, s.dy = (float)d.y, s.dz = (float)d.z;
  s.dd = __builtin_fmaf(s.dx, s.dx, __builtin_fmaf(s.dy, s.dy, s.dz * s.dz));
  s.Sx = fabsf(s.ox) + fabsf(s.oy) + fabsf(s.oz) + S.sph_scale;
  s.ms2 = CULL_M * s.Sx * s.Sx;
  s.mS = CULL_M * s.Sx;
  s.kline = s.dd * s.ms2;
  s.qneg = -CULL_M * s.Sx * sqrtf(s.dd);
  // slab set-up: reciprocal direction and the dilated origin terms
  const float l1 = fabsf(s.dx) + fabsf(s.dy) + fabsf(s.dz);
  const float tiny = 1e-20f * l1;
  const float ex = fabsf(s.dx) < tiny ? copysignf(tiny, s.dx) : s.dx;
  const float ey = fabsf(s.dy) < tiny ? copysignf(tiny, s.dy) : s.dy;
  const float ez = fabsf(s.dz) < tiny ? copysignf(tiny, s.dz) : s.dz;
  const float ix = 1.0f / ex, iy = 1.0f / ey, iz = 1.0f / ez;
  const float ax = (s.ox + s.mS) * ix, ay = (s.oy + s.mS) * iy, az = (s.oz + s.mS) * iz;   // lo - mS side
  const float bx = (s.ox - s.mS) * ix, by = (s.oy - s.mS) * iy, bz = (s.oz - s.mS) * iz;   // hi + mS side
  s.pix = F2{ix, ix}, s.piy = F2{iy, iy}, s.piz = F2{iz, iz};
  s.pax = F2{-ax, -bx}, s.pay = F2{-ay, -by}, s.paz = F2{-az, -bz};
  s.fin = __builtin_isfinite(s.dd) && __builtin_isfinite(s.Sx) && l1 > 0.0f && __builtin_isfinite(ix) &&
          __builtin_isfinite(iy) && __builtin_isfinite(iz);
  return s;
}

// Entry distance of child box k of `node` if the ray may want it (the slab test
// of the box dilated by m*S, §2.2, against the far bound thi), else +inf.
template <typename NR>
__device__ __forceinline__ float slab_key(const NR& node, int k, const SlabRay& s, float tlo, float thi) {
  // {t0, t1} per axis in one v_pk_fma_f32 each: the same fused FP32 operations as
  // fmaf(lo, i, -a), fmaf(hi, i, -b)
  const F2 tx = __builtin_elementwise_fma(*reinterpret_cast<const F2*>(&node.lh[0][k][0]), s.pix, s.pax);
  const F2 ty = __builtin_elementwise_fma(*reinterpret_cast<const F2*>(&node.lh[1][k][0]), s.piy, s.pay);
  const F2 tz = __builtin_elementwise_fma(*reinterpret_cast<const F2*>(&node.lh[2][k][0]), s.piz, s.paz);
  const float t0x = tx.x, t1x = tx.y, t0y = ty.x, t1y = ty.y, t0z = tz.x, t1z = tz.y;
  const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
  const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
  // empty slots hold a box at (3e38, 3e38, 3e38): never wanted by a finite ray
  return (tn <= tf && tf >= tlo && tn <= thi) ? tn : __builtin_inff();
}

// exact_raises (above): the cone's extent in t over the spheres' box, for each
// nappe.  A point Q(t) = T + t d within radius |t| + mg of the box on axis a has
// |t| (|d_a| - radius) <= (the box's far side from T along the nappe's
// direction on a) + mg, so for every axis with |d_a| > radius: t <= tf going
// towards the light, -t <= tb going away from it.  The child boxes are then
// slab-tested dilated by radius max(tb, tf) + mg over t in [-tb, tf], which
// holds the segment's own boxes (t in [0, 1], dilated by m S <= mg).  ok false
// when no finite bound exists (the caller walks every sphere).
__device__ __forceinline__ SlabRay xr_setup(const SceneDev& S, const SlabRay& s0, double radius, float& tlo,
                                            float& thi, bool& ok) {
  SlabRay s = s0;
  ok = false;
  if (!s.fin) return s;
  const float rad = (float)radius;
  const float mg = CULL_M * s.Sx * (1.0f + rad * __builtin_amdgcn_rsqf(s.dd));   // (node boxes are exact: no decoding error)
  float tf = __builtin_inff(), tb = __builtin_inff();
  const float o[3] = {s.ox, s.oy, s.oz}, dv[3] = {s.dx, s.dy, s.dz};
#pragma unroll
  for (int a = 0; a < 3; a++) {
    const float ad = fabsf(dv[a]), den = ad - rad;
    if (!(den > 1e-5f * (ad + rad))) continue;
    const float iden = __builtin_amdgcn_rcpf(den);                     // (1 ulp; the bounds are widened below)
    const float up = (S.root_c[a] + S.root_h[a] + mg - o[a]) * iden;   // to the box's high side
    const float dn = (o[a] - (S.root_c[a] - S.root_h[a]) + mg) * iden; // to its low side
    tf = fminf(tf, dv[a] > 0.0f ? up : dn);
    tb = fminf(tb, dv[a] > 0.0f ? dn : up);
  }
  tf = fmaxf(tf, 0.0f) * (1.0f + 1e-5f);
  tb = fmaxf(tb, 0.0f) * (1.0f + 1e-5f);
  if (!(tf < 1e30f && tb < 1e30f)) return s;
  const float r = __builtin_fmaf(rad, fmaxf(tf, tb), mg) * (1.0f + 1e-5f);   // >= m S: the covers' dilation too
  const float ix = s.pix.x, iy = s.piy.x, iz = s.piz.x;
  s.pax = F2{-((s.ox + r) * ix), -((s.ox - r) * ix)};
  s.pay = F2{-((s.oy + r) * iy), -((s.oy - r) * iy)};
  s.paz = F2{-((s.oz + r) * iz), -((s.oz - r) * iz)};
  tlo = -tb;
  thi = tf;
  ok = __builtin_isfinite(r);
  return s;
}

// Planes and boxes first, in run order (their order does not matter either).
template <int BS>
__device__ __forceinline__ void walk_planes_boxes(const SceneDev& S, bool ext, V3 o, V3 d, V3 L, double r,
                                                  double& best, int& besti, V3& bhit, bool& bin, float& thi, int* ci,
                                                  double* cv, int& ncov, bool& ovf, int after = -1) {
  const RTX_CONST Run* runs = cptr(S.runs);
  const int n_runs = uni(S.n_runs);
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
      } else if (obj0 + k > after && vdot(vsub(hit, L), vsub(o, L)) > 0) {
        push_cover<BS>(ci, cv, ncov, ovf, obj0 + k, 1.0);
      }
    }
  }
}

// A leaf's 4 pre-test records as {x0..x3}, {y0..y3}, {z0..z3}, {R^2 0..3}:
// float32 records (LDS or global), or the 16-bit records of SPH_BVH_QLDS
// decoded with the host's operations (quantize_leaves in rtx_capi.cpp: a
// decoded ball holds the true one).
struct QLeaf {
  const uint4* q;            // 2 per leaf
  float ox, oy, oz, sx, sy, sz, rs;
};

// SPH_BVH_QLDS's 16-bit traversal stacks (stride BS entries): lane l of a wave
// owns the low (l < 32) or high half of dword l mod 32 of each 128-B row, so
// each 32-lane group of a stack access meets 32 banks.
__device__ __forceinline__ int16_t* qstack(char* lds, const KParams& p) {
  const int t = (int)threadIdx.x;
  return reinterpret_cast<int16_t*>(lds + p.lds_stack) + (t & ~63) + ((t & 31) << 1) + ((t >> 5) & 1);
}

__device__ __forceinline__ void leaf_records(const float4* l, int v, float4& cx, float4& cy, float4& cz, float4& cw) {
  const int slot0 = (v >> 2) * BVH_LEAF;
  cx = l[slot0], cy = l[slot0 + 1], cz = l[slot0 + 2], cw = l[slot0 + 3];
}

__device__ __forceinline__ void leaf_records(const QLeaf& l, int v, float4& cx, float4& cy, float4& cz, float4& cw) {
  const uint4 a = l.q[(v >> 2) * 2], b = l.q[(v >> 2) * 2 + 1];
  auto lo = [](uint32_t w) { return (float)(w & 0xffffu); };
  auto hi = [](uint32_t w) { return (float)(w >> 16); };
  cx = make_float4(__builtin_fmaf(lo(a.x), l.sx, l.ox), __builtin_fmaf(hi(a.x), l.sx, l.ox),
                   __builtin_fmaf(lo(a.y), l.sx, l.ox), __builtin_fmaf(hi(a.y), l.sx, l.ox));
  cy = make_float4(__builtin_fmaf(lo(a.z), l.sy, l.oy), __builtin_fmaf(hi(a.z), l.sy, l.oy),
                   __builtin_fmaf(lo(a.w), l.sy, l.oy), __builtin_fmaf(hi(a.w), l.sy, l.oy));
  cz = make_float4(__builtin_fmaf(lo(b.x), l.sz, l.oz), __builtin_fmaf(hi(b.x), l.sz, l.oz),
                   __builtin_fmaf(lo(b.y), l.sz, l.oz), __builtin_fmaf(hi(b.y), l.sz, l.oz));
  const float r0 = lo(b.z) * l.rs, r1 = hi(b.z) * l.rs, r2 = lo(b.w) * l.rs, r3 = hi(b.w) * l.rs;
  cw = make_float4(r0 * r0, r1 * r1, r2 * r2, r3 * r3);
}

// One leaf (reference lf < 0): the §2.1 pre-test of its spheres, the exact
// test for those not ruled out, then the nearest-hit update or the cover list.
template <int BS, typename LP, typename XP, typename OP>
__device__ __forceinline__ void walk_leaf(int lf, LP leaf4, XP x64, OP xobj, const SlabRay& s, bool ext, V3 o, V3 d,
                                          V3 dn, double r, double r2, V3 L, double radius, double& best, int& besti,
                                          V3& bhit, bool& bin, float& thi, uint32_t& err, int* ci, double* cv,
                                          int& ncov, bool& ovf, bool xr, float qerr, int after = -1) {
  const int v = ~lf;
  const int slot0 = (v >> 2) * BVH_LEAF;
  const int cnt = (v & 3) + 1;
  // the pre-test of §2.1 on two spheres per packed FP32 instruction (the same
  // operations as the per-sphere form in query())
  float4 cx, cy, cz, cw;
  leaf_records(leaf4, v, cx, cy, cz, cw);
  uint32_t keep = 0, xkeep = 0;
  const XrRay xrr = xr ? xr_ray(s.Sx, s.dd, radius, qerr) : XrRay{};
  const F2 po = {s.ox, s.ox}, poy = {s.oy, s.oy}, poz = {s.oz, s.oz};
  const F2 pdx = {s.dx, s.dx}, pdy = {s.dy, s.dy}, pdz = {s.dz, s.dz}, pdd = {s.dd, s.dd};
  const F2 pkl = {s.kline, s.kline}, pms = {s.ms2, s.ms2};
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const F2 X = h ? F2{cx.z, cx.w} : F2{cx.x, cx.y}, Y = h ? F2{cy.z, cy.w} : F2{cy.x, cy.y};
    const F2 Z = h ? F2{cz.z, cz.w} : F2{cz.x, cz.y}, Wr = h ? F2{cw.z, cw.w} : F2{cw.x, cw.y};
    const F2 ocx = X - po, ocy = Y - poy, ocz = Z - poz;
    const F2 sq = __builtin_elementwise_fma(ocx, ocx, __builtin_elementwise_fma(ocy, ocy, ocz * ocz));
    const F2 q = __builtin_elementwise_fma(ocx, pdx, __builtin_elementwise_fma(ocy, pdy, ocz * pdz));
    const F2 l = __builtin_elementwise_fma(sq, pdd, -(q * q));
    const F2 rr = __builtin_elementwise_fma(pdd, Wr, pkl);
    const F2 wm = Wr + pms;
    const bool m0 = l.x > rr.x || (q.x < s.qneg && sq.x > wm.x);   // misses the line, or wholly behind
    const bool m1 = l.y > rr.y || (q.y < s.qneg && sq.y > wm.y);
    keep |= (m0 ? 0u : 1u << (2 * h)) | (m1 ? 0u : 2u << (2 * h));
    if (xr)                                         // exact_raises: rho within mg of |R - r1|
      xkeep |= (xr_band(xrr, s.dd, l.x, q.x, sq.x, __builtin_amdgcn_sqrtf(Wr.x)) ? 1u << (2 * h) : 0u) |
               (xr_band(xrr, s.dd, l.y, q.y, sq.y, __builtin_amdgcn_sqrtf(Wr.y)) ? 2u << (2 * h) : 0u);
  }
  keep &= (1u << cnt) - 1u;
  xkeep &= (1u << cnt) - 1u;
  while (xkeep && !(err & 0xffu)) {                 // their cover_area's acos arguments in binary64
    const int u = __builtin_ctz(xkeep);
    xkeep &= xkeep - 1;
    const Sphere64 sp64 = x64[slot0 + u];
    if (penumbra_raises(v3(sp64.c[0], sp64.c[1], sp64.c[2]), sp64.r, o, d, radius)) seterr(err, ERR_DOMAIN);
  }
  while (keep) {
    const int u = __builtin_ctz(keep);
    keep &= keep - 1;
    const Sphere64 sp64 = x64[slot0 + u];
    const V3 C = v3(sp64.c[0], sp64.c[1], sp64.c[2]);
    V3 hit;
    bool in;
    if (!sphere_exact(C, sp64.r, o, d, dn, r2, hit, in)) continue;
    const int obj = xobj[slot0 + u];
    if (!ext && obj <= after) continue;              // (a later pass of query_lbuf's ordered cover sum)
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

// World#lit_area's result from a shadow walk's ordered cover list.
template <int BS>
__device__ __forceinline__ void walk_covers(const SceneDev& S, V3 o, V3 d, V3 L, double radius, double& best,
                                            int& besti, V3& bhit, bool& bin, double& total, uint32_t& err,
                                            const double* cv, int ncov, bool ovf, bool xr) {
  total = 1.0;
#ifndef RTX_DIAG_NOOVF
#define RTX_DIAG_NOOVF 0           // diagnostic builds only (wrong results where a shadow ray meets > COVER_K covers)
#endif
  if (ovf && !RTX_DIAG_NOOVF) {
    // more than COVER_K non-zero covers: the ordered linear walk (rare)
    query<false>(S, cptr(S.sph32), false, o, d, L, radius, best, besti, bhit, bin, total, err, nullptr, xr);
  } else {
    for (int k = 0; k < ncov; k++) total -= cv[k * BS];
  }
}

// The light buffer's cube-map cell of direction v (float32):
// face 2a + (v_a < 0) of the dominant axis a, cell (floor((v_b / |v_a| + 1) n
// / 2), likewise for c), b = a + 1, c = a + 2 (mod 3).  -1: no usable cell.
__device__ __forceinline__ int lbuf_cell(float vx, float vy, float vz, int n, int& face, int& i, int& j) {
  const float ax = fabsf(vx), ay = fabsf(vy), az = fabsf(vz);
  float m, fs, ft;
  if (ax >= ay && ax >= az) {
    face = vx < 0.0f ? 1 : 0, m = ax, fs = vy, ft = vz;
  } else if (ay >= az) {
    face = vy < 0.0f ? 3 : 2, m = ay, fs = vz, ft = vx;
  } else {
    face = vz < 0.0f ? 5 : 4, m = az, fs = vx, ft = vy;
  }
  if (!(m > 0.0f)) return -1;
  const float h = 0.5f * (float)n / m;
  i = min(max((int)floorf(__builtin_fmaf(fs, h, 0.5f * (float)n)), 0), n - 1);
  j = min(max((int)floorf(__builtin_fmaf(ft, h, 0.5f * (float)n)), 0), n - 1);
  return (face * n + i) * n + j;
}

// exact_raises through the raise buffer: the band test
// (xr_band) of every sphere of one leaf, whatever its factor, and the binary64
// test (penumbra_raises) of those it keeps.
template <typename LP, typename XP>
__device__ __forceinline__ void leaf_raises(int lf, LP leaf4, XP x64, const SlabRay& s, const XrRay& xrr, V3 o, V3 d,
                                            double radius, uint32_t& err) {
  const int v = ~lf;
  const int slot0 = (v >> 2) * BVH_LEAF;
  const int cnt = (v & 3) + 1;
  float4 cx, cy, cz, cw;
  leaf_records(leaf4, v, cx, cy, cz, cw);
  const F2 po = {s.ox, s.ox}, poy = {s.oy, s.oy}, poz = {s.oz, s.oz};
  const F2 pdx = {s.dx, s.dx}, pdy = {s.dy, s.dy}, pdz = {s.dz, s.dz}, pdd = {s.dd, s.dd};
  uint32_t xkeep = 0;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const F2 X = h ? F2{cx.z, cx.w} : F2{cx.x, cx.y}, Y = h ? F2{cy.z, cy.w} : F2{cy.x, cy.y};
    const F2 Z = h ? F2{cz.z, cz.w} : F2{cz.x, cz.y}, Wr = h ? F2{cw.z, cw.w} : F2{cw.x, cw.y};
    const F2 ocx = X - po, ocy = Y - poy, ocz = Z - poz;
    const F2 sq = __builtin_elementwise_fma(ocx, ocx, __builtin_elementwise_fma(ocy, ocy, ocz * ocz));
    const F2 q = __builtin_elementwise_fma(ocx, pdx, __builtin_elementwise_fma(ocy, pdy, ocz * pdz));
    const F2 l = __builtin_elementwise_fma(sq, pdd, -(q * q));
    xkeep |= (xr_band(xrr, s.dd, l.x, q.x, sq.x, __builtin_amdgcn_sqrtf(Wr.x)) ? 1u << (2 * h) : 0u) |
             (xr_band(xrr, s.dd, l.y, q.y, sq.y, __builtin_amdgcn_sqrtf(Wr.y)) ? 2u << (2 * h) : 0u);
  }
  xkeep &= (1u << cnt) - 1u;
  while (xkeep && !(err & 0xffu)) {
    const int u = __builtin_ctz(xkeep);
    xkeep &= xkeep - 1;
    const Sphere64 sp64 = x64[slot0 + u];
    if (penumbra_raises(v3(sp64.c[0], sp64.c[1], sp64.c[2]), sp64.r, o, d, radius)) seterr(err, ERR_DOMAIN);
  }
}

// One sphere's pre-test record (slot = 4 leaf + u): float32 records (LDS or
// global) or the 16-bit records of SPH_BVH_QLDS, decoded as leaf_records does.
__device__ __forceinline__ void sphere_record(const float4* l, int slot, float& cx, float& cy, float& cz, float& w) {
  const float* f = reinterpret_cast<const float*>(l + (slot >> 2) * BVH_LEAF);
  const int u = slot & 3;
  cx = f[u], cy = f[4 + u], cz = f[8 + u], w = f[12 + u];
}
__device__ __forceinline__ void sphere_record(const QLeaf& l, int slot, float& cx, float& cy, float& cz, float& w) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(l.q + (slot >> 2) * 2);
  const int u = slot & 3, sh = (u & 1) * 16, k = u >> 1;
  auto f16 = [sh](uint32_t x) { return (float)((x >> sh) & 0xffffu); };
  cx = __builtin_fmaf(f16(q[k]), l.sx, l.ox);
  cy = __builtin_fmaf(f16(q[2 + k]), l.sy, l.oy);
  cz = __builtin_fmaf(f16(q[4 + k]), l.sz, l.oz);
  const float r = f16(q[6 + k]) * l.rs;
  w = r * r;
}

// exact_raises for one sphere of the raise buffer's per-sphere lists (slot):
// the band test and, when it keeps the sphere, the binary64 test.
template <typename LP, typename XP>
__device__ __forceinline__ void sphere_raises(int slot, LP leaf4, XP x64, const SlabRay& s, const XrRay& xrr, V3 o,
                                              V3 d, double radius, uint32_t& err) {
  float cx, cy, cz, w;
  sphere_record(leaf4, slot, cx, cy, cz, w);
  const float ocx = cx - s.ox, ocy = cy - s.oy, ocz = cz - s.oz;
  const float sq = __builtin_fmaf(ocx, ocx, __builtin_fmaf(ocy, ocy, ocz * ocz));
  const float q = __builtin_fmaf(ocx, s.dx, __builtin_fmaf(ocy, s.dy, ocz * s.dz));
  const float l = __builtin_fmaf(sq, s.dd, -(q * q));
  if (!xr_band(xrr, s.dd, l, q, sq, __builtin_amdgcn_sqrtf(w))) return;
  const Sphere64 sp64 = x64[slot];
  if (penumbra_raises(v3(sp64.c[0], sp64.c[1], sp64.c[2]), sp64.r, o, d, radius)) seterr(err, ERR_DOMAIN);
}

// The raise buffer's reach for a shadow ray (o = T, d = L - T, s its float32
// set-up): ql = 16 log2(l / floor) = 8 (log2 |d|^2 - log2 floor^2), first as
// a cheap lower bound qa from the bits of |d|^2 (a float's bits / 2^23 - 127
// is log2 x less the mantissa's log2(1 + f) - f, which lies in [0, 0.0861]:
// qa <= ql <= qa + QA_SLACK); the exact value (raise_rq) only when a gate
// opens.  false when l lies below the light's floor or ql may exceed 254: the
// caller walks the hierarchy.  f2, lf2: the light's floor^2 (rounded up) and
// log2 floor^2 (LightDev: with the light's other data, not behind a load of
// their own).  gates: this light's gate block (16-bit words: floor^2 and log2
// floor^2 as float bits, 4 of padding, a gate per raise-buffer cell), in LDS
// or global memory.
constexpr float QA_SLACK = 0.7f;             // 8 x 0.0861 + the int-to-float rounding of the bits
__device__ __forceinline__ bool raise_qa(float f2, float lf2, const SlabRay& s, float& qa) {
  qa = 8.0f * (__builtin_fmaf((float)__float_as_int(s.dd), 1.0f / 8388608.0f, -127.0f) - lf2);
  // l >= floor (1 + 1e-4): |d|^2 >= floor^2 (1 + 2.1e-4), floor^2 rounded up
  return s.dd >= f2 * (1.0f + 2.1e-4f) && qa + QA_SLACK <= 254.0f;
}
__device__ __forceinline__ float raise_rq(float lf2, const SlabRay& s) { return 8.0f * (__log2f(s.dd) - lf2); }

// The raise buffer's lists (rtx_bvh_build.h build_raise_buffer): B2 and B1 at
// the parent (raise-buffer) cell of the light buffer's cell (face, i, j) of
// -d, M at the parent of its opposite cell (face ^ 1, n - 1 - i, n - 1 - j:
// the cell of d, or a neighbour sharing the boundary d lies on, which the
// cells' slack covers), each read while its entries' thresholds admit ql and
// only when the cell's gate opens; each listed leaf gets leaf_raises (each
// listed sphere sphere_raises, in the per-sphere lists of larger scenes).  (The
// light buffer's own cell, walked with walk_leaf's band test, holds regime A.)
template <typename LP, typename XP>
__device__ __forceinline__ void raise_lists(const SceneDev& S, int light, const uint16_t* gates, LP leaf4, XP x64,
                                            const SlabRay& s, const XrRay& xrr, V3 o, V3 d, double radius, int face,
                                            int i, int j, float qa, float lf2, uint32_t& err) {
  const int nu = S.lbuf_n, nc = S.rbuf_n, cells = 6 * nc * nc;
  // parent cells: i / m as (int)((i + 0.5) / m) in float32 (no integer division: i, m < 2^12, so
  // (i + 0.5) / m lies at least 0.5 / m from an integer, far beyond the rounding)
  const float im = S.rbuf_inv_m;
  auto up = [im](int k) { return (int)(((float)k + 0.5f) * im); };
  const int pc = (face * nc + up(i)) * nc + up(j), mc = ((face ^ 1) * nc + up(nu - 1 - i)) * nc + up(nu - 1 - j);
  // the gates (rtx_bvh_build.h gate_word: 5-bit fields in GATE_UNIT q units; 31 in g2 / gm: always open),
  // tested with ql's bounds [qa, qa + QA_SLACK]; scenes with per-sphere lists (C4) skip them: their
  // gates open for nine walks in ten, and the gate read would add a global round trip
  bool o2 = true, o1 = true, om = true;
  if (!S.rbuf_sphere) {
    const uint32_t gp = gates[8 + pc], gm = gates[8 + mc];
    const uint32_t g2 = gp & 31u, g1 = (gp >> 5) & 31u, gmm = (gm >> 10) & 31u;
    constexpr float U = (float)GATE_UNIT;
    o2 = g2 == 31u || qa <= U * (float)g2, o1 = qa + QA_SLACK >= U * (float)g1, om = gmm == 31u || qa <= U * (float)gmm;
    if (!(o2 || o1 || om)) return;
  }
  const float ql = raise_rq(lf2, s);
  const uint32_t* blk = S.rbuf + (size_t)light * S.rbuf_stride;
  const uint32_t* off = blk + 2;
  const uint32_t* ent = blk + rbuf_head(cells);
  // the open lists' ranges, loaded together; then the first four entries of
  // every list at once, later ones four at a time, one 16-byte load each (every
  // list starts at a multiple of 4 entries; global memory: a round trip per
  // batch, not per entry or per list)
  uint32_t ka[3], kb[3];
#pragma unroll
  for (int t = 0; t < 3; t++) {
    const bool on = t == 0 ? o2 : t == 1 ? o1 : om;
    const uint32_t* oc = off + t * (cells + 1) + (t < 2 ? pc : mc);
    ka[t] = on ? oc[0] : 0u;
    kb[t] = on ? oc[1] : 0u;
  }
  // (16-byte loads in the kernels of the larger scenes, whose lists are read on most walks: C4 283.4 ->
  // 282.6 ms, r11ai; C2's gated lists keep word loads, its kernels measured slower with them)
  constexpr bool V4 = std::is_same<LP, QLeaf>::value;
  uint32_t pre[3][4];
#pragma unroll
  for (int t = 0; t < 3; t++) {
    if (V4) {
      const uint4 v = ka[t] < kb[t] ? *reinterpret_cast<const uint4*>(ent + ka[t]) : make_uint4(0u, 0u, 0u, 0u);
      pre[t][0] = v.x, pre[t][1] = v.y, pre[t][2] = v.z, pre[t][3] = v.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; u++) pre[t][u] = ka[t] + u < kb[t] ? ent[ka[t] + u] : 0u;
    }
  }
#pragma unroll 1
  for (int t = 0; t < 3; t++) {
    uint32_t k = ka[t];
    const uint32_t k1 = kb[t];
    uint32_t e0 = t == 0 ? pre[0][0] : t == 1 ? pre[1][0] : pre[2][0];
    uint32_t e1 = t == 0 ? pre[0][1] : t == 1 ? pre[1][1] : pre[2][1];
    uint32_t e2 = t == 0 ? pre[0][2] : t == 1 ? pre[1][2] : pre[2][2];
    uint32_t e3 = t == 0 ? pre[0][3] : t == 1 ? pre[1][3] : pre[2][3];
    bool go = true;
    while (go && k < k1 && !(err & 0xffu)) {
      const uint32_t n = k1 - k < 4u ? k1 - k : 4u;
      for (uint32_t u = 0; u < n; u++) {
        const uint32_t e = e0;
        e0 = e1, e1 = e2, e2 = e3;
        const float q = (float)(e & 255u);      // the sort key (the entry's other bound is not tested:
        if (t == 1 ? q > ql : q < ql) {         //  r11s, C4 294 -> 300 ms with the test)
          go = false;                           // (sorted: the rest of the list is not needed either)
          break;
        }
        if (S.rbuf_sphere) sphere_raises((int)(e >> 16), leaf4, x64, s, xrr, o, d, radius, err);
        else leaf_raises((int)(int16_t)(e >> 16), leaf4, x64, s, xrr, o, d, radius, err);
      }
      k += 4;
      if (go && k < k1) {
        if (V4) {
          const uint4 v = *reinterpret_cast<const uint4*>(ent + k);
          e0 = v.x, e1 = v.y, e2 = v.z, e3 = v.w;
        } else {
          e0 = ent[k], e1 = k + 1 < k1 ? ent[k + 1] : 0u, e2 = k + 2 < k1 ? ent[k + 2] : 0u,
          e3 = k + 3 < k1 ? ent[k + 3] : 0u;
        }
      }
    }
  }
}

// World#lit_area's walk through the light buffer (SceneDev::
// lbuf; lb: this light's block): planes and boxes first, then only the leaves
// listed in the cell of the direction from the light towards o, each with the
// hierarchy walk's own leaf test (walk_leaf), then the ordered cover sum.  Every
// sphere that covers o lies in a listed leaf (the cell holds the direction of
// its crossing point as seen from the light), and the covers are summed in
// object order, so the result is the hierarchy walk's.  With xr (exact_raises)
// the listed leaves also get the raise band test, and the raise buffer's lists
// the rest of World#lit_area's raise region (raise_lists; gates: this light's
// gate block).  false: no usable cell (a non-finite or zero
// ray), or (xr) a target nearer the light than the raise buffer's floor; the
// caller walks the hierarchy.
template <int BS, typename LP, typename XP, typename OP>
__device__ __forceinline__ bool query_lbuf(const SceneDev& S, const uint16_t* lb, LP leaf4, XP x64, OP xobj, int* ci,
                                           double* cv, V3 o, V3 d, V3 L, double radius, double& best, int& besti,
                                           V3& bhit, bool& bin, double& total, uint32_t& err, bool xr = false,
                                           int light = 0, const uint16_t* gates = nullptr) {
  const SlabRay s = slab_setup(S, o, d);
  if (!s.fin) return false;
  // the cube-map cell of v = o - L = -d
  const int n = S.lbuf_n;
  int face, i, j;
  const int cell = lbuf_cell(-s.dx, -s.dy, -s.dz, n, face, i, j);
  if (cell < 0) return false;
  // exact_raises: a light of radius 0 never raises (r1 = 0); without the raise
  // buffer, or below its floor, the hierarchy walk checks the cone
  xr = xr && radius > 0.0;
  float qa = 0.0f;
  const RTX_CONST LightDev& LD = cptr(S.light)[light];
  const float f2 = LD.raise_f2, lf2 = LD.raise_lf2;
  if (xr && !(S.rbuf && gates && raise_qa(f2, lf2, s, qa))) return false;
  const int k0 = lb[cell], k1 = lb[cell + 1];
  const uint16_t* ent = lb + 6 * n * n + 1;
  const double r = vr(d);
  const double r2 = r * r;                        // front.r2
  V3 dn = d;
  if (r != 0) dn = v3(d.x / r, d.y / r, d.z / r); // front.normalize (the hierarchy walk's bits)
  float thi = 1.0f + 1e-5f + s.mS / (float)r;
  int ncov = 0;
  bool ovf = false;
  constexpr bool Q16 = std::is_same<LP, QLeaf>::value;   // 16-bit leaf records: their decoding error
  const float qerr = Q16 ? S.q_err : 0.0f;
#ifndef RTX_DIAG_XR_NOBAND
#define RTX_DIAG_XR_NOBAND 0       // diagnostic builds only (wrong results on raise inputs)
#endif
#ifndef RTX_DIAG_XR_NOLISTS
#define RTX_DIAG_XR_NOLISTS 0      // diagnostic builds only (wrong results on raise inputs)
#endif
  walk_planes_boxes<BS>(S, false, o, d, L, r, best, besti, bhit, bin, thi, ci, cv, ncov, ovf);
  for (int k = k0; k < k1; k++)
    walk_leaf<BS>((int)(int16_t)ent[k], leaf4, x64, xobj, s, false, o, d, dn, r, r2, L, radius, best, besti, bhit,
                  bin, thi, err, ci, cv, ncov, ovf, xr && !RTX_DIAG_XR_NOBAND, qerr);
  if (xr && !RTX_DIAG_XR_NOLISTS)
    raise_lists(S, light, gates, leaf4, x64, s, xr_ray(s.Sx, s.dd, radius, qerr), o, d, radius, face, i, j, qa, lf2,
                err);
  // More than COVER_K covers: the list holds the COVER_K smallest object indices (push_cover).  They
  // are subtracted, and the cell is walked again for the next COVER_K above the last, until one pass
  // fits: the covers in object order, as the ordered linear walk sums them (which the other walks
  // repeat instead).  The band tests above and the raise buffer's lists have checked every factor-0
  // raise, so the later passes do not test the band.
#ifndef RTX_OVF_XR
#define RTX_OVF_XR 0
#endif
#ifndef RTX_OVF_PASSES
#define RTX_OVF_PASSES 1
#endif
  if (ovf && RTX_OVF_PASSES && !RTX_DIAG_NOOVF) {
    total = 1.0;
    while (true) {
      for (int k = 0; k < ncov; k++) total -= cv[k * BS];
      if (!ovf) break;
      const int after = ci[(ncov - 1) * BS];
      ncov = 0;
      ovf = false;
      walk_planes_boxes<BS>(S, false, o, d, L, r, best, besti, bhit, bin, thi, ci, cv, ncov, ovf, after);
      for (int k = k0; k < k1; k++)
        walk_leaf<BS>((int)(int16_t)ent[k], leaf4, x64, xobj, s, false, o, d, dn, r, r2, L, radius, best, besti, bhit,
                      bin, thi, err, ci, cv, ncov, ovf, false, qerr, after);
    }
    return true;
  }
  walk_covers<BS>(S, o, d, L, radius, best, besti, bhit, bin, total, err, cv, ncov, ovf, xr && RTX_OVF_XR);
  return true;
}

// Does World#lit_area(T, L, radius) raise (Math.acos in a cover_area,
// DESIGN.md §2.4)?  Through the light buffer's cell of T - L (its leaves' band
// test: regime A) and the raise buffer's lists, global memory, float32 leaf
// records (S.bvh_sph32): the highlight check of k_hl_raise on large scenes.
// -1: the buffers cannot serve this target (below the floor, a degenerate
// ray): the caller walks the hierarchy (lit_area_raises).
__device__ __forceinline__ int lit_area_raises_lbuf(const SceneDev& S, int light, V3 T, V3 L, double radius) {
  if (!(radius > 0.0) || S.n_sphere == 0) return 0;   // as lit_area_raises
  const V3 d = vsub(L, T);
  const SlabRay s = slab_setup(S, T, d);
  if (!s.fin) return -1;
  int face, i, j;
  const int n = S.lbuf_n;
  const int cell = lbuf_cell(-s.dx, -s.dy, -s.dz, n, face, i, j);
  if (cell < 0) return -1;
  const uint16_t* gates = S.rgate + (size_t)light * S.rgate_stride;
  float qa;
  const RTX_CONST LightDev& LD = cptr(S.light)[light];
  if (!raise_qa(LD.raise_f2, LD.raise_lf2, s, qa)) return -1;
  const uint16_t* lb = S.lbuf + (size_t)light * S.lbuf_stride;
  const int k0 = lb[cell], k1 = lb[cell + 1];
  const uint16_t* ent = lb + 6 * n * n + 1;
  const float4* leaf4 = reinterpret_cast<const float4*>(S.bvh_sph32);
  const XrRay xrr = xr_ray(s.Sx, s.dd, radius, 0.0f);
  uint32_t err = 0;
  for (int k = k0; k < k1 && !err; k++) leaf_raises((int)(int16_t)ent[k], leaf4, S.bvh_sph64, s, xrr, T, d, radius, err);
  if (!err) raise_lists(S, light, gates, leaf4, S.bvh_sph64, s, xrr, T, d, radius, face, i, j, qa, LD.raise_lf2, err);
  return err ? 1 : 0;
}

// Resumable: a lane whose walk is still running when fewer than `postpone`
// lanes of its wave are is postponed (returns false) with its walk in
// ref / sp (+ the LDS stack) / ncov / ovf (+ the LDS cover list) and best /
// besti / bhit / bin, and continues where it stopped at the next call with
// resume = true; meanwhile the wave's other lanes shade and start new
// queries instead of idling.  Every lane visits the same nodes and leaves in
// the same order either way, so the result is unchanged.
template <int BS, bool PP, typename NP, typename LP, typename XP, typename OP, typename SP>
__device__ __forceinline__ bool query_bvh(const SceneDev& S, NP nodes, LP leaf4, XP x64, OP xobj, SP stk, int* ci,
                                          double* cv,
                                          bool ext, V3 o, V3 d, V3 L, double radius, double& best, int& besti,
                                          V3& bhit, bool& bin, double& total, uint32_t& err, int& ref, int& sp,
                                          int& ncov, bool& ovf, bool resume, int postpone, bool xr = false) {
  const double r = vr(d);
  const double r2 = r * r;                        // front.r2
  V3 dn = d;
  if (r != 0) dn = v3(d.x / r, d.y / r, d.z / r); // front.normalize (same bits as the walk)
  const SlabRay s0 = slab_setup(S, o, d);
  xr = xr && !ext;                                // exact_raises: the shadow walk also checks the raises
  constexpr bool Q16 = std::is_same<LP, QLeaf>::value;   // 16-bit leaf records: their decoding error
  const float rf = (float)r;
  // ray parameter range: EXTEND [0, the current best hit], SHADOW [0, the light]; with
  // exact_raises the cone bound [-tm, tm] (xr_setup), the child boxes dilated to its radius
  float tlo = 0.0f;
  float thi = ext ? (float)(best / r * (1.0 + 1e-6)) : 1.0f + 1e-5f + s0.mS / rf;
  bool xok = true;
  const SlabRay s = xr ? xr_setup(S, s0, radius, tlo, thi, xok) : s0;
  // A non-finite or zero ray makes no cull (comparisons would be unordered).
  if (!s.fin || !xok) {
    // no float32 cull is valid for this ray: the ordered linear walk (same result)
    if (!ext) total = 1.0;
    query<false>(S, cptr(S.sph32), ext, o, d, L, radius, best, besti, bhit, bin, total, err, nullptr, xr);
    return true;
  }
  if (!resume) {
    ncov = 0;
    ovf = false;
    ref = S.bvh_root;
    sp = 0;
    walk_planes_boxes<BS>(S, ext, o, d, L, r, best, besti, bhit, bin, thi, ci, cv, ncov, ovf);
  }

  unsigned long long ws_ni = 0, ws_nl = 0, ws_li = 0, ws_ll = 0;   // RTX_WALKSTATS only
  // Speculative traversal (without postponing): a lane that reaches a leaf
  // while other lanes of its wave still search holds it (`pend`) and keeps
  // descending; the leaves are tested once every searching lane holds one.
  // The visiting order changes, the result cannot (order independence, above).
#ifndef RTX_SPEC
#define RTX_SPEC 1             // speculative traversal (diagnostic builds may turn it off to compare)
#endif
  constexpr bool SPEC = !PP && RTX_SPEC;
  int pend = BVH_NONE;
  while (ref != BVH_NONE || pend != BVH_NONE) {
    if (SPEC && ref < 0 && pend == BVH_NONE) {    // hold the leaf, search on
      pend = ref;
      ref = sp > 0 ? stk[(--sp) * BS] : BVH_NONE;
    }
    // ---- inner nodes: slab-test the four child boxes, descend into the nearest
    while (ref >= 0 && ref != BVH_NONE) {
      if (SPEC && !__ballot(pend == BVH_NONE)) break;   // every searching lane holds a leaf
      if (RTX_WALKSTATS) {
        const unsigned long long am = __ballot(1);
        ws_nl++;
        if ((int)__lane_id() == __builtin_ctzll(am)) ws_ni++;
      }
      float key[4];
      int ch[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        ch[k] = nodes[ref].child[k];
        key[k] = slab_key(nodes[ref], k, s, tlo, thi);
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
      if (SPEC && ref < 0 && pend == BVH_NONE) {  // reached a leaf: hold it, search on
        pend = ref;
        ref = sp > 0 ? stk[(--sp) * BS] : BVH_NONE;
      }
    }
    int lf;
    if (SPEC) {
      lf = pend;                                 // (a lane that found none yet waits here)
      pend = BVH_NONE;
    } else {
      if (ref == BVH_NONE) break;
      lf = ref;
    }
    // ---- leaf: pre-test its spheres, exact test for those not ruled out
    if (RTX_WALKSTATS && lf != BVH_NONE) {
      const unsigned long long am = __ballot(1);
      ws_ll++;
      if ((int)__lane_id() == __builtin_ctzll(am)) ws_li++;
    }
    if (lf != BVH_NONE)
      walk_leaf<BS>(lf, leaf4, x64, xobj, s, ext, o, d, dn, r, r2, L, radius, best, besti, bhit, bin, thi, err, ci, cv,
                    ncov, ovf, xr, Q16 ? S.q_err : 0.0f);
    if (!SPEC) {
      ref = sp > 0 ? stk[(--sp) * BS] : BVH_NONE;
      if (PP && __popcll(__ballot(ref != BVH_NONE)) < postpone && ref != BVH_NONE) return false;
    }
  }
  if (RTX_WALKSTATS) {
    unsigned long long* w = rtx_walkstats + (ext ? 0 : 4);
    atomicAdd(&w[0], ws_ni);
    atomicAdd(&w[1], ws_nl);
    atomicAdd(&w[2], ws_li);
    atomicAdd(&w[3], ws_ll);
  }
  if (!ext) walk_covers<BS>(S, o, d, L, radius, best, besti, bhit, bin, total, err, cv, ncov, ovf, xr);
  return true;
}

// Which spheres can raise, in float32 (s: signed distance of the center along
// the unit axis u from T, rho: its distance from the axis line, k = radius /
// |L - T|, so r1 = k |s|).  A raise needs d = |R - r1| up to rounding:
//   (A) R > r1: rho ~ R - r1 <= R, the axis line meets the ball;
//   (B) r1 > R: rho + R ~ k |s|, the ball touches the cone rho = k |s| from
//       inside (its point farthest from the axis lies on the cone).
// A child box is searched when its bounding ball (center c, radius h) could
// hold such a sphere: the line meets the ball, or f = rho - k |s| takes values
// of both signs on it.  mg covers the float32 rounding of T, u, k, the centers
// and the box bounds (each a few ulps of the scene scale Sx, times 1 + k for
// the cone): 2e-5 Sx (1 + k) is more than ten times that.
struct RaiseAxis {
  float tx, ty, tz, ux, uy, uz, k, mg;
};

__device__ __forceinline__ void raise_sr(const RaiseAxis& a, float cx, float cy, float cz, float& s, float& rho) {
  const float wx = cx - a.tx, wy = cy - a.ty, wz = cz - a.tz;
  s = __builtin_fmaf(wx, a.ux, __builtin_fmaf(wy, a.uy, wz * a.uz));
  const float px = __builtin_fmaf(wy, a.uz, -wz * a.uy), py = __builtin_fmaf(wz, a.ux, -wx * a.uz),
              pz = __builtin_fmaf(wx, a.uy, -wy * a.ux);
  rho = sqrtf(__builtin_fmaf(px, px, __builtin_fmaf(py, py, pz * pz)));
}

// (A) for child k of a node: the slab test of the box dilated by m S (§2.2)
// along the whole line (both directions: no t >= 0, no far bound).
template <typename NR>
__device__ __forceinline__ bool slab_line(const NR& node, int k, const SlabRay& s) {
  const F2 tx = __builtin_elementwise_fma(*reinterpret_cast<const F2*>(&node.lh[0][k][0]), s.pix, s.pax);
  const F2 ty = __builtin_elementwise_fma(*reinterpret_cast<const F2*>(&node.lh[1][k][0]), s.piy, s.pay);
  const F2 tz = __builtin_elementwise_fma(*reinterpret_cast<const F2*>(&node.lh[2][k][0]), s.piz, s.paz);
  const float tn = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fminf(tz.x, tz.y));
  const float tf = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
  return tn <= tf;
}

// (B) for a box: its bounding ball (center, h >= the half diagonal) meets the
// cone surface rho = k |s| (f = rho - k |s| takes both signs on the ball).
__device__ __forceinline__ bool raise_box(const RaiseAxis& a, float lx, float hx, float ly, float hy, float lz, float hz) {
  float s, rho;
  raise_sr(a, 0.5f * (lx + hx), 0.5f * (ly + hy), 0.5f * (lz + hz), s, rho);
  const float h = 0.5f * ((hx - lx) + (hy - ly) + (hz - lz));   // >= the half diagonal
  const float as = fabsf(s);
  const float fmin = fmaxf(rho - h, 0.0f) - a.k * (as + h);
  const float fmax = rho + h - a.k * fmaxf(as - h, 0.0f);
  return fmin <= a.mg && fmax >= -a.mg;                                    // (B); NaN: false
}

__device__ __forceinline__ bool raise_sphere(const RaiseAxis& a, float cx, float cy, float cz, float R2) {
  float s, rho;
  raise_sr(a, cx, cy, cz, s, rho);
  const float R = sqrtf(R2);
  return rho <= R + a.mg || fabsf(rho + R - a.k * fabsf(s)) <= a.mg;
}

// Does World#lit_area(T, L, radius) raise?  `nodes`/`leaf4`/`x64` are the
// hierarchy (LDS or global; nullptr: every sphere in record order), `stk`
// this lane's traversal stack (stride BS entries, free while this runs).
// (stk: int or, SPH_BVH_QLDS, int16_t entries.)
template <typename SP>
__device__ __forceinline__ bool lit_area_raises(const SceneDev& S, const Bvh4Node* nodes, const float4* leaf4,
                                                const Sphere64* x64, SP stk, int bs, V3 T, V3 L, double radius) {
  if (!(radius > 0.0) || S.n_sphere == 0) return false;   // r1 <= 0: no d with |R - r1| < d < r1 + R
  const V3 lt = vsub(L, T);
  RaiseAxis a;
  a.tx = (float)T.x, a.ty = (float)T.y, a.tz = (float)T.z;
  const float lx = (float)lt.x, ly = (float)lt.y, lz = (float)lt.z;
  const float ln = sqrtf(__builtin_fmaf(lx, lx, __builtin_fmaf(ly, ly, lz * lz)));
  a.ux = lx / ln, a.uy = ly / ln, a.uz = lz / ln;
  a.k = (float)radius / ln;
  const float Sx = fabsf(a.tx) + fabsf(a.ty) + fabsf(a.tz) + S.sph_scale;
  a.mg = CULL_M * Sx * (1.0f + a.k);
  const SlabRay sl = slab_setup(S, T, lt);
  const bool fin = __builtin_isfinite(a.ux) && __builtin_isfinite(a.uy) && __builtin_isfinite(a.uz) &&
                   __builtin_isfinite(a.k) && __builtin_isfinite(a.mg) && ln > 0.0f && sl.fin;
  if (nodes == nullptr || S.bvh_root == BVH_NONE || !fin) {
    // every sphere in record order (the float32 filter only where it is valid)
    for (int i = 0; i < S.n_sphere; i++) {
      if (fin && !raise_sphere(a, S.sph32[4 * i], S.sph32[4 * i + 1], S.sph32[4 * i + 2], S.sph32[4 * i + 3]))
        continue;
      const Sphere64 sp = S.sph64[i];
      if (penumbra_raises(v3p(sp.c), sp.r, T, lt, radius)) return true;
    }
    return false;
  }
  int sp = 0;
  int ref = S.bvh_root;
  while (true) {
    if (ref >= 0 && ref != BVH_NONE) {           // inner node: every child that may hold a raising sphere
      const Bvh4Node& nd = nodes[ref];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int ch = nd.child[k];
        if (ch == BVH_NONE) continue;
        if (slab_line(nd, k, sl) || raise_box(a, nd.lh[0][k][0], nd.lh[0][k][1], nd.lh[1][k][0], nd.lh[1][k][1],
                                              nd.lh[2][k][0], nd.lh[2][k][1]))
          stk[(sp++) * bs] = ch;
      }
    } else if (ref != BVH_NONE) {                // leaf
      const int v = ~ref;
      const int slot0 = (v >> 2) * BVH_LEAF;
      const int cnt = (v & 3) + 1;
      const float4 cx = leaf4[slot0], cy = leaf4[slot0 + 1], cz = leaf4[slot0 + 2], cw = leaf4[slot0 + 3];
      const float X[4] = {cx.x, cx.y, cx.z, cx.w}, Y[4] = {cy.x, cy.y, cy.z, cy.w}, Z[4] = {cz.x, cz.y, cz.z, cz.w},
                  W[4] = {cw.x, cw.y, cw.z, cw.w};
#pragma unroll
      for (int u = 0; u < 4; u++) {
        if (u >= cnt || !raise_sphere(a, X[u], Y[u], Z[u], W[u])) continue;
        const Sphere64 s64 = x64[slot0 + u];
        if (penumbra_raises(v3p(s64.c), s64.r, T, lt, radius)) return true;
      }
    }
    if (sp == 0) break;
    ref = stk[(--sp) * bs];
  }
  return false;
}

// lit_area_raises over a launch's sphere mode (the lanes engine's inline highlight
// check): the hierarchy from where the
// workgroup staged it (SphMode), the lane's LDS traversal stack.
template <int SPH, int BS>
__device__ __forceinline__ bool raises_walk(const KParams& p, char* lds, V3 T, V3 L, double radius) {
  const SceneDev& S = p.scene;
  if (SPH == SPH_BVH_QLDS)                     // (the float32 leaf records from global memory)
    return lit_area_raises(S, reinterpret_cast<const Bvh4Node*>(lds), reinterpret_cast<const float4*>(S.bvh_sph32),
                           S.bvh_sph64, qstack(lds, p), BS, T, L, radius);
  int* stk = reinterpret_cast<int*>(lds + p.lds_stack) + threadIdx.x;
  if (SPH == SPH_BVH_LDS || SPH == SPH_BVH_LDSX)
    return lit_area_raises(S, reinterpret_cast<const Bvh4Node*>(lds), reinterpret_cast<const float4*>(lds + p.lds_leaf),
                           SPH == SPH_BVH_LDSX ? reinterpret_cast<const Sphere64*>(lds + p.lds_x64) : S.bvh_sph64, stk,
                           BS, T, L, radius);
  if (SPH == SPH_BVH_MIX)
    return lit_area_raises(S, reinterpret_cast<const Bvh4Node*>(lds), reinterpret_cast<const float4*>(S.bvh_sph32),
                           S.bvh_sph64, stk, BS, T, L, radius);
  if (SPH == SPH_BVH_GLOBAL)
    return lit_area_raises(S, S.bvh, reinterpret_cast<const float4*>(S.bvh_sph32), S.bvh_sph64, stk, BS, T, L,
                           radius);
  return lit_area_raises(S, nullptr, nullptr, nullptr, (int*)nullptr, 0, T, L, radius);
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
// `m` is the object's material and `sph64` the sphere records (global memory,
// or the copies a bounce-level workgroup staged in LDS).
template <typename SP>
RTX_SHADE_FN void hit_info_m(const SceneDev& S, const Material& m, SP sph64, const Ray& ray, V3& hit, V3& delta,
                             V3& n, bool& in) {
  if (m.type == OBJ_SPHERE) {
    const Sphere64 sp = sph64[m.rec];
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
RTX_SHADE_FN void hit_info(const SceneDev& S, int obj, const Ray& ray, V3& hit, V3& delta, V3& n, bool& in) {
  hit_info_m(S, S.mat[obj], S.sph64, ray, hit, delta, n, in);
}

// Per-lane LIFO of pending rays (RayTracer#trace_sync's Array, ray_tracer.rb:21-30).
// The bottom `slots` entries live in LDS (11 eight-byte words per entry, laid
// out word-major across the workgroup's lanes so a wave's accesses are
// conflict-free); deeper entries go to the lane's own contiguous region of a
// global buffer (12 doubles per entry: one push or pop touches two 64-B lines,
// where a private-array entry, swizzled across the wave, touched 21).
constexpr int ITEM_WORDS = 11;
constexpr int GITEM_DOUBLES = 12;
struct Stack {
  int n;
  int maxs;        // entries a lane may hold (its global region's size; sized on the host)
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
__device__ __forceinline__ void emit(Stack& st, Item& pend, bool& has, uint32_t& err, const Ray& r,
                                     V3 att, uint64_t path, int depth) {
  if (depth <= 0 || vr(att) < 0.0001) return;
  if (has) {
    if (st.n < st.maxs) st.push(pend);
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
RTX_SHADE_FN bool shade_finish(const SceneDev& S, const CameraDev& cam, uint64_t seed, int x, int y,
                                          int sample, int obj, bool in, V3 hit, V3 delta, V3 n, V3 nn, V3 lc,
                                          int nl,
                                          Item& cur, Stack& st, V3& sum, uint32_t& err) {
  const Material& m = S.mat[obj];
  Item pend;
  bool has = false;
  const uint64_t R = (uint64_t)cam.pt + 3;
  const double c = vcos(cur.ray.d, n, err);
  const Ray refl = reflection(cur.ray, nn, c, hit, delta, err);
  emit(st, pend, has, err, refl, vmul(cur.att, v3p(m.refl_att)), cur.path * R + 1, cur.depth - 1);
  Ray refr;
  bool has_refr = false;
  if (m.type == OBJ_SPHERE)                                  // sphere.rb:92-94: rate inverted leaving
    has_refr = refraction(cur.ray, nn, c, hit, refl.d, in ? m.rr : 1.0 / m.rr, refr, err);
  else if (m.has_rr)                                         // plane.rb:57-61: same rate both ways
    has_refr = refraction(cur.ray, nn, c, hit, refl.d, m.rr, refr, err);
  if (has_refr)
    emit(st, pend, has, err, refr, vmul(cur.att, v3p(m.refr_att)), cur.path * R + 2, cur.depth - 1);
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
      emit(st, pend, has, err, r, att, cur.path * R + 3 + (uint64_t)k, cur.depth - 1);
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
// stops, ray_tracer.rb:77).  The `&& lit_area(ray.position, light.position,
// light.radius, object)` of a light whose cone the ray is in is always truthy
// in Ruby (a number), but it runs, and its Sphere#cover_area can raise
// (Math.acos, sphere.rb:45-46): `raises(T, L, radius)` answers whether it does
// (lit_area_raises), asked only while the ray has no raise yet.
// att_fn() gives the ray's attenuation, asked for only when a light fires.
#ifndef RTX_HL_RAISES
#define RTX_HL_RAISES 1      // 0: diagnostic builds only (timing without the highlight's lit_area raise walk)
#endif
template <typename Att, typename Leaf, typename Rz>
__device__ __forceinline__ bool highlight_leaves_att(const SceneDev& S, const Ray& ray, Att&& att_fn, Leaf&& leaf,
                                                     uint32_t& err, Rz&& raises) {
  Item it;
  it.ray = ray;
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
      if (RTX_HL_RAISES && !(err & 0xffu) && raises(it.ray.o, v3(L.pos[0], L.pos[1], L.pos[2]), L.radius, l))
        seterr(err, ERR_DOMAIN);
    }
  }
  if (!nfired) return false;
  it.att = att_fn();
  for (int l = 0; l < S.n_light; l++) {
    if (!(fired >> l & 1)) continue;
    const RTX_CONST LightDev& L = lights[l];
    leaf(vdiv(vmul(it.att, vsc(v3(L.color[0], L.color[1], L.color[2]), L.hl_rate)), (double)nfired));
  }
  return true;
}

template <typename Leaf, typename Rz>
__device__ __forceinline__ bool highlight_leaves(const SceneDev& S, const Item& it, Leaf&& leaf, uint32_t& err,
                                                 Rz&& raises) {
  return highlight_leaves_att(S, it.ray, [&] { return it.att; }, leaf, err, raises);
}

// The same into a running sum.  REDUCE: leaves go through rt_reduce
// (trace_sync); path_trace adds them with a plain `ret +=` (ray_tracer.rb:210),
// no "color greater than 1" check.
template <bool REDUCE = true, typename Rz>
__device__ __forceinline__ bool highlights(const SceneDev& S, const Item& it, V3& sum, uint32_t& err, Rz&& raises) {
  return highlight_leaves(S, it, [&](V3 c) {
    if (REDUCE) add_leaf(sum, c, err);
    else sum = vadd(sum, c);
  }, err, raises);
}

// `key` orders the raise sites as the reference meets them: (x * height + y) * 2
// + phase for pixels (render_sync runs x in the outer loop, y in the inner one,
// camera.rb:102-103; within a pixel render_at traces the pre samples before the
// extra ones, camera.rb:72-97, so a pre-sample raise (phase 0) comes before an
// extra-sample raise (phase 1) whatever their codes), the ray index for rtx_trace.
__device__ __forceinline__ void record_error(ErrState* e, uint32_t code, unsigned long long key) {
  atomicOr(&e->flags, 1u << code);
  atomicMin(&e->first[code], key);
}
__device__ __forceinline__ unsigned long long px_key(int x, int y, int H, int phase = 0) {
  return ((unsigned long long)x * (unsigned long long)H + (unsigned long long)y) << 1 | (unsigned long long)phase;
}

__device__ __forceinline__ int row_to_y(const KParams& p, int row) {
  if (p.tile_rows == 0) return p.y0 + row;
  const int k = row / p.tile_rows;
  const int t = p.row_tiles ? p.row_tiles[k] : k * p.nranks + p.rank;
  return t * p.tile_rows + (row - k * p.tile_rows);
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
    const int tile = p.lv_t0 + slot * p.lv_tstride;
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

// Fills the LDS layout of `p` for `mode` and returns the dynamic LDS bytes.
inline size_t lds_layout(KParams& p, int mode, int bs) {
  const SceneDev& S = p.scene;
  size_t off = 0;
  if (mode == SPH_LIN_LDS) off = (size_t)(S.n_sphere + 4) * 16;
  p.lds_x64 = p.lds_xobj = p.lds_mat = p.lds_sphr = p.lds_lbuf = p.lds_rgate = -1;
  if (mode == SPH_BVH_LDS || mode == SPH_BVH_MIX || mode == SPH_BVH_LDSX || mode == SPH_BVH_QLDS) {
    off = (size_t)S.n_nodes * sizeof(Bvh4Node);
    p.lds_leaf = (int32_t)off;
    if (mode == SPH_BVH_QLDS) off += (size_t)S.n_slots * 8;   // 16-bit records
    else if (mode != SPH_BVH_MIX) off += (size_t)S.n_slots * 16;
    if (mode == SPH_BVH_LDSX) {
      p.lds_x64 = (int32_t)off;
      off += (size_t)S.n_slots * sizeof(Sphere64);
      p.lds_xobj = (int32_t)off;
      off += (size_t)S.n_slots * 4;
      off = (off + 15) & ~(size_t)15;
      p.lds_mat = (int32_t)off;                 // shading's material and sphere record of the hit object
      off += (size_t)S.n_obj * sizeof(Material);
      p.lds_sphr = (int32_t)off;
      off += (size_t)S.n_sphere * sizeof(Sphere64);
    }
  }
  off = (off + 15) & ~(size_t)15;
  p.lds_stack = (int32_t)off;
  p.lds_cov = (int32_t)off;
  if (sph_is_bvh(mode)) {
    off += (size_t)S.bvh_stack * bs * (mode == SPH_BVH_QLDS ? 2 : 4);   // QLDS: int16 entries
    off = (off + 15) & ~(size_t)15;
    p.lds_cov = (int32_t)off;
    off += (size_t)COVER_K * bs * 12;
  }
  // the bottom of every lane's ray stack, as many entries as fit the budget
  off = (off + 15) & ~(size_t)15;
  p.lds_items = (int32_t)off;
  const size_t budget = sph_is_bvh(mode) ? LDS_TOTAL_BYTES : LDS_LIN_BLOCK_BYTES;
  const size_t per = (size_t)ITEM_WORDS * 8 * bs;
  int slots = budget > off ? (int)((budget - off) / per) : 0;
  if (slots > p.stk_slots_max) slots = p.stk_slots_max;
  p.stk_slots = slots;
  off += (size_t)slots * per;
  return off;
}

}  // namespace rtx
