// rtx_vec3.h — binary64 Vec3 with the semantics of the reference's only native
// code, Fast4DMatrix::Vec3 (ext/fast_4d_matrix/fast_4d_matrix.c), for host and
// device.  Compiled with -ffp-contract=off everywhere: no FMA, left-to-right
// sums, exactly the C extension's arithmetic (extconf.rb:6-10).
//
//   r      sqrt(x*x + y*y + z*z)                      (:62-73, cached there)
//   r2     r * r  (NOT x*x+y*y+z*z)                   (:280-284)
//   dot    0 + x1*x2 + y1*y2 + z1*z2                  (:98-107)
//   cos    sqrt(dot*dot / |a|^2 / |b|^2) <= 1  = |cos| (:109-129)
//   normalize  /r, zero vector is an error            (:286-293)
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define RTX_HD __host__ __device__ __forceinline__
#else
#define RTX_HD static inline
#endif

namespace rtx {

enum : uint32_t { ERR_NONE = 0, ERR_ZERO_VEC = 1, ERR_COLOR_GT1 = 2, ERR_DOMAIN = 3, ERR_TYPE = 4, ERR_N = 5 };

struct V3 {
  double x, y, z;
};

RTX_HD V3 v3(double x, double y, double z) { V3 v; v.x = x; v.y = y; v.z = z; return v; }
RTX_HD V3 v3p(const double* p) { return v3(p[0], p[1], p[2]); }
RTX_HD double vsq(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
RTX_HD double vr(V3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
RTX_HD double vr2(V3 a) { double r = vr(a); return r * r; }
RTX_HD double vdot(V3 a, V3 b) {
  double s = 0.0;
  s += a.x * b.x;
  s += a.y * b.y;
  s += a.z * b.z;
  return s;
}
RTX_HD V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RTX_HD V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RTX_HD V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
RTX_HD V3 vsc(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
RTX_HD V3 vdiv(V3 a, double s) { return v3(a.x / s, a.y / s, a.z / s); }
RTX_HD V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }
RTX_HD V3 vcross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
RTX_HD V3 vnorm(V3 a, uint32_t& err) {
  double r = sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  if (r == 0) {
    if (!err) err = ERR_ZERO_VEC;
    return a;
  }
  return v3(a.x / r, a.y / r, a.z / r);
}
RTX_HD double vcos(V3 a, V3 b, uint32_t& err) {
  double ret = 0.0;
  ret += a.x * b.x;
  ret += a.y * b.y;
  ret += a.z * b.z;
  double r1 = a.x * a.x + a.y * a.y + a.z * a.z;
  double r2 = b.x * b.x + b.y * b.y + b.z * b.z;
  if (r1 == 0 || r2 == 0) {
    if (!err) err = ERR_ZERO_VEC;
    return 0.0;
  }
  double v = sqrt(ret * ret / r1 / r2);
  if (v > 1) v = 1;
  return v;
}

// ---- the counter RNG contract (DESIGN.md "RNG"; oracle/rng.py) --------------
RTX_HD uint64_t fmix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  return h;
}
RTX_HD double rand01(uint64_t seed, int32_t x, int32_t y, int32_t sample, uint64_t path, int32_t draw) {
  uint64_t h = seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  h = fmix64(h ^ (((uint64_t)(uint32_t)x << 32) | (uint32_t)y));
  h = fmix64(h ^ (((uint64_t)(uint32_t)sample << 32) | (uint32_t)draw));
  h = fmix64(h ^ path);
  return (double)(h >> 11) * (1.0 / 9007199254740992.0);
}

}  // namespace rtx
