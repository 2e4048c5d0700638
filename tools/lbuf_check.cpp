// Host-only check of the light buffer (tests/test_lbuf.py).
// stdin: "light x y z" lines, then "x y z r" sphere lines.  Builds the
// hierarchy as rtx_scene_upload does (binned SAH) and the light buffer
// (build_light_buffer, cells per face side argv[1]), then for argv[2] random
// shadow-ray targets T per light (in and around the spheres' box, on and just
// off the spheres' surfaces, next to the light) finds every sphere within R of
// the segment [T, L] in binary64 (a superset of the spheres whose cover the
// reference counts) and checks that its leaf is listed in the cell the device
// looks up (query_lbuf's float32 arithmetic, restated below).  Prints the
// number of targets, of covering spheres and of misses (must be 0).
//
// Raise mode (argv[3] = "raise", argv[4] = the raise buffer's cells per face
// side; lights given as "light x y z radius"): builds the raise buffer as
// rtx_scene_upload does (floor: 0.99 of the nearest sphere surface) and, for
// argv[2] targets per light, places a random sphere exactly at a tangency of
// World#lit_area's acos raise (sphere.rb:42: d = |R - r1|, regime A or B, with
// a random axis through the light), rounds the target to binary64, checks in
// binary64 that it lies within 1e-9 S of the tangency, and counts those whose
// leaf is in none of the device's lists (the light buffer's cell, the raise
// buffer's B2 / B1 / M lists, lbuf_lookup.h shadow_lists) unless the device
// would walk the hierarchy for that target.  Prints the tangencies tested, the
// hierarchy fallbacks and the misses (must be 0).
#include <math.h>
#include <stdio.h>

#include <iostream>
#include <random>
#include <string>

#include "../raytracing_rb_amd/csrc/rtx_bvh_build.h"
#include "lbuf_lookup.h"

using namespace rtx;

namespace {

using lbuf_host::device_cell;

// distance from C to the segment [A, B] (binary64)
double seg_dist(const double A[3], const double B[3], const double C[3]) {
  double ab[3], ac[3];
  for (int a = 0; a < 3; a++) ab[a] = B[a] - A[a], ac[a] = C[a] - A[a];
  const double dd = ab[0] * ab[0] + ab[1] * ab[1] + ab[2] * ab[2];
  double t = dd > 0 ? (ac[0] * ab[0] + ac[1] * ab[1] + ac[2] * ab[2]) / dd : 0.0;
  t = std::min(1.0, std::max(0.0, t));
  double e = 0.0;
  for (int a = 0; a < 3; a++) {
    const double q = A[a] + t * ab[a] - C[a];
    e += q * q;
  }
  return sqrt(e);
}

}  // namespace

int raise_main(int n, int per_light, int nc, const std::vector<double>& lp, const std::vector<double>& lr,
               const std::vector<Sphere64>& s64, Bvh4Builder& bb, int root, const std::vector<int32_t>& leaf_of);

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 16;
  const int per_light = argc > 2 ? atoi(argv[2]) : 100000;
  const bool raise_mode = argc > 3 && std::string(argv[3]) == "raise";
  const int nc = argc > 4 ? atoi(argv[4]) : 8;
  std::vector<double> lp, lr;
  std::vector<Sphere64> s64;
  std::vector<float> s32;
  std::vector<int32_t> obj;
  std::string tok;
  while (std::cin >> tok) {
    if (tok == "light") {
      double x, y, z, r = 0.0;
      std::cin >> x >> y >> z;
      if (raise_mode) std::cin >> r;
      lp.insert(lp.end(), {x, y, z});
      lr.push_back(r);
      continue;
    }
    Sphere64 s;
    s.c[0] = std::stod(tok);
    std::cin >> s.c[1] >> s.c[2] >> s.r;
    s64.push_back(s);
    for (float v : {(float)s.c[0], (float)s.c[1], (float)s.c[2], (float)(s.r * s.r)}) s32.push_back(v);
    obj.push_back((int)obj.size());
  }
  std::vector<BSph> bs(s64.size());
  for (size_t k = 0; k < s64.size(); k++) {
    for (int a = 0; a < 3; a++) bs[k].c[a] = s64[k].c[a];
    bs[k].r = s64[k].r;
    bs[k].rec = (int)k;
  }
  Bvh4Builder bb{bs, s64, s32, obj};
  bb.sah = true;
  const int root = bs.empty() ? BVH_NONE : bb.build(0, (int)bs.size(), 0);
  const int nl = (int)lp.size() / 3;
  const LightBuffer lb = build_light_buffer(bb, root, reinterpret_cast<const double(*)[3]>(lp.data()), nl, n, 1u << 30,
                                            raise_mode ? lr.data() : nullptr);
  if (!lb.n) {
    printf("no light buffer\n");
    return 1;
  }
  // sphere -> its leaf reference
  std::vector<int32_t> leaf_of(s64.size(), BVH_NONE);
  auto note = [&](int32_t ref) {
    const int v = ~ref, slot0 = (v >> 2) * BVH_LEAF, cnt = (v & 3) + 1;
    for (int u = 0; u < cnt; u++) {
      const int rec = bb.slot_obj[(size_t)slot0 + u];
      if (rec >= 0) leaf_of[(size_t)rec] = ref;
    }
  };
  if (root < 0 && root != BVH_NONE) note(root);
  for (const Bvh4Node& nd : bb.nodes)
    for (int k = 0; k < 4; k++)
      if (nd.child[k] < 0 && nd.child[k] != BVH_NONE) note(nd.child[k]);
  if (raise_mode) return raise_main(n, per_light, nc, lp, lr, s64, bb, root, leaf_of);
  double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
  for (const Sphere64& s : s64)
    for (int a = 0; a < 3; a++) lo[a] = std::min(lo[a], s.c[a] - s.r), hi[a] = std::max(hi[a], s.c[a] + s.r);
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  long targets = 0, covers = 0, misses = 0, listed = 0;
  for (int li = 0; li < nl; li++) {
    const double* L = &lp[3 * li];
    const uint16_t* blk = lb.words.data() + (size_t)lb.stride * li;
    const uint16_t* ent = blk + 6 * n * n + 1;
    for (int k = 0; k < per_light; k++) {
      double T[3];
      const int kind = k % 4;
      if (kind == 0 || s64.empty()) {                 // the box and around it
        for (int a = 0; a < 3; a++) {
          const double w = hi[a] - lo[a] + 1.0;
          T[a] = lo[a] - 0.5 * w + 2.0 * w * U(rng);
        }
      } else if (kind <= 2) {                         // on or just off a sphere (shading targets)
        const Sphere64& s = s64[(size_t)(U(rng) * s64.size()) % s64.size()];
        double u[3], r2 = 0;
        do {
          r2 = 0;
          for (int a = 0; a < 3; a++) u[a] = 2 * U(rng) - 1, r2 += u[a] * u[a];
        } while (r2 > 1 || r2 < 1e-6);
        const double off = kind == 1 ? 1e-5 : (U(rng) - 0.5) * 1e-3;
        for (int a = 0; a < 3; a++) T[a] = s.c[a] + u[a] / sqrt(r2) * (s.r + off);
      } else {                                        // near the light
        for (int a = 0; a < 3; a++) T[a] = L[a] + (2 * U(rng) - 1) * 0.5;
      }
      const double d[3] = {L[0] - T[0], L[1] - T[1], L[2] - T[2]};
      // the device's float images: d = L - T rounded, v = -d
      const int cell = device_cell(-(float)d[0], -(float)d[1], -(float)d[2], n);
      if (cell < 0) continue;                         // (the device walks the hierarchy)
      targets++;
      listed += blk[cell + 1] - blk[cell];
      for (size_t si = 0; si < s64.size(); si++) {
        if (!(seg_dist(T, L, s64[si].c) <= s64[si].r * (1 + 1e-9))) continue;
        covers++;
        bool found = false;
        for (int e = blk[cell]; e < blk[cell + 1] && !found; e++) found = (int32_t)(int16_t)ent[e] == leaf_of[si];
        if (!found) {
          misses++;
          if (misses < 10)
            fprintf(stderr, "miss: light %d T (%.17g %.17g %.17g) sphere %zu cell %d\n", li, T[0], T[1], T[2], si, cell);
        }
      }
    }
  }
  size_t words = 0;
  for (int li = 0; li < nl; li++) words += lb.stride;
  printf("n %d targets %ld covers %ld misses %ld words %zu listed_x100 %ld\n", n, targets, covers, misses, words,
         targets ? 100 * listed / targets : 0);
  return misses ? 3 : 0;
}

// ------------------------------------------------------------------ raise mode
int raise_main(int n, int per_light, int nc, const std::vector<double>& lp, const std::vector<double>& lr,
               const std::vector<Sphere64>& s64, Bvh4Builder& bb, int root, const std::vector<int32_t>& leaf_of) {
  const int nl = (int)lr.size();
  std::vector<double> lf(nl);
  for (int li = 0; li < nl; li++) {
    double fl = HUGE_VAL;
    for (const Sphere64& s : s64) {
      const double w[3] = {s.c[0] - lp[3 * li], s.c[1] - lp[3 * li + 1], s.c[2] - lp[3 * li + 2]};
      fl = std::min(fl, sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]) - s.r);
    }
    lf[li] = std::isfinite(fl) ? std::max(0.0, 0.99 * fl) : 0.0;
  }
  LightBuffer lb = build_light_buffer(bb, root, reinterpret_cast<const double(*)[3]>(lp.data()), nl, n, 1u << 30,
                                      lr.data());
  const bool per_sphere = s64.size() > 512;          // (rtx_scene_upload's choice)
  RaiseBuffer rb = build_raise_buffer(bb, root, reinterpret_cast<const double(*)[3]>(lp.data()), lr.data(), lf.data(),
                                      nl, nc, (size_t)1 << 30, nullptr, per_sphere);
  std::vector<int32_t> slot_of(s64.size(), -1);
  for (size_t k = 0; k < bb.slot_obj.size(); k++)
    if (bb.slot_obj[k] >= 0) slot_of[(size_t)bb.slot_obj[k]] = (int32_t)k;
  if (!lb.n || !rb.n || lb.n % rb.n) {
    printf("no buffers\n");
    return 1;
  }
  const std::vector<uint16_t> gates = raise_gates(rb, nl);
  std::mt19937_64 rng(777);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  long tested = 0, fallback = 0, misses = 0, listed = 0;
  for (int li = 0; li < nl; li++) {
    const double* L = &lp[3 * li];
    const double rad = lr[li];
    if (!(rad > 0.0)) continue;
    for (int k = 0; k < per_light; k++) {
      const size_t si = (size_t)(U(rng) * s64.size()) % s64.size();
      const Sphere64& sp = s64[si];
      double u[3], r2;
      do {
        r2 = 0;
        for (int a = 0; a < 3; a++) u[a] = 2 * U(rng) - 1, r2 += u[a] * u[a];
      } while (r2 > 1 || r2 < 1e-6);
      for (int a = 0; a < 3; a++) u[a] /= sqrt(r2);
      // bias half the axes towards the sphere (its projection lands near the center)
      if (k % 2) {
        double w[3], wn = 0;
        for (int a = 0; a < 3; a++) w[a] = sp.c[a] - L[a], wn += w[a] * w[a];
        wn = sqrt(wn);
        const double spread = (sp.r + rad) / wn * 1.5 * U(rng);
        double un = 0;
        for (int a = 0; a < 3; a++) u[a] = w[a] / wn + spread * u[a], un += u[a] * u[a];
        for (int a = 0; a < 3; a++) u[a] /= sqrt(un);
      }
      double mu = 0;
      for (int a = 0; a < 3; a++) mu += (sp.c[a] - L[a]) * u[a];
      double dd = 0;
      for (int a = 0; a < 3; a++) {
        const double q = sp.c[a] - L[a] - mu * u[a];
        dd += q * q;
      }
      const double d = sqrt(dd);
      const bool regA = (k / 2) % 2 == 0;
      if (regA && !(d < sp.r)) continue;
      const double c = regA ? (sp.r - d) / rad : (sp.r + d) / rad;
      const double t = (k / 4) % 2 == 0 || fabs(1.0 - c) < 1e-6 ? mu / (1.0 + c) : mu / (1.0 - c);
      double T[3];
      for (int a = 0; a < 3; a++) T[a] = L[a] + t * u[a];
      // the reference's quantities in binary64 at the rounded target
      double lt[3], ctv[3], ltn2 = 0, dot = 0;
      for (int a = 0; a < 3; a++) lt[a] = L[a] - T[a], ctv[a] = sp.c[a] - T[a], ltn2 += lt[a] * lt[a], dot += ctv[a] * lt[a];
      const double tt = dot / ltn2;
      double x1t = 0, x1c = 0;
      for (int a = 0; a < 3; a++) {
        const double x1 = T[a] + lt[a] * tt;
        x1t += (x1 - T[a]) * (x1 - T[a]);
        x1c += (x1 - sp.c[a]) * (x1 - sp.c[a]);
      }
      const double r1 = rad * (sqrt(x1t) / sqrt(ltn2)), dd1 = sqrt(x1c);
      const double scale = fabs(L[0]) + fabs(L[1]) + fabs(L[2]) + fabs(sp.c[0]) + fabs(sp.c[1]) + fabs(sp.c[2]) + sp.r;
      if (!(fabs(dd1 - fabs(sp.r - r1)) <= 1e-9 * scale) || !(sqrt(ltn2) > 0)) continue;   // (not near a tangency)
      tested++;
      const lbuf_host::Lists ls = lbuf_host::shadow_lists(lb.words.data() + (size_t)lb.stride * li, lb.n,
                                                          rb.words.data() + (size_t)rb.stride * li,
                                                          gates.data() + (size_t)6 * rb.n * rb.n * li, rb.n, lt,
                                                          raise_floor2(rb, li), raise_lf2(rb, li), per_sphere);
      if (ls.fallback) {
        fallback++;
        continue;
      }
      bool found = false;
      for (const auto* v : {&ls.cover, &ls.b2, &ls.b1, &ls.m}) {
        listed += v->size();
        const bool slots = per_sphere && v != &ls.cover;
        for (int32_t r : *v) found = found || r == (slots ? slot_of[si] : leaf_of[si]);
      }
      if (!found) {
        misses++;
        if (misses < 10)
          fprintf(stderr, "raise miss: light %d T (%.17g %.17g %.17g) sphere %zu regime %c t %.6g\n", li, T[0], T[1],
                  T[2], si, regA ? 'A' : 'B', t);
      }
    }
  }
  printf("n %d nc %d per_sphere %d tangencies %ld fallbacks %ld misses %ld rbuf_words %d listed_x100 %ld\n", n, nc,
         (int)per_sphere, tested, fallback, misses, rb.stride, tested ? 100 * listed / std::max(1L, tested - fallback) : 0);
  return misses ? 3 : 0;
}
