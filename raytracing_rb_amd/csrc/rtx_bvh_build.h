// rtx_bvh_build.h — host-only: the four-wide sphere hierarchy builder and
// the 16-bit leaf records of SPH_BVH_QLDS.
// Included by rtx_capi.cpp (rtx_scene_upload) and by tools/walk_sim.cpp, the
// CPU walk simulator, so both see the same trees.  No HIP calls.
#pragma once
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "rtx_scene.h"

#ifndef RTX_SAH_PUSHES
#define RTX_SAH_PUSHES 12                     // SAH only while <= this many traversal-stack entries sit above
#endif

namespace rtx {
// ------------------------------------------------------------------ BVH build
// Four-wide hierarchy: each node splits its spheres in two (binned SAH near
// the root, median of the longest centroid axis below), then splits each half
// again (up to four children);
// groups of <= BVH_LEAF spheres become leaves.  Child boxes are float32 and
// contain every member sphere exactly (bounds rounded outwards); see
// DESIGN.md §2.1 and rtx_scene.h.
namespace bvhb {
struct BSph {
  double c[3];
  double r;
  int rec;
};

static float f32_down(double x) {           // largest float <= x
  float f = (float)x;
  if ((double)f > x) f = nextafterf(f, -INFINITY);
  return f;
}
static float f32_up(double x) {             // smallest float >= x
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, INFINITY);
  return f;
}

struct Bvh4Builder {
  std::vector<BSph>& sp;
  const std::vector<Sphere64>& sph64;
  const std::vector<float>& sph32;
  const std::vector<int32_t>& sph_obj;
  std::vector<Bvh4Node> nodes;
  std::vector<float> slot32;
  std::vector<Sphere64> slot64;
  std::vector<int32_t> slot_obj;
  int stack = 0;                              // worst-case traversal stack (3 pushes per internal level)

  // float32 box containing every sphere of sp[lo, hi); the double bounds are
  // widened by a relative 1e-12 to cover their own rounding.
  void box(int lo, int hi, float blo[3], float bhi[3]) {
    for (int a = 0; a < 3; a++) {
      double mn = INFINITY, mx = -INFINITY;
      for (int i = lo; i < hi; i++) {
        const double r = fabs(sp[i].r);
        mn = fmin(mn, sp[i].c[a] - r);
        mx = fmax(mx, sp[i].c[a] + r);
      }
      blo[a] = f32_down(mn - 1e-12 * fabs(mn) - 1e-300);
      bhi[a] = f32_up(mx + 1e-12 * fabs(mx) + 1e-300);
    }
  }

  // Split sp[lo, hi) in two.  Binned surface-area heuristic (16 centroid bins
  // per axis, cost = area(left) * n_left + area(right) * n_right over the
  // spheres' boxes) while the traversal stack above stays shallow; otherwise,
  // or when no bin boundary separates the centroids, the median of the longest
  // centroid axis.  Deterministic: stable partitions, first-best bin wins.
  bool sah = true;
  int split(int lo, int hi, int pushes = 0) {
    double cmn[3] = {INFINITY, INFINITY, INFINITY}, cmx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = lo; i < hi; i++)
      for (int a = 0; a < 3; a++) {
        cmn[a] = fmin(cmn[a], sp[i].c[a]);
        cmx[a] = fmax(cmx[a], sp[i].c[a]);
      }
    if (sah && pushes <= RTX_SAH_PUSHES) {
      constexpr int NB = 16;
      auto bin_of = [&](double x, int a) {
        int b = (int)((x - cmn[a]) / (cmx[a] - cmn[a]) * NB);
        return b < 0 ? 0 : (b >= NB ? NB - 1 : b);
      };
      auto area = [](const double* mn, const double* mx) {
        const double dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        return dx * dy + dy * dz + dz * dx;
      };
      double best = INFINITY;
      int best_axis = -1, best_bin = -1;
      for (int a = 0; a < 3; a++) {
        if (!(cmx[a] - cmn[a] > 0)) continue;
        double bmn[NB][3], bmx[NB][3];
        int cnt[NB] = {0};
        for (int b = 0; b < NB; b++)
          for (int k = 0; k < 3; k++) {
            bmn[b][k] = INFINITY;
            bmx[b][k] = -INFINITY;
          }
        for (int i = lo; i < hi; i++) {
          const int b = bin_of(sp[i].c[a], a);
          const double r = fabs(sp[i].r);
          cnt[b]++;
          for (int k = 0; k < 3; k++) {
            bmn[b][k] = fmin(bmn[b][k], sp[i].c[k] - r);
            bmx[b][k] = fmax(bmx[b][k], sp[i].c[k] + r);
          }
        }
        double rmn[NB][3], rmx[NB][3];                  // suffix boxes over bins b..NB-1
        int rcnt[NB];
        double amn[3] = {INFINITY, INFINITY, INFINITY}, amx[3] = {-INFINITY, -INFINITY, -INFINITY};
        int acc = 0;
        for (int b = NB - 1; b >= 0; b--) {
          for (int k = 0; k < 3; k++) {
            rmn[b][k] = amn[k] = fmin(amn[k], bmn[b][k]);
            rmx[b][k] = amx[k] = fmax(amx[k], bmx[b][k]);
          }
          rcnt[b] = acc += cnt[b];
        }
        double lmn[3] = {INFINITY, INFINITY, INFINITY}, lmx[3] = {-INFINITY, -INFINITY, -INFINITY};
        int lc = 0;
        for (int b = 0; b + 1 < NB; b++) {              // left = bins 0..b, right = bins b+1..
          for (int k = 0; k < 3; k++) {
            lmn[k] = fmin(lmn[k], bmn[b][k]);
            lmx[k] = fmax(lmx[k], bmx[b][k]);
          }
          lc += cnt[b];
          if (lc == 0 || rcnt[b + 1] == 0) continue;
          const double cost = area(lmn, lmx) * lc + area(rmn[b + 1], rmx[b + 1]) * rcnt[b + 1];
          if (cost < best) {
            best = cost;
            best_axis = a;
            best_bin = b;
          }
        }
      }
      if (best_axis >= 0) {
        const int a = best_axis;
        auto it = std::stable_partition(sp.begin() + lo, sp.begin() + hi,
                                        [&](const BSph& q) { return bin_of(q.c[a], a) <= best_bin; });
        const int mid = (int)(it - sp.begin());
        if (mid > lo && mid < hi) return mid;
      }
    }
    int axis = 0;
    for (int a = 1; a < 3; a++)
      if (cmx[a] - cmn[a] > cmx[axis] - cmn[axis]) axis = a;
    const int mid = (lo + hi) / 2;
    std::nth_element(sp.begin() + lo, sp.begin() + mid, sp.begin() + hi, [axis](const BSph& a, const BSph& b) {
      return a.c[axis] < b.c[axis] || (a.c[axis] == b.c[axis] && a.rec < b.rec);
    });
    return mid;
  }

  int32_t leaf(int lo, int hi) {
    const int id = (int)(slot_obj.size() / BVH_LEAF);
    float soa[4][BVH_LEAF];                      // a leaf's float32 records component-major:
    for (int u = 0; u < BVH_LEAF; u++) {         // {x0..x3}, {y0..y3}, {z0..z3}, {R^2 0..3}
      const int rec = lo + u < hi ? sp[lo + u].rec : -1;
      slot_obj.push_back(rec >= 0 ? sph_obj[rec] : -1);
      slot64.push_back(rec >= 0 ? sph64[rec] : Sphere64{{0.0, 0.0, 0.0}, -1.0});
      for (int k = 0; k < 4; k++) soa[k][u] = rec >= 0 ? sph32[4 * rec + k] : 0.0f;
    }
    for (int k = 0; k < 4; k++)
      for (int u = 0; u < BVH_LEAF; u++) slot32.push_back(soa[k][u]);
    return ~(int32_t)((id << 2) | (hi - lo - 1));
  }

  // Reference to the subtree over sp[lo, hi); `pushes` = stack entries above it.
  int32_t build(int lo, int hi, int pushes) {
    if (hi - lo <= BVH_LEAF) return leaf(lo, hi);
    const int me = (int)nodes.size();
    nodes.push_back(Bvh4Node{});
    int g[5], ng = 0;
    const int mid = split(lo, hi, pushes);
    for (int h = 0; h < 2; h++) {
      const int a = h ? mid : lo, b = h ? hi : mid;
      g[ng++] = a;
      if (b - a > BVH_LEAF) g[ng++] = split(a, b, pushes);
    }
    g[ng] = hi;
    Bvh4Node n;
    for (int k = 0; k < 4; k++) {               // empty slot: a point far outside every scene,
      n.child[k] = BVH_NONE;                     // which no finite ray's slab test accepts
      for (int a = 0; a < 3; a++) {
        n.lh[a][k][0] = 3e38f;
        n.lh[a][k][1] = 3e38f;
      }
    }
    const int below = pushes + ng - 1;          // visiting one child leaves <= ng-1 siblings pushed
    if (below > stack) stack = below;
    for (int k = 0; k < ng; k++) {
      float blo[3], bhi[3];
      box(g[k], g[k + 1], blo, bhi);
      for (int a = 0; a < 3; a++) {
        n.lh[a][k][0] = blo[a];
        n.lh[a][k][1] = bhi[a];
      }
      n.child[k] = build(g[k], g[k + 1], below);
    }
    nodes[me] = n;
    return me;
  }
};
}  // namespace bvhb

using bvhb::BSph;
using bvhb::Bvh4Builder;
using bvhb::f32_down;
using bvhb::f32_up;

// 16-bit pre-test records of the hierarchy's leaves (SPH_BVH_QLDS, DESIGN.md
// §3.15): per leaf 8 words, {x 0..3}, {y 0..3}, {z 0..3}, {r 0..3} as 16-bit
// pairs (slot u in the low half of word 2k for u = 0, 2).  The device decodes
// center axis a as fmaf(q, step[a], org[a]) and the radius as q * rstep, in
// float32, the operations repeated here: a decoded center lies e from the true
// one (exact, in binary64) and the decoded radius is at least R + e, so the
// decoded ball holds the true one and the §2.1 pre-test stays conservative;
// its "wholly behind" half also needs e below half its margin (m S).
struct QuantLeaves {
  std::vector<uint32_t> rec;
  float org[3] = {0.0f, 0.0f, 0.0f}, step[3] = {1.0f, 1.0f, 1.0f}, rstep = 1.0f;
  bool ok = false;
  double max_err = 0.0;
  double max_r = 0.0;
};

inline QuantLeaves quantize_leaves(const Bvh4Builder& bb, float sph_scale) {
  QuantLeaves ql;
  const size_t n_slots = bb.slot64.size();
  ql.rec.assign(n_slots * 2, 0u);
  double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
  for (const Sphere64& s : bb.slot64) {
    if (!(s.r >= 0.0)) continue;                  // padding slot
    for (int a = 0; a < 3; a++) lo[a] = std::min(lo[a], s.c[a]), hi[a] = std::max(hi[a], s.c[a]);
  }
  if (!(lo[0] <= hi[0])) return ql;               // no spheres
  for (int a = 0; a < 3; a++) {
    ql.org[a] = (float)lo[a];
    const float st = (float)((hi[a] - lo[a]) / 65535.0 * (1.0 + 1e-6));
    ql.step[a] = st > 0.0f ? st : 1.0f;
  }
  std::vector<double> grown(n_slots, 0.0);        // R + e per slot
  double max_r = 0.0;
  for (size_t k = 0; k < n_slots; k++) {
    const Sphere64& s = bb.slot64[k];
    if (!(s.r >= 0.0)) continue;
    double e2 = 0.0;
    for (int a = 0; a < 3; a++) {
      double qd = std::nearbyint((s.c[a] - (double)ql.org[a]) / (double)ql.step[a]);
      qd = std::min(65535.0, std::max(0.0, qd));
      const uint32_t qv = (uint32_t)qd;
      const double dec = (double)std::fmaf((float)qv, ql.step[a], ql.org[a]);
      e2 += (dec - s.c[a]) * (dec - s.c[a]);
      const size_t w = (k / BVH_LEAF) * 8 + (size_t)a * 2 + (k % BVH_LEAF) / 2;
      ql.rec[w] |= qv << (16 * (k % 2));
    }
    const double e = std::sqrt(e2) * (1.0 + 1e-9);
    ql.max_err = std::max(ql.max_err, e);
    grown[k] = (s.r + e) * (1.0 + 1e-12);
    max_r = std::max(max_r, grown[k]);
  }
  if (!std::isfinite(max_r)) return ql;
  ql.max_r = max_r;
  ql.rstep = max_r > 0.0 ? (float)(max_r / 65535.0 * (1.0 + 1e-6)) : 1.0f;
  for (size_t k = 0; k < n_slots; k++) {
    if (!(bb.slot64[k].r >= 0.0)) continue;
    double qd = std::ceil(grown[k] / (double)ql.rstep);
    while (qd <= 65535.0 && (double)((float)qd * ql.rstep) < grown[k]) qd += 1.0;
    if (qd > 65535.0) return ql;
    const size_t w = (k / BVH_LEAF) * 8 + 6 + (k % BVH_LEAF) / 2;
    ql.rec[w] |= (uint32_t)qd << (16 * (k % 2));
  }
  ql.ok = ql.max_err <= 0.5 * CULL_M * (double)sph_scale;
  return ql;
}

// Light buffer: for each light, a cube map of 6 x n x n cells
// around its position; cell c lists the hierarchy's leaves that hold a sphere
// whose disc, as seen from the light, meets the cell.  A sphere that covers a
// shadow ray's target T (World#lit_area: it crosses the segment from T to the
// light L, short of L) meets the ray from L towards T, so its disc holds that
// direction and its leaf is in the direction's cell: the shadow walk visits
// those leaves only, with the same leaf tests.  The discs are widened by
// DELTA radians, far more than the float32 cell lookup's error (the cell of
// direction v is found on face 2a + (v_a < 0) of its dominant axis a, at
// i = floor((s + 1) n / 2), s = v_b / |v_a|, b = (a + 1) mod 3, likewise j for
// c = (a + 2) mod 3); a light inside or on a sphere puts that sphere's leaf in
// every cell.  Layout per light (uint16 words, `stride` per light): 6 n n + 1
// offsets into the light's leaf list, then the list (leaf references, int16).
struct LightBuffer {
  int n = 0, stride = 0;
  std::vector<uint16_t> words;
};

inline LightBuffer build_light_buffer(const Bvh4Builder& bb, int root, const double (*lpos)[3], int n_light, int n,
                                      size_t max_words) {
  LightBuffer lb;
  if (n_light <= 0 || root == BVH_NONE || n <= 0) return lb;
  std::vector<int32_t> leaves;                     // every leaf reference of the hierarchy
  if (root < 0) leaves.push_back(root);
  for (const Bvh4Node& nd : bb.nodes)
    for (int k = 0; k < 4; k++)
      if (nd.child[k] < 0 && nd.child[k] != BVH_NONE) leaves.push_back(nd.child[k]);
  for (int32_t ref : leaves)
    if (ref < -32768) return lb;                   // (the lists hold 16-bit references: at most 32,768 leaves)
  const double DELTA = 1e-4, PI = 3.141592653589793;
  const int cells = 6 * n * n;
  const int B = n % 8 == 0 ? n / 8 : (n % 4 == 0 ? n / 4 : 1);   // cells per block side
  const int nb = n / B;
  auto dir = [](int face, double s, double t, double v[3]) {   // the direction of face `face` at (s, t)
    const int a = face >> 1, b = (a + 1) % 3, c = (a + 2) % 3;
    v[a] = (face & 1) ? -1.0 : 1.0;
    v[b] = s;
    v[c] = t;
    const double r = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    for (int k = 0; k < 3; k++) v[k] /= r;
  };
  auto angle = [](const double u[3], const double v[3]) {
    const double d = u[0] * v[0] + u[1] * v[1] + u[2] * v[2];
    return std::acos(std::max(-1.0, std::min(1.0, d)));
  };
  // a rectangle of face coordinates: its center direction and angular radius (from boundary samples)
  auto region = [&](int face, double s0, double s1, double t0, double t1, double ctr[3]) {
    dir(face, 0.5 * (s0 + s1), 0.5 * (t0 + t1), ctr);
    double rho = 0.0;
    for (int k = 0; k <= 8; k++) {
      const double e = k / 8.0;
      const double pts[4][2] = {{s0 + e * (s1 - s0), t0}, {s0 + e * (s1 - s0), t1}, {s0, t0 + e * (t1 - t0)},
                                {s1, t0 + e * (t1 - t0)}};
      for (const auto& q : pts) {
        double v[3];
        dir(face, q[0], q[1], v);
        rho = std::max(rho, angle(ctr, v));
      }
    }
    return rho * (1.0 + 1e-6);
  };
  std::vector<double> cctr(3 * (size_t)cells), crho(cells), bctr(3 * (size_t)6 * nb * nb), brho(6 * nb * nb);
  for (int face = 0; face < 6; face++) {
    for (int i = 0; i < n; i++)
      for (int j = 0; j < n; j++) {
        const int cell = (face * n + i) * n + j;
        crho[cell] = region(face, -1.0 + 2.0 * i / n, -1.0 + 2.0 * (i + 1) / n, -1.0 + 2.0 * j / n,
                            -1.0 + 2.0 * (j + 1) / n, &cctr[3 * (size_t)cell]);
      }
    for (int bi = 0; bi < nb; bi++)
      for (int bj = 0; bj < nb; bj++) {
        const int blk = (face * nb + bi) * nb + bj;
        brho[blk] = region(face, -1.0 + 2.0 * bi * B / n, -1.0 + 2.0 * (bi + 1) * B / n, -1.0 + 2.0 * bj * B / n,
                           -1.0 + 2.0 * (bj + 1) * B / n, &bctr[3 * (size_t)blk]);
      }
  }
  auto within = [&](const double u[3], const double* c, double lim) {   // angle(u, c) <= lim
    if (lim >= PI) return true;
    return u[0] * c[0] + u[1] * c[1] + u[2] * c[2] >= std::cos(lim);
  };
  std::vector<std::vector<uint16_t>> per(n_light);
  for (int li = 0; li < n_light; li++) {
    const double* L = lpos[li];
    std::vector<std::vector<int>> in_cell(cells);   // leaf numbers per cell, ascending
    for (size_t f = 0; f < leaves.size(); f++) {
      const int v = ~leaves[f], slot0 = (v >> 2) * BVH_LEAF, cnt = (v & 3) + 1;
      std::vector<char> mark(cells, 0);
      for (int u = 0; u < cnt; u++) {
        const Sphere64& sp = bb.slot64[(size_t)slot0 + u];
        if (!(sp.r >= 0.0)) continue;
        const double w[3] = {sp.c[0] - L[0], sp.c[1] - L[1], sp.c[2] - L[2]};
        const double D = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        const double scale = std::fabs(L[0]) + std::fabs(L[1]) + std::fabs(L[2]) + std::fabs(sp.c[0]) +
                             std::fabs(sp.c[1]) + std::fabs(sp.c[2]) + sp.r;
        if (!(D > sp.r * (1.0 + 1e-9) + 1e-12 * scale) || !std::isfinite(D)) {   // the light in or on it
          std::fill(mark.begin(), mark.end(), 1);
          continue;
        }
        const double du[3] = {w[0] / D, w[1] / D, w[2] / D};
        const double alpha = std::asin(std::min(1.0, sp.r / D)) + 2.0 * DELTA;
        for (int face = 0; face < 6; face++)
          for (int bi = 0; bi < nb; bi++)
            for (int bj = 0; bj < nb; bj++) {
              const int blk = (face * nb + bi) * nb + bj;
              if (!within(du, &bctr[3 * (size_t)blk], alpha + brho[blk])) continue;
              for (int i = bi * B; i < (bi + 1) * B; i++)
                for (int j = bj * B; j < (bj + 1) * B; j++) {
                  const int cell = (face * n + i) * n + j;
                  if (!mark[cell] && within(du, &cctr[3 * (size_t)cell], alpha + crho[cell])) mark[cell] = 1;
                }
            }
      }
      for (int cell = 0; cell < cells; cell++)
        if (mark[cell]) in_cell[cell].push_back((int)f);
    }
    std::vector<uint16_t> off(cells + 1, 0);
    std::vector<uint16_t> list;
    for (int cell = 0; cell < cells; cell++) {
      off[cell] = (uint16_t)list.size();
      for (int f : in_cell[cell]) list.push_back((uint16_t)(int16_t)leaves[(size_t)f]);
      if (list.size() > 65535) return LightBuffer{};
    }
    off[cells] = (uint16_t)list.size();
    per[li] = off;
    per[li].insert(per[li].end(), list.begin(), list.end());
  }
  size_t stride = 0;
  for (const auto& v : per) stride = std::max(stride, v.size());
  stride = (stride + 7) & ~(size_t)7;               // (16-B aligned blocks)
  if (stride * (size_t)n_light > max_words) return LightBuffer{};
  lb.n = n;
  lb.stride = (int)stride;
  lb.words.assign(stride * (size_t)n_light, 0);
  for (int li = 0; li < n_light; li++) std::copy(per[li].begin(), per[li].end(), lb.words.begin() + stride * li);
  return lb;
}

}  // namespace rtx
