// rtx_bvh_build.h — host-only: the four-wide sphere hierarchy builder and
// the 16-bit leaf records of SPH_BVH_QLDS.
// Included by rtx_capi.cpp (rtx_scene_upload) and by tools/walk_sim.cpp, the
// CPU walk simulator, so both see the same trees.  No HIP calls.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <thread>
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

// The cube map of directions around a light shared by the light buffer and
// the raise buffer: 6 faces x n x n cells; the cell of direction v is on face
// 2a + (v_a < 0) of its dominant axis a, at i = floor((s + 1) n / 2),
// s = v_b / |v_a|, b = (a + 1) mod 3, likewise j for c = (a + 2) mod 3
// (query_lbuf's float32 lookup).  Each cell (and each block of B x B cells)
// keeps its center direction and its angular radius (from boundary samples).
struct CubeCells {
  int n = 0, cells = 0, B = 1, nb = 0;
  std::vector<double> cctr, crho, bctr, brho;
  static constexpr double PI = 3.141592653589793;

  static void dir(int face, double s, double t, double v[3]) {   // the direction of face `face` at (s, t)
    const int a = face >> 1, b = (a + 1) % 3, c = (a + 2) % 3;
    v[a] = (face & 1) ? -1.0 : 1.0;
    v[b] = s;
    v[c] = t;
    const double r = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    for (int k = 0; k < 3; k++) v[k] /= r;
  }
  static double angle(const double u[3], const double v[3]) {
    const double d = u[0] * v[0] + u[1] * v[1] + u[2] * v[2];
    return std::acos(std::max(-1.0, std::min(1.0, d)));
  }
  // a rectangle of face coordinates: its center direction and angular radius
  static double region(int face, double s0, double s1, double t0, double t1, double ctr[3]) {
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
  }
  explicit CubeCells(int n_) : n(n_), cells(6 * n_ * n_) {
    B = n % 8 == 0 ? n / 8 : (n % 4 == 0 ? n / 4 : 1);   // cells per block side
    nb = n / B;
    cctr.resize(3 * (size_t)cells), crho.resize(cells), bctr.resize(3 * (size_t)6 * nb * nb), brho.resize(6 * nb * nb);
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
  }
  static bool within(const double u[3], const double* c, double lim) {   // angle(u, c) <= lim
    if (lim >= PI) return true;
    return u[0] * c[0] + u[1] * c[1] + u[2] * c[2] >= std::cos(lim);
  }
  // every cell whose region comes within `lim` of direction u (blocks first)
  template <typename F>
  void visit(const double u[3], double lim, F&& f) const {
    for (int face = 0; face < 6; face++)
      for (int bi = 0; bi < nb; bi++)
        for (int bj = 0; bj < nb; bj++) {
          const int blk = (face * nb + bi) * nb + bj;
          if (!within(u, &bctr[3 * (size_t)blk], lim + brho[blk])) continue;
          for (int i = bi * B; i < (bi + 1) * B; i++)
            for (int j = bj * B; j < (bj + 1) * B; j++) {
              const int cell = (face * n + i) * n + j;
              if (within(u, &cctr[3 * (size_t)cell], lim + crho[cell])) f(cell);
            }
        }
  }
  // the least angle between u and a direction of `cell` (0 when u is inside)
  double gap(const double u[3], int cell) const {
    return std::max(0.0, angle(u, &cctr[3 * (size_t)cell]) - crho[cell]);
  }
  // the largest
  double gapmax(const double u[3], int cell) const {
    return std::min(PI, angle(u, &cctr[3 * (size_t)cell]) + crho[cell]);
  }
};

// Every leaf reference of the hierarchy (int16 list entries: at most 8,192
// leaves, since a reference is ~((leaf << 2) | (count - 1)) >= -32768); empty
// when some reference does not fit.
inline std::vector<int32_t> leaf_refs(const Bvh4Builder& bb, int root) {
  std::vector<int32_t> leaves;
  if (root < 0 && root != BVH_NONE) leaves.push_back(root);
  for (const Bvh4Node& nd : bb.nodes)
    for (int k = 0; k < 4; k++)
      if (nd.child[k] < 0 && nd.child[k] != BVH_NONE) leaves.push_back(nd.child[k]);
  for (int32_t ref : leaves)
    if (ref < -32768) return {};
  return leaves;
}

// Light buffer: for each light, a cube map of 6 x n x n cells
// around its position; cell c lists the hierarchy's leaves that hold a sphere
// whose disc, as seen from the light, meets the cell.  A sphere that covers a
// shadow ray's target T (World#lit_area: it crosses the segment from T to the
// light L, short of L) meets the ray from L towards T, so its disc holds that
// direction and its leaf is in the direction's cell: the shadow walk visits
// those leaves only, with the same leaf tests.  The discs are widened by
// DELTA radians, far more than the float32 cell lookup's error (CubeCells);
// a light inside or on a sphere puts that sphere's leaf in every cell.
// Layout per light (uint16 words, `stride` per light): 6 n n + 1 offsets into
// the light's leaf list, then the list (leaf references, int16).
struct LightBuffer {
  int n = 0, stride = 0;
  std::vector<uint16_t> words;
};

inline LightBuffer build_light_buffer(const Bvh4Builder& bb, int root, const double (*lpos)[3], int n_light, int n,
                                      size_t max_words, const double* lrad = nullptr) {
  LightBuffer lb;
  if (n_light <= 0 || root == BVH_NONE || n <= 0) return lb;
  // the offsets alone must fit (skip a resolution before building it)
  if ((size_t)(6 * n * n + 1) * (size_t)n_light > max_words) return lb;
  const std::vector<int32_t> leaves = leaf_refs(bb, root);
  if (leaves.empty()) return lb;
  const double DELTA = 1e-4;
  const CubeCells cc(n);
  const int cells = cc.cells;
  std::vector<std::vector<uint16_t>> per(n_light);
  size_t total = 0;
  for (int li = 0; li < n_light; li++) {
    const double* L = lpos[li];
    const double rad_pad = lrad && std::isfinite(lrad[li]) ? std::fabs(lrad[li]) : 0.0;
    std::vector<std::vector<int>> in_cell(cells);   // leaf numbers per cell, ascending
    std::vector<char> mark(cells, 0);
    for (size_t f = 0; f < leaves.size(); f++) {
      const int v = ~leaves[f], slot0 = (v >> 2) * BVH_LEAF, cnt = (v & 3) + 1;
      std::fill(mark.begin(), mark.end(), 0);
      for (int u = 0; u < cnt; u++) {
        const Sphere64& sp = bb.slot64[(size_t)slot0 + u];
        if (!(sp.r >= 0.0)) continue;
        const double w[3] = {sp.c[0] - L[0], sp.c[1] - L[1], sp.c[2] - L[2]};
        const double D = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        const double scale = std::fabs(L[0]) + std::fabs(L[1]) + std::fabs(L[2]) + std::fabs(sp.c[0]) +
                             std::fabs(sp.c[1]) + std::fabs(sp.c[2]) + sp.r + rad_pad;
        if (!(D > sp.r + 1e-6 * scale) || !std::isfinite(D)) {   // the light in, on or next to it
          std::fill(mark.begin(), mark.end(), 1);
          continue;
        }
        const double du[3] = {w[0] / D, w[1] / D, w[2] / D};
        // the disc (sin <= R / D), with the raise buffer's slack 1e-9 S / D: the
        // cells also serve its regime (A) (build_raise_buffer)
        const double alpha = std::asin(std::min(1.0, sp.r / D + 1e-9 * scale / D)) + 2.0 * DELTA;
        cc.visit(du, alpha, [&](int cell) { mark[cell] = 1; });
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
    total += per[li].size();
    if (total > max_words) return LightBuffer{};   // (stop once the lights so far cannot fit)
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

// Raise buffer: which spheres (per-sphere lists, larger
// scenes) or leaves can hold a sphere whose Sphere#cover_area (sphere.rb:28-57)
// raises Math::DomainError for a target T and light (L, radius), whatever its
// binary factor.  The raise needs d within a few ulps of |R - r1| (d: the
// distance of the center C from the line through T and L; r1 = radius |s_T| /
// l, the cone's radius at C's projection, s_T its signed distance from T along
// the line, l = |L - T|).  Let w be the unit direction from L towards T,
// sigma = (C - L).w = D cos(theta) with D = |C - L| and theta the angle of
// C - L from w (from -w when sigma < 0), so d = D sin(theta):
//   (A) R > r1, d ~ R - r1 <= R: the line meets the ball (the light buffer's
//       cells, whose discs include this slack, for sigma > 0; list M, always,
//       for sigma < 0);
//   (B) r1 > R, d ~ r1 - R, i.e. h(theta, l) = d - r1 + R ~ 0 with
//     B2, sigma > l:  h2 = D sin + R + radius - radius D cos / l (increasing in
//         theta and in l),
//     B1, 0 <= sigma <= l:  h1 = D sin + R - radius + radius D cos / l
//         (concave in theta, decreasing in l),
//     BM, sigma < 0:  hm = D sin + R - radius - radius D cos / l (increasing
//         in theta and in l).
// Over a cell's directions theta ranges over [ta, tb] (the sphere direction's
// least and largest angle to the cell, widened by 2 DELTA: the lookup's slack,
// as the light buffer's), so some theta has |h| <= ep only for l in an
// interval: B2 [radius D cos tb / (D sin tb + R + radius + ep), radius D cos ta
// / (D sin ta + R + radius - ep)]; B1 from the least of radius D cos t / (radius
// - R - D sin t + ep) over t = ta, tb (h1's minimum is at an end) up to radius
// D cos ta / (radius - R - D sin tb - ep) (its maximum is below D sin tb +
// radius D cos ta / l - radius + R); BM [radius D cos tb / (D sin tb - radius +
// R + ep), radius D cos ta / (D sin ta - radius + R - ep)], each bound open
// where its denominator has no sign.  ep = 1e-9 S (S: the coordinates' scale:
// d and r1 are computed to a few ulps of S, a raise needs them within a few
// ulps of tangency); a light within 1e-6 S of a sphere's surface puts that
// sphere in every cell.  Bounds below `floor` (per light) are cut: a query with
// l < floor walks the hierarchy instead.
// Three lists per cell (n cells per face side; the light buffer's n is a
// multiple, and its cell's parent is looked up): B2 and M sorted by their upper
// bound, descending, B1 by its lower bound, ascending (a query reads a list
// until its key leaves ql; the entry keeps its other bound too, which the
// device does not test: skipping by it cost more than the tests it saved),
// with ql = 16 log2(l / floor), upper bounds rounded up (255: unbounded) and
// lower ones down (0: the floor); a query with ql > 254 walks the hierarchy.
// Layout per light (uint32 words, `stride` per light): word 0 the floor (float,
// rounded up), word 1 the entry count, 3 (6 n n + 1) offsets (B2's cells, B1's,
// M's, counting entries from the list start), then from word rbuf_head the
// entries: sphere slot or leaf reference (16 bits) << 16 | the other bound << 8
// | the sort key.  Each list starts at a multiple of 4 entries; the words up to
// the next list's start hold keys that end any read (0 in B2 / M, 255 in B1).
struct RaiseBuffer {
  int n = 0, stride = 0;
  std::vector<uint32_t> words;
};

enum { RB_B2 = 0, RB_B1 = 1, RB_M = 2, RB_LISTS = 3 };

inline RaiseBuffer build_raise_buffer(const Bvh4Builder& bb, int root, const double (*lpos)[3], const double* lrad,
                                      const double* lfloor, int n_light, int n, size_t max_words,
                                      std::vector<double>* floors_used = nullptr, bool per_sphere = false,
                                      int max_doublings = 31) {
  RaiseBuffer rb;
  if (n_light <= 0 || root == BVH_NONE || n <= 0) return rb;
  const int cells = 6 * n * n;
  const size_t head = rbuf_head(cells);
  if (head * (size_t)n_light > max_words) return rb;
  const std::vector<int32_t> leaves = leaf_refs(bb, root);
  if (leaves.empty()) return rb;
  if (per_sphere && leaves.size() * BVH_LEAF > 65536) return rb;   // (16-bit slot indices)
  const double DELTA = 1e-4, PI = CubeCells::PI, QMAX = 254.0 / 16.0;
  const CubeCells cc(n);
  std::vector<std::vector<uint32_t>> per(n_light);
  if (floors_used) floors_used->assign(n_light, 0.0);
  size_t total = 0;
  auto as = [PI](double x) { return x >= 1.0 ? PI / 2 : (x <= 0.0 ? 0.0 : std::asin(x)); };
  for (int li = 0; li < n_light; li++) {
    const double* L = lpos[li];
    const double rad = lrad[li];
    double floor_l = std::max(0.0, lfloor[li]);
    if (!(floor_l > 1e-6 * rad)) floor_l = 1e-6 * rad;
    std::vector<uint32_t> blk;
    for (int attempt = 0; attempt <= max_doublings; attempt++, floor_l *= 2.0) {
      blk.clear();
      if (!(rad > 0.0) || !std::isfinite(rad)) {      // a point light: no cover_area raises (r1 = 0)
        blk.assign(head, 0);
        break;
      }
      auto q_up = [&](double l2) -> uint32_t {        // ceil(16 log2(l2 / floor)), 255: always
        if (!(l2 < floor_l * std::exp2(QMAX))) return 255u;
        const double q = std::ceil(16.0 * std::log2(std::max(l2 * (1.0 + 1e-4) / floor_l, 1.0)));
        return (uint32_t)std::min(254.0, q);
      };
      auto q_lo = [&](double l1) -> uint32_t {        // floor(16 log2(l1 / floor)), 0 at or below it, 255: never
        if (!(l1 < floor_l * std::exp2(QMAX))) return 255u;
        if (!(l1 * (1.0 - 1e-4) > floor_l)) return 0u;
        return (uint32_t)std::max(0.0, std::floor(16.0 * std::log2(l1 * (1.0 - 1e-4) / floor_l)));
      };
      // The units' entries, in unit order: units split into contiguous ranges over up
      // to 16 threads (a large scene's finer cells take seconds on one), each with its
      // own interval scratch, each range's entries kept as (list, entry) pairs and
      // gathered per list in range order: the lists are those of one thread.
      const size_t units = per_sphere ? leaves.size() * BVH_LEAF : leaves.size();
      const size_t nth = std::max<size_t>(1, std::min<size_t>({16, (size_t)std::max(1u, std::thread::hardware_concurrency()),
                                                                (units + 255) / 256}));
      std::vector<std::vector<std::pair<uint32_t, uint32_t>>> outs(nth);
      auto run = [&](size_t th) {
        // per cell: the unit's combined l-intervals per list (the hull of its spheres')
        std::vector<double> ilo[RB_LISTS], ihi[RB_LISTS];
        for (int t = 0; t < RB_LISTS; t++) ilo[t].assign(cells, INFINITY), ihi[t].assign(cells, -1.0);
        std::vector<int> touched;
        std::vector<char> seen(cells, 0);
        auto& out = outs[th];
        const size_t f0 = units * th / nth, f1 = units * (th + 1) / nth;
        // entries per sphere (slot index), or per leaf (reference): the device's choice
        for (size_t f = f0; f < f1; f++) {
          const int lf = (int)(per_sphere ? f / BVH_LEAF : f);
          const int v = ~leaves[lf], slot0 = (v >> 2) * BVH_LEAF, cnt0 = (v & 3) + 1;
          const int u0 = per_sphere ? (int)(f % BVH_LEAF) : 0, cnt = per_sphere ? (u0 < cnt0 ? u0 + 1 : 0) : cnt0;
          touched.clear();
          auto note = [&](int cell, int t, double lo, double hi) {   // needed for l in [lo, hi]
            if (!(lo <= hi) || !(hi >= floor_l)) return;
            if (!seen[cell]) seen[cell] = 1, touched.push_back(cell);
            ilo[t][cell] = std::min(ilo[t][cell], lo);
            ihi[t][cell] = std::max(ihi[t][cell], hi);
          };
          for (int u = u0; u < cnt; u++) {
            const Sphere64& sp = bb.slot64[(size_t)slot0 + u];
            if (!(sp.r >= 0.0)) continue;
            const double R = sp.r;
            const double w[3] = {sp.c[0] - L[0], sp.c[1] - L[1], sp.c[2] - L[2]};
            const double D = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
            const double scale = std::fabs(L[0]) + std::fabs(L[1]) + std::fabs(L[2]) + std::fabs(sp.c[0]) +
                                 std::fabs(sp.c[1]) + std::fabs(sp.c[2]) + R + rad;
            if (!(D > R + 1e-6 * scale) || !std::isfinite(D)) {   // the light in, on or next to it: every cell
              for (int cell = 0; cell < cells; cell++) note(cell, RB_M, 0.0, INFINITY);
              continue;                                 // (P: the light buffer lists it in every cell)
            }
            const double du[3] = {w[0] / D, w[1] / D, w[2] / D};
            const double ep = 1e-9 * scale;             // d and r1's tolerance (distance)
            const double kf = rad / floor_l;            // k at the floor: the widest reach
            const double reach = std::max({as((R + ep) / D), as((rad - R + ep) / D), as(kf), as((rad - R + ep) / D + kf)}) +
                                 2.0 * DELTA;
            cc.visit(du, reach, [&](int cell) {
              // theta, the angle of C - L from the axis direction (w for P's cells, -w for M's),
              // ranges over [ta, tb] for the cell's directions (with the lookup's slack)
              const double ta = std::max(0.0, cc.gap(du, cell) - 2.0 * DELTA);
              if (ta >= PI / 2) return;
              const double tb = std::min(PI / 2, cc.gapmax(du, cell) + 2.0 * DELTA);
              const double sa = std::sin(ta), ca = std::cos(ta), sb = std::sin(tb), cb = std::cos(tb);
              const double k1 = rad * D;                // (radius D cos(theta) / l: the cone's share of h)
              // B2: h2 = D sin - k1 cos / l + radius + R, increasing in theta and l
              {
                const double a = D * sa + rad + R - ep, b = D * sb + rad + R + ep;
                note(cell, RB_B2, k1 * cb / b, a <= 0.0 ? INFINITY : k1 * ca / a);
              }
              // B1: h1 = D sin + k1 cos / l - radius + R, concave in theta, decreasing in l
              {
                auto lower = [&](double st, double ct) {   // h1(theta, l) <= ep from this l on
                  const double r = rad - R - D * st + ep;
                  return r < 0.0 ? INFINITY : (ct <= 0.0 ? 0.0 : (r == 0.0 ? INFINITY : k1 * ct / r));
                };
                const double lo = std::min(lower(sa, ca), lower(sb, cb));
                const double r = rad - R - D * sb - ep;   // max h1 <= D sin(tb) + k1 cos(ta) / l - radius + R
                note(cell, RB_B1, lo, r <= 0.0 ? INFINITY : k1 * ca / r);
              }
              // M: regime A (the line through the ball beyond the light) always; BM: hm = D sin -
              // k1 cos / l - radius + R, increasing in theta and l
              if (D * sa <= R + ep) {
                note(cell, RB_M, 0.0, INFINITY);
              } else {
                const double a = D * sa - rad + R - ep, b = D * sb - rad + R + ep;
                if (b >= 0.0) note(cell, RB_M, cb <= 0.0 ? 0.0 : (b == 0.0 ? INFINITY : k1 * cb / b),
                                   a <= 0.0 ? INFINITY : k1 * ca / a);
              }
            });
          }
          const uint32_t ref = per_sphere ? (uint32_t)(((~leaves[lf]) >> 2) * BVH_LEAF + (int)(f % BVH_LEAF)) << 16
                                          : (uint32_t)(uint16_t)(int16_t)leaves[f] << 16;
          for (int cell : touched) {
            seen[cell] = 0;
            for (int t = 0; t < RB_LISTS; t++) {
              if (ihi[t][cell] >= floor_l && ilo[t][cell] <= ihi[t][cell]) {
                const uint32_t qh = q_up(ihi[t][cell]), qlo = q_lo(ilo[t][cell]);
                if (qlo != 255u && qlo <= qh) {
                  // the sort key in bits 0-7 (B1: the lower bound, else the upper), the other bound in 8-15
                  const uint32_t key = t == RB_B1 ? qlo : qh, oth = t == RB_B1 ? qh : qlo;
                  out.emplace_back((uint32_t)(t * cells + cell), ref | oth << 8 | key);
                }
              }
              ilo[t][cell] = INFINITY, ihi[t][cell] = -1.0;
            }
          }
        }
      };
      if (nth == 1) {
        run(0);
      } else {
        std::vector<std::thread> pool;
        for (size_t th = 0; th < nth; th++) pool.emplace_back(run, th);
        for (auto& th : pool) th.join();
      }
      // the lists in layout order (list t, cell): a counting pass, the entries placed in
      // range order (so unit order within a list), then each list sorted by its key
      // (each list starts at a multiple of 4 entries; the gap to the next list's start holds
      // entries whose key ends every query's read: 0 in B2 / M, 255 in B1)
      const size_t nlist = (size_t)RB_LISTS * cells;
      std::vector<uint32_t> at(nlist + 1, 0u), cnt(nlist, 0u);
      for (const auto& out : outs)
        for (const auto& pe : out) cnt[pe.first]++;
      for (size_t q = 0; q < nlist; q++) at[q + 1] = at[q] + ((cnt[q] + 3u) & ~3u);
      const size_t nent = at[nlist];
      if (head + nent > max_words) continue;          // too large: raise the floor
      blk.assign(head + nent, 0);
      float ff = (float)floor_l;
      if ((double)ff < floor_l) ff = nextafterf(ff, INFINITY);
      memcpy(&blk[0], &ff, 4);
      blk[1] = (uint32_t)nent;
      uint32_t* off = &blk[2];
      for (int t = 0; t < RB_LISTS; t++) {
        for (int cell = 0; cell < cells; cell++) off[t * (cells + 1) + cell] = at[(size_t)t * cells + cell];
        off[t * (cells + 1) + cells] = at[(size_t)(t + 1) * cells];
      }
      {
        std::vector<uint32_t> cur(at.begin(), at.end() - 1);
        uint32_t* ent = &blk[head];
        for (const auto& out : outs)
          for (const auto& pe : out) ent[cur[pe.first]++] = pe.second;
        for (size_t q = 0; q < nlist; q++)
          for (uint32_t k = at[q] + cnt[q]; k < at[q + 1]; k++) ent[k] = q / cells == RB_B1 ? 255u : 0u;
      }
      outs.clear();
      auto sort_lists = [&](size_t q0, size_t q1) {   // (stable: ties keep unit order)
        uint32_t* ent = &blk[head];
        for (size_t q = q0; q < q1; q++) {
          uint32_t *x0 = ent + at[q], *x1 = ent + at[q] + cnt[q];
          if (x1 - x0 < 2) continue;
          if (q / cells == RB_B1)
            std::stable_sort(x0, x1, [](uint32_t a, uint32_t b) { return (a & 255u) < (b & 255u); });
          else
            std::stable_sort(x0, x1, [](uint32_t a, uint32_t b) { return (a & 255u) > (b & 255u); });
        }
      };
      if (nth == 1) {
        sort_lists(0, nlist);
      } else {
        std::vector<std::thread> pool;
        for (size_t th = 0; th < nth; th++) pool.emplace_back(sort_lists, nlist * th / nth, nlist * (th + 1) / nth);
        for (auto& th : pool) th.join();
      }
      break;
    }
    if (blk.empty()) return RaiseBuffer{};
    if (floors_used) (*floors_used)[li] = floor_l;
    total += blk.size();
    if (total > max_words) return RaiseBuffer{};
    per[li].swap(blk);
  }
  size_t stride = 0;
  for (const auto& v : per) stride = std::max(stride, v.size());
  stride = (stride + 3) & ~(size_t)3;               // (16-B aligned blocks)
  if (stride * (size_t)n_light > max_words) return RaiseBuffer{};
  rb.n = n;
  rb.stride = (int)stride;
  rb.words.assign(stride * (size_t)n_light, 0);
  for (int li = 0; li < n_light; li++) std::copy(per[li].begin(), per[li].end(), rb.words.begin() + stride * li);
  return rb;
}

// The raise buffer's gates: one 16-bit word per light and raise-buffer cell
// summarising the q of the first entry of each list in 5-bit fields of
// GATE_UNIT q units (an eighth of an octave of l): bits 0-4 g2 = ceil(q /
// unit) of B2's (0 when empty), bits 5-9 g1 = floor(q / unit) of B1's (31 when
// empty), bits 10-14 gm = ceil(q / unit) of M's (0 when empty), each clamped
// to 31.  A query reads the lists only when ql <= unit g2 or ql >= unit g1
// (P), or ql <= unit gm (M), a field of 31 in g2 / gm opening always (a
// threshold beyond 2^3.9 floors): small scenes stage the gates in LDS and
// rarely touch the lists (ql > 0 always).
inline uint16_t gate_word(uint32_t q2, uint32_t q1, uint32_t qm) {
  auto up = [](uint32_t q) { return std::min<uint32_t>(31u, (q + GATE_UNIT - 1) / GATE_UNIT); };
  return (uint16_t)(up(q2) | (std::min<uint32_t>(31u, q1 / GATE_UNIT) << 5) | (up(qm) << 10));
}
inline bool gate_open(uint16_t g, int t, float ql) {   // (the device's test, rtx_device.h raise_lists)
  const uint32_t f = (g >> (5 * t)) & 31u;
  return t == 1 ? ql >= (float)(GATE_UNIT * f) : (f == 31u || ql <= (float)(GATE_UNIT * f));
}

// A light's floor^2 rounded up and log2 floor^2 (the gate block's header;
// rtx_device.h raise_qa / raise_rq).  ql = 8 (log2 |d|^2 - log2 floor^2) is
// 16 log2(l / floor) to float rounding, far inside the 1e-4 slack of the q's.
inline float raise_floor2(const RaiseBuffer& rb, int li) {
  float fl;
  memcpy(&fl, &rb.words[(size_t)rb.stride * li], 4);
  const double f2 = (double)fl * (double)fl;
  float r = (float)f2;
  if ((double)r < f2) r = nextafterf(r, INFINITY);
  return r;
}
inline float raise_lf2(const RaiseBuffer& rb, int li) {
  float fl;
  memcpy(&fl, &rb.words[(size_t)rb.stride * li], 4);
  return (float)(2.0 * std::log2((double)fl));
}

inline std::vector<uint16_t> raise_gates(const RaiseBuffer& rb, int n_light) {
  std::vector<uint16_t> g;
  if (!rb.n) return g;
  const int cells = 6 * rb.n * rb.n;
  g.assign((size_t)cells * n_light, 0);
  for (int li = 0; li < n_light; li++) {
    const uint32_t* blk = rb.words.data() + (size_t)rb.stride * li;
    const uint32_t* off = blk + 2;
    const uint32_t* ent = blk + rbuf_head(cells);
    for (int c = 0; c < cells; c++) {
      uint32_t q[RB_LISTS];
      for (int t = 0; t < RB_LISTS; t++) {
        const uint32_t k0 = off[t * (cells + 1) + c], k1 = off[t * (cells + 1) + c + 1];
        q[t] = k1 > k0 ? (ent[k0] & 255u) : (t == RB_B1 ? 255u : 0u);
      }
      g[(size_t)cells * li + c] = gate_word(q[RB_B2], q[RB_B1], q[RB_M]);
    }
  }
  return g;
}

}  // namespace rtx
