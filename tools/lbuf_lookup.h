// Host restatement of the device's light-buffer and raise-buffer lookups
// (rtx_device.h query_lbuf / raise_lbuf, float32 operations), shared by
// tools/lbuf_check.cpp (conservativeness checks) and tools/walk_sim.cpp (cost
// predictions).  Analysis code: not product code, not the oracle.
#pragma once
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../raytracing_rb_amd/csrc/rtx_bvh_build.h"

namespace lbuf_host {

// query_lbuf's cell of direction v (float32); -1: no usable cell
inline int device_cell(float vx, float vy, float vz, int n) {
  const float ax = fabsf(vx), ay = fabsf(vy), az = fabsf(vz);
  int face;
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
  const int i = std::min(std::max((int)floorf(fmaf(fs, h, 0.5f * (float)n)), 0), n - 1);
  const int j = std::min(std::max((int)floorf(fmaf(ft, h, 0.5f * (float)n)), 0), n - 1);
  return (face * n + i) * n + j;
}

// The device's shadow-walk lists for a target T and light L (d = L - T in
// binary64, as the device holds it): the light buffer's cell of -d (covers,
// and the raise check of regime A),
// then the raise buffer's B2 and B1 lists at that cell's parent and its M list
// at the parent of the cell of d, each read until its early exit (B2, M: q <
// ql; B1: q > ql; ql = 16 log2(l / floor)) and only when its gate opens.  fallback: the device walks the hierarchy instead
// (no usable cell, l below the floor or ql above 254).
struct Lists {
  bool fallback = false;
  std::vector<int32_t> cover, b2, b1, m;            // cover: leaf references; b2, b1, m: leaves or sphere slots
  int scanned = 0;                                  // raise-buffer entries read
};

inline Lists shadow_lists(const uint16_t* lblk, int nu, const uint32_t* rblk, const uint16_t* gates, int nc,
                          const double d[3], float floor2 = 0.0f, float lf2 = 0.0f, bool per_sphere = false) {
  Lists r;
  const float dx = (float)d[0], dy = (float)d[1], dz = (float)d[2];
  const int cu = device_cell(-dx, -dy, -dz, nu);
  if (cu < 0) {
    r.fallback = true;
    return r;
  }
  const uint16_t* ent = lblk + 6 * nu * nu + 1;
  for (int k = lblk[cu]; k < lblk[cu + 1]; k++) r.cover.push_back((int32_t)(int16_t)ent[k]);
  if (!rblk) return r;
  // rtx_device.h raise_qa: the bit-pattern bound of ql, then (gates open) the exact one
  const float dd = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
  int32_t bits;
  memcpy(&bits, &dd, 4);
  const float qa = 8.0f * (fmaf((float)bits, 1.0f / 8388608.0f, -127.0f) - lf2);
  if (!(dd >= floor2 * (1.0f + 2.1e-4f)) || !(qa + 0.7f <= 254.0f)) {
    r.fallback = true;
    return r;
  }
  const int m = nu / nc, cells = 6 * nc * nc;
  const int face = cu / (nu * nu), i = cu / nu % nu, j = cu % nu;
  const int pc = (face * nc + i / m) * nc + j / m, mc = ((face ^ 1) * nc + (nu - 1 - i) / m) * nc + (nu - 1 - j) / m;
  const uint32_t* off = rblk + 2;
  const uint32_t* re = rblk + rtx::rbuf_head(cells);
  const uint32_t gp = gates[pc], gm = gates[mc];
  const uint32_t g2 = gp & 31u, g1 = (gp >> 5) & 31u, gmm = (gm >> 10) & 31u;
  const float U = (float)rtx::GATE_UNIT;
  // (per-sphere lists, larger scenes: the device reads them without the gates)
  const bool open[3] = {per_sphere || g2 == 31u || qa <= U * (float)g2, per_sphere || qa + 0.7f >= U * (float)g1,
                        per_sphere || gmm == 31u || qa <= U * (float)gmm};
  if (!(open[0] || open[1] || open[2])) return r;
  const float ql = 8.0f * (log2f(dd) - lf2);
  for (int t = 0; t < 3; t++) {
    if (!open[t]) continue;
    const int c = t < 2 ? pc : mc;
    for (uint32_t k = off[t * (cells + 1) + c]; k < off[t * (cells + 1) + c + 1]; k++) {
      const uint32_t e = re[k];
      r.scanned++;
      const float q = (float)(e & 255u);
      if (t == 1 ? q > ql : q < ql) break;
      // (per-sphere lists: the entry is a sphere slot; else a leaf reference)
      (t == 0 ? r.b2 : t == 1 ? r.b1 : r.m).push_back(per_sphere ? (int32_t)(e >> 16) : (int32_t)(int16_t)(e >> 16));
    }
  }
  return r;
}

}  // namespace lbuf_host
