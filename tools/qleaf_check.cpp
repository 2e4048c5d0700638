// Host-only check of SPH_BVH_QLDS's 16-bit leaf records (tests/test_qleaf.py):
// reads "x y z r" lines, builds the hierarchy as rtx_scene_upload does (median
// or SAH, argv[1]), quantizes its leaves (quantize_leaves) and prints, per
// occupied slot, the true sphere and the float32 ball the device decodes
// (fmaf(q, step, org) per axis, q * rstep), as exact hex floats, then the
// scene's q_ok and max_err.  Links librtx's host code only (no GPU call).
#include "../raytracing_rb_amd/csrc/rtx_capi.cpp"

#include <iostream>

int main(int argc, char** argv) {
  using namespace rtx;
  const bool sah = argc > 1 && argv[1][0] == '1';
  std::vector<Sphere64> s64;
  std::vector<float> s32;
  std::vector<int32_t> obj;
  float scale = 0.0f;
  double x, y, z, r;
  while (std::cin >> x >> y >> z >> r) {
    Sphere64 s;
    s.c[0] = x, s.c[1] = y, s.c[2] = z, s.r = r;
    s64.push_back(s);
    for (float v : {(float)x, (float)y, (float)z, (float)(r * r)}) s32.push_back(v);
    obj.push_back((int)obj.size());
    const float sc = (float)((fabs(x) + fabs(y) + fabs(z) + fabs(r)) * (1.0 + 1e-6));   // as rtx_scene_upload
    if (sc > scale) scale = sc;
  }
  std::vector<BSph> bs(s64.size());
  for (size_t k = 0; k < s64.size(); k++) {
    for (int a = 0; a < 3; a++) bs[k].c[a] = s64[k].c[a];
    bs[k].r = s64[k].r;
    bs[k].rec = (int)k;
  }
  Bvh4Builder b{bs, s64, s32, obj};
  b.sah = sah;
  if (!bs.empty()) b.build(0, (int)bs.size(), 0);
  const QuantLeaves ql = quantize_leaves(b, scale);
  for (size_t k = 0; k < b.slot64.size(); k++) {
    const Sphere64& s = b.slot64[k];
    if (!(s.r >= 0.0)) continue;
    const uint32_t* w = ql.rec.data() + (k / BVH_LEAF) * 8;
    const int h = (int)(k % BVH_LEAF);
    auto q = [&](int comp) { return (w[comp * 2 + h / 2] >> (16 * (h % 2))) & 0xffffu; };
    const float dx = std::fmaf((float)q(0), ql.step[0], ql.org[0]), dy = std::fmaf((float)q(1), ql.step[1], ql.org[1]),
                dz = std::fmaf((float)q(2), ql.step[2], ql.org[2]), dr = (float)q(3) * ql.rstep;
    printf("%a %a %a %a %a %a %a %a\n", s.c[0], s.c[1], s.c[2], s.r, (double)dx, (double)dy, (double)dz, (double)dr);
  }
  printf("ok %d %a %a\n", ql.ok ? 1 : 0, ql.max_err, (double)scale);
  return 0;
}
