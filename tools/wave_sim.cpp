// wave_sim.cpp — CPU emulation of the level engine's wave occupancy (analysis
// tool; not product code, not the oracle).  It reuses walk_sim.cpp's scene
// loader, host hierarchy builder and binary64 geometry, traces ray trees level
// by level in the order the level engine holds them, and runs each 64-ray
// chunk's hierarchy walk as one wave would: every lane's stack, the
// speculative traversal of query_bvh (rtx_device.h: a lane that reaches a leaf
// holds it while the wave's other lanes search on; leaves are tested once every
// searching lane holds one), the leaf phase with its per-slot exact tests.
// Per wave step it counts the lanes that execute, so the walks' lane occupancy
// (active lanes per executed step) and a time proxy (steps x their cost) can be
// compared across ray orderings and walk policies without a GPU:
//
//   order  base     parent order (the level engine's slices, hits in ray order);
//          oct      children bucketed by direction octant (stable);
//          morton   sorted by the Morton code of the origin (scene box, 10 bits/axis);
//          octm     sorted by (octant, Morton of origin);
//   walk   spec     speculative traversal (the shipped walk);
//          nospec   while-while without holding leaves;
//          spec75   spec, leaves tested once 3/4 of the searching lanes hold one.
//
// Level 0 follows decode_item (rtx_device.h): 8x8 tiles, Morton pixel order in
// a tile, pre samples per pixel (lens jitter on the aperture disk).
//
//   g++ -O2 -std=c++17 -o tools/wave_sim tools/wave_sim.cpp -lz
//   tools/wave_sim scenes/c2_world.yml scenes/c2_camera.yml [tile_step] [max_rays_per_level]
#define WALK_SIM_NO_MAIN
#include "walk_sim.cpp"

#include <algorithm>
#include <array>
#include <functional>

namespace {

// step costs in VALU instructions per lane (rough counts from the ISA of k_level_c):
// an inner node (fetch, 4 slab tests, sort, pushes), a leaf's float pre-test of
// its 4 spheres, one binary64 exact sphere test
constexpr double C_LEAF = 70, C_EXACT = 160;
// (WAVE_SIM_NODE_COST: another per-node cost, e.g. a node format that decodes its boxes)
const double C_NODE = getenv("WAVE_SIM_NODE_COST") ? atof(getenv("WAVE_SIM_NODE_COST")) : 60.0;

struct Occ {
  double steps[3] = {0, 0, 0}, lanes[3] = {0, 0, 0}, waves = 0, exact_ideal = 0;
  void add(const Occ& o) {
    for (int k = 0; k < 3; k++) steps[k] += o.steps[k], lanes[k] += o.lanes[k];
    waves += o.waves;
    exact_ideal += o.exact_ideal;
  }
  double time() const { return steps[0] * C_NODE + steps[1] * C_LEAF + steps[2] * C_EXACT; }
  double occ() const {
    const double w = lanes[0] * C_NODE + lanes[1] * C_LEAF + lanes[2] * C_EXACT;
    return time() > 0 ? w / time() : 0;
  }
};

enum Walk { SPEC = 0, NOSPEC, SPEC75, NWALK };
const char* walk_name[NWALK] = {"spec", "nospec", "spec75"};

struct Lane {
  bool ext = true;
  V3 o, d;
  RayF r;
  float thi = 0;
  double best = INFINITY;
  int besti = -1;
  bool inside = false;
  int ref = BVH_NONE, pend = BVH_NONE;
  std::vector<int> stk;
  int pop() {
    if (stk.empty()) return BVH_NONE;
    const int v = stk.back();
    stk.pop_back();
    return v;
  }
};

// planes first (walk_planes_boxes), then the hierarchy
void lane_start(const Sim& S, Lane& L, bool ext, V3 o, V3 d) {
  L.ext = ext, L.o = o, L.d = d;
  L.r = rayf(S, o, d);
  L.best = INFINITY, L.besti = -1, L.inside = false;
  L.stk.clear();
  L.pend = BVH_NONE;
  const double D = sqrt(vdot(d, d));
  if (ext) {
    for (size_t i = 0; i < S.obj.size(); i++) {
      if (S.obj[i].type != RTX_PLANE) continue;
      double t;
      if (plane_hit(S.obj[i], o, d, t) && t < L.best && vr(vsc(d, t)) < S.maxd) L.best = t, L.besti = (int)i;
    }
    L.thi = std::isfinite(L.best) ? (float)(L.best * (1 + 1e-6)) : INFINITY;
  } else {
    L.thi = 1.0f + 1e-5f + L.r.mS / (float)D;
  }
  L.ref = S.root;
}

void lane_node(const Sim& S, Lane& L) {
  const Bvh4Node& n = S.bb->nodes[L.ref];
  float key[4];
  int ch[4];
  for (int k = 0; k < 4; k++) {
    ch[k] = n.child[k];
    key[k] = INFINITY;
    if (ch[k] == BVH_NONE) continue;
    const float lo[3] = {n.lh[0][k][0], n.lh[1][k][0], n.lh[2][k][0]};
    const float hi[3] = {n.lh[0][k][1], n.lh[1][k][1], n.lh[2][k][1]};
    key[k] = slab(L.r, lo, hi, L.r.mS, 0.0f, L.thi);
  }
  int idx[4] = {0, 1, 2, 3};
  std::sort(idx, idx + 4, [&](int a, int b) { return key[a] < key[b]; });
  for (int k = 3; k >= 1; k--)
    if (key[idx[k]] < INFINITY) L.stk.push_back(ch[idx[k]]);
  L.ref = key[idx[0]] < INFINITY ? ch[idx[0]] : L.pop();
}

// the leaf's float pre-test; returns the slots that go to the binary64 test
// (EXTEND: the line within the sphere's radius + margin inside [0, thi];
// SHADOW: the segment crosses the sphere), and does those tests
int lane_leaf(const Sim& S, Lane& L, int lf) {
  const int v = ~lf, slot0 = (v >> 2) * BVH_LEAF, cnt = (v & 3) + 1;
  int mask = 0;
  for (int u = 0; u < cnt; u++) {
    const Sphere64& s = S.bb->slot64[slot0 + u];
    const V3 C = v3p(s.c);
    const V3 oc = vsub(C, L.o);
    const double dd = vdot(L.d, L.d), t = vdot(oc, L.d) / dd;
    const double nd = vr(vsub(vadd(L.o, vsc(L.d, t)), C));
    const double rel = s.r * (1 + 1e-5) + 1e-5 * vr(oc);
    const double h = s.r / sqrt(dd);
    if (!(nd <= rel) || t + h < 0 || t - h > L.thi) continue;
    mask |= 1 << u;
    double th;
    bool in;
    if (L.ext && sphere_hit(s, L.o, L.d, th, in) && th < L.best) {
      L.best = th, L.besti = S.bb->slot_obj[slot0 + u], L.inside = in;
      L.thi = (float)(th * (1 + 1e-6));
    } else if (!L.ext && sphere_hit(s, L.o, L.d, th, in) && th < 1.0) {
      if (th < L.best) L.best = th, L.besti = S.bb->slot_obj[slot0 + u];
    }
  }
  return mask;
}

// one wave: lanes.size() <= 64
Occ run_wave(const Sim& S, std::vector<Lane>& lanes, Walk w) {
  Occ oc;
  oc.waves = 1;
  const int n = (int)lanes.size();
  const bool spec = w != NOSPEC;
  auto active = [&](const Lane& L) { return L.ref != BVH_NONE || L.pend != BVH_NONE; };
  for (;;) {
    bool any = false;
    for (Lane& L : lanes) any |= active(L);
    if (!any) break;
    std::vector<int> act;
    for (int i = 0; i < n; i++)
      if (active(lanes[i])) act.push_back(i);
    if (spec)
      for (int i : act) {
        Lane& L = lanes[i];
        if (L.ref < 0 && L.ref != BVH_NONE && L.pend == BVH_NONE) L.pend = L.ref, L.ref = L.pop();
      }
    std::vector<int> in;
    for (int i : act)
      if (lanes[i].ref >= 0 && lanes[i].ref != BVH_NONE) in.push_back(i);
    for (;;) {
      std::vector<int> still;
      for (int i : in)
        if (lanes[i].ref >= 0 && lanes[i].ref != BVH_NONE) still.push_back(i);
      in.swap(still);
      if (in.empty()) break;
      if (spec) {
        int holding = 0;
        for (int i : in) holding += lanes[i].pend != BVH_NONE;
        if (holding == (int)in.size()) break;
        if (w == SPEC75 && 4 * holding >= 3 * (int)in.size()) break;
      }
      oc.steps[0]++;
      oc.lanes[0] += in.size();
      for (int i : in) {
        Lane& L = lanes[i];
        lane_node(S, L);
        if (spec && L.ref < 0 && L.ref != BVH_NONE && L.pend == BVH_NONE) L.pend = L.ref, L.ref = L.pop();
      }
    }
    // leaf phase
    std::vector<std::pair<int, int>> lf;
    for (int i : act) {
      Lane& L = lanes[i];
      int leaf;
      if (spec) {
        leaf = L.pend;
        L.pend = BVH_NONE;
      } else {
        if (L.ref == BVH_NONE) continue;
        leaf = L.ref;
      }
      if (leaf != BVH_NONE) lf.push_back({i, leaf});
    }
    if (!lf.empty()) {
      oc.steps[1]++;
      oc.lanes[1] += lf.size();
      // the exact tests: each lane loops over its own kept spheres (walk_leaf's
      // while (keep)), so the wave runs max over lanes of their count passes
      int passes = 0, total = 0;
      for (auto& [i, leaf] : lf) {
        const int n = __builtin_popcount(lane_leaf(S, lanes[i], leaf));
        passes = std::max(passes, n);
        total += n;
      }
      oc.steps[2] += passes;
      oc.lanes[2] += total;
      oc.exact_ideal += (total + 63) / 64;       // (candidates compacted across the wave)
    }
    if (!spec)
      for (auto& [i, leaf] : lf) lanes[i].ref = lanes[i].pop();
  }
  return oc;
}

struct WRay {
  V3 o, d, att;
  int depth;
  uint32_t key = 0;
};

uint32_t spread10(uint32_t x) {
  x &= 1023;
  x = (x | (x << 16)) & 0x030000FF;
  x = (x | (x << 8)) & 0x0300F00F;
  x = (x | (x << 4)) & 0x030C30C3;
  x = (x | (x << 2)) & 0x09249249;
  return x;
}

enum Order { BASE = 0, OCT, MORTON, OCTM, W128, W256, W512, W4096, M6, M9, M12, O_M6, O_M9, O_M12, D6_M6, NORDER };
const char* order_name[NORDER] = {"base", "oct", "morton", "octm", "w128", "w256", "w512", "w4096",
                                  "m6", "m9", "m12", "o+m6", "o+m9", "o+m12", "d6+m6"};

// the key of a ray: (direction octant, Morton code of the origin in the scene box)
uint32_t ray_key(const Sim& S, const WRay& r, bool oct_only, bool morton_only) {
  const uint32_t oct = (r.d.x < 0) | ((r.d.y < 0) << 1) | ((r.d.z < 0) << 2);
  uint32_t m = 0;
  const double p[3] = {r.o.x, r.o.y, r.o.z};
  for (int a = 0; a < 3; a++) {
    const double lo = S.root_c[a] - S.root_h[a], w = 2.0 * S.root_h[a];
    const double f = std::min(std::max((p[a] - lo) / w, 0.0), 0.999999);
    m |= spread10((uint32_t)(f * 1024)) << a;
  }
  return oct_only ? oct : morton_only ? m : (oct << 29) | (m >> 3);
}

// whole-level orders, coarse buckets (mN, o+mN), or (wN) the octant-Morton sort inside consecutive windows
// of N rays (what a wave or workgroup could sort of the chunks it takes)
void order_level(const Sim& S, std::vector<WRay>& lv, Order ord) {
  if (ord == BASE) return;
  for (WRay& r : lv) {
    r.key = ray_key(S, r, ord == OCT, ord == MORTON || (ord >= M6 && ord <= M12));
    // coarse buckets (one counting-sort pass; stable = arrival order inside a bucket):
    // the top 6 / 9 / 12 Morton bits of the origin, with or without the octant
    if (ord == M6) r.key >>= 24;
    if (ord == M9) r.key >>= 21;
    if (ord == M12) r.key >>= 18;
    if (ord == O_M6) r.key >>= 23;
    if (ord == O_M9) r.key >>= 20;
    if (ord == O_M12) r.key >>= 17;
    if (ord == D6_M6) {                     // 6 direction bits (octant + which components dominate) + 6 origin bits
      const double ax = fabs(r.d.x), ay = fabs(r.d.y), az = fabs(r.d.z), n = sqrt(ax * ax + ay * ay + az * az);
      const uint32_t dom = (ax > 0.577 * n ? 1u : 0u) | (ay > 0.577 * n ? 2u : 0u) | (az > 0.577 * n ? 4u : 0u);
      r.key = ((r.key >> 23) & ~63u) << 3 | dom << 6 | ((r.key >> 23) & 63u);
    }
  }
  const size_t win = ord == W128 ? 128 : ord == W256 ? 256 : ord == W512 ? 512 : ord == W4096 ? 4096 : lv.size();
  for (size_t a = 0; a < lv.size(); a += win)
    std::stable_sort(lv.begin() + a, lv.begin() + std::min(lv.size(), a + win),
                     [](const WRay& x, const WRay& y) { return x.key < y.key; });
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s world.yml camera.yml [tile_step] [max_rays_per_level]\n", argv[0]);
    return 2;
  }
  // tile_step > 0: every tile_step-th tile of the frame; < 0: the dense block of
  // -tile_step x -tile_step tiles at the frame's centre (ray density as in a full frame)
  const int tstep = argc > 3 ? atoi(argv[3]) : 16;
  const bool only_spec = getenv("WAVE_SIM_SPEC_ONLY") != nullptr;
  const int norder = getenv("WAVE_SIM_BASE_ONLY") ? 1 : NORDER;   // (WAVE_SIM_TREE=sah|median: the hierarchy)
  const int nwalk = only_spec ? 1 : NWALK;
  const size_t cap = argc > 4 ? (size_t)atoll(argv[4]) : 400000;
  rtxcli::Scene sc;
  rtxcli::load_world(argv[1], sc);
  const rtx_camera_desc cam = rtxcli::load_camera(argv[2]);
  Sim S;
  S.obj = sc.objects;
  S.lights = sc.lights;
  S.maxd = sc.desc.max_distance;
  S.build(true);
  printf("scene: %zu spheres, %zu nodes, %zu leaf slots, stack %d, q16 %d, tree %s\n", S.sph64.size(),
         S.bb->nodes.size(), S.bb->slot_obj.size(), S.bb->stack + 1, (int)S.q16,
         getenv("WAVE_SIM_TREE") ? getenv("WAVE_SIM_TREE") : "library rule");
  const V3 pos = v3p(cam.position), front = v3p(cam.front), up = v3p(cam.up);
  uint32_t e = 0;
  const V3 left = vnorm(vcross(up, front), e), upn = vnorm(up, e), fn = vnorm(front, e);
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> U(0, 1);
  // level 0: every tstep-th 8x8 tile, decode_item order, pre samples per pixel
  std::vector<WRay> lv0;
  const int tiles_x = (cam.width + 7) / 8, tiles_y = (cam.height + 7) / 8;
  std::vector<int> tiles;
  if (tstep > 0) {
    for (int tile = 0; tile < tiles_x * tiles_y; tile += tstep) tiles.push_back(tile);
  } else {
    const int b = -tstep, x0 = (tiles_x - b) / 2, y0 = (tiles_y - b) / 2;
    for (int ty = y0; ty < y0 + b; ty++)
      for (int tx = x0; tx < x0 + b; tx++) tiles.push_back(ty * tiles_x + tx);
  }
  for (int tile : tiles)
    for (int l = 0; l < 64; l++)
      for (int smp = 0; smp < cam.pre_sample_times; smp++) {
        const int x = (tile % tiles_x) * 8 + ((l & 1) | ((l >> 1) & 2) | ((l >> 2) & 4));
        const int y = (tile / tiles_x) * 8 + (((l >> 1) & 1) | ((l >> 2) & 2) | ((l >> 3) & 4));
        const double u = 2.0 * ((x + U(rng)) / cam.width - 0.5) * cam.retina_width;
        const double w = 2.0 * ((y + U(rng)) / cam.height - 0.5) * cam.retina_height;
        const V3 pix = vadd(vsc(fn, cam.image_distance), vadd(vsc(left, -u), vsc(upn, -w)));
        const V3 focus = vadd(pos, vsc(pix, cam.focal_distance / cam.image_distance));
        double a, b;
        do a = 2 * U(rng) - 1, b = 2 * U(rng) - 1;
        while (a * a + b * b > 1);
        const V3 lo = vadd(pos, vadd(vsc(left, a * cam.aperture_radius), vsc(upn, b * cam.aperture_radius)));
        lv0.push_back(WRay{lo, vsub(focus, lo), v3(1, 1, 1), cam.trace_depth});
      }
  printf("level-0 rays %zu (tile_step %d)\n", lv0.size(), tstep);
  Occ tot_e[NORDER][NWALK], tot_s[NORDER][NWALK];
  const char* only = getenv("WAVE_SIM_ORDERS");   // e.g. "base,o+m9,octm": these orders only
  auto wanted = [&](int ord) {
    if (!only) return true;
    const std::string list = std::string(",") + only + ",";
    return list.find(std::string(",") + order_name[ord] + ",") != std::string::npos;
  };
  for (int ord = 0; ord < norder; ord++) {
    if (!wanted(ord)) continue;
    std::vector<WRay> level = lv0;
    std::mt19937_64 rng2(7);
    for (int lev = 0; lev < cam.trace_depth && !level.empty(); lev++) {
      if (level.size() > cap) {                 // keep whole chunks: a contiguous run from the middle
        const size_t st = (level.size() - cap) / 2 / 64 * 64;
        level = std::vector<WRay>(level.begin() + st, level.begin() + st + cap);
      }
      if (lev > 0) order_level(S, level, (Order)ord);
      std::vector<WRay> next;
      Occ le[NWALK], ls[NWALK];
      for (size_t c0 = 0; c0 < level.size(); c0 += 64) {
        const size_t c1 = std::min(level.size(), c0 + 64);
        std::vector<Lane> ln[NWALK];
        for (int w = 0; w < nwalk; w++) {
          ln[w].resize(c1 - c0);
          for (size_t k = c0; k < c1; k++) lane_start(S, ln[w][k - c0], true, level[k].o, level[k].d);
          le[w].add(run_wave(S, ln[w], (Walk)w));
        }
        // shading of this chunk's hits (walk results are order independent: take SPEC's)
        for (size_t k = c0; k < c1; k++) {
          const Lane& L = ln[SPEC][k - c0];
          if (L.besti < 0) continue;
          const WRay& ray = level[k];
          const rtx_object_desc& ob = S.obj[L.besti];
          const V3 hit = vadd(ray.o, vsc(ray.d, L.best));
          V3 n, delta;
          if (ob.type == RTX_SPHERE) {
            const V3 C = v3p(ob.center);
            n = L.inside ? vsub(C, hit) : vsub(hit, C);
            delta = vsc(vsub(hit, C), 1e-5 * (L.inside ? -1.0 : 1.0));
          } else {
            n = v3p(ob.front);
            if (vdot(n, ray.d) > 0) n = vneg(n);
            delta = vsc(n, 1e-5);
          }
          const V3 T = vadd(hit, delta);
          next.push_back(WRay{T, n, ray.att, ray.depth, 0xffffffffu});   // (a hit marker; rebuilt below)
          (void)T;
        }
      }
      // shadow walks: the hits in ray order, 64 per wave, one per light
      std::vector<WRay> hits;
      hits.swap(next);
      for (const rtx_light_desc& Lt : S.lights) {
        for (size_t c0 = 0; c0 < hits.size(); c0 += 64) {
          const size_t c1 = std::min(hits.size(), c0 + 64);
          for (int w = 0; w < nwalk; w++) {
            std::vector<Lane> ln(c1 - c0);
            for (size_t k = c0; k < c1; k++)
              lane_start(S, ln[k - c0], false, hits[k].o, vsub(v3p(Lt.position), hits[k].o));
            ls[w].add(run_wave(S, ln, (Walk)w));
          }
        }
      }
      // children (level order: parent order, reflection then refraction then diffusion)
      size_t hi = 0;
      for (size_t k = 0; k < level.size(); k++) {
        const WRay& ray = level[k];
        Lane L;
        lane_start(S, L, true, ray.o, ray.d);
        // (the nearest hit again, cheaply: plain walk)
        std::vector<Lane> one{L};
        run_wave(S, one, NOSPEC);
        L = one[0];
        if (L.besti < 0) continue;
        const WRay& hr = hits[hi++];
        if (ray.depth - 1 <= 0) continue;
        const rtx_object_desc& ob = S.obj[L.besti];
        const V3 hit = vadd(ray.o, vsc(ray.d, L.best));
        const V3 nn = vnorm(hr.d, e), dn = vnorm(ray.d, e);
        bool lit = true;
        for (const rtx_light_desc& Lt : S.lights) {
          Lane sl;
          lane_start(S, sl, false, hr.o, vsub(v3p(Lt.position), hr.o));
          std::vector<Lane> one2{sl};
          run_wave(S, one2, NOSPEC);
          if (one2[0].besti >= 0) lit = false;
        }
        const V3 ra = vmul(ray.att, v3p(ob.reflective_attenuation));
        if (vr(ra) >= 1e-4) next.push_back(WRay{hr.o, vsub(dn, vsc(nn, 2.0 * vdot(dn, nn))), ra, ray.depth - 1});
        const V3 fa = vmul(ray.att, v3p(ob.refractive_attenuation));
        if (ob.type == RTX_SPHERE && vr(fa) >= 1e-4) {
          const double eta = L.inside ? ob.refractive_rate : 1.0 / ob.refractive_rate;
          const double ci = -vdot(dn, nn), kk = 1 - eta * eta * (1 - ci * ci);
          if (kk >= 0) next.push_back(WRay{vsub(hit, vsc(nn, 1e-5)), vadd(vsc(dn, eta), vsc(nn, eta * ci - sqrt(kk))), fa,
                                          ray.depth - 1});
        }
        if (!lit && cam.monte_carlo_diffusion_times > 0) {
          for (int k2 = 0; k2 < cam.monte_carlo_diffusion_times; k2++) {
            V3 dir = v3(U(rng2) - 0.5, U(rng2) - 0.5, U(rng2) - 0.5);
            if (vdot(dir, nn) < 0) dir = vneg(dir);
            const V3 pa = vmul(ray.att, vsc(v3p(ob.diffuse_rate), 1.0 / cam.monte_carlo_diffusion_times));
            if (vr(pa) >= 1e-4) next.push_back(WRay{hr.o, dir, pa, ray.depth - 1});
          }
        }
      }
      for (int w = 0; w < nwalk; w++) {
        printf("order %-6s level %d rays %7zu hits %7zu walk %-6s | extend node %5.1f leaf %5.1f exact %5.1f occ %5.1f "
               "time/ray %6.1f | shadow node %5.1f leaf %5.1f exact %5.1f occ %5.1f time/ray %6.1f\n",
               order_name[ord], lev, level.size(), hits.size(), walk_name[w], le[w].lanes[0] / std::max(1.0, le[w].steps[0]),
               le[w].lanes[1] / std::max(1.0, le[w].steps[1]), le[w].lanes[2] / std::max(1.0, le[w].steps[2]),
               le[w].occ(), le[w].time() / level.size(), ls[w].lanes[0] / std::max(1.0, ls[w].steps[0]),
               ls[w].lanes[1] / std::max(1.0, ls[w].steps[1]), ls[w].lanes[2] / std::max(1.0, ls[w].steps[2]), ls[w].occ(),
               ls[w].time() / std::max<size_t>(1, hits.size()));
        tot_e[ord][w].add(le[w]);
        tot_s[ord][w].add(ls[w]);
      }
      fflush(stdout);
      level.swap(next);
    }
  }
  printf("\nall levels (time: VALU-instruction proxy per wave, summed; occ: cost-weighted active lanes)\n");
  for (int ord = 0; ord < norder; ord++)
    for (int w = 0; w < nwalk && wanted(ord); w++)
      printf("order %-6s walk %-6s | extend occ %5.1f time %10.4g | shadow occ %5.1f time %10.4g | total %10.4g (x base/spec %.3f)"
             " | lanes per step (RTX_WALKSTATS form): extend node %.1f leaf %.1f, shadow node %.1f leaf %.1f"
             " | steps node/leaf/exact: extend %.3g %.3g %.3g (exact %.1f lanes; compacted %.3g), shadow %.3g %.3g %.3g"
             " (exact %.1f lanes; compacted %.3g)\n",
             order_name[ord], walk_name[w], tot_e[ord][w].occ(), tot_e[ord][w].time(), tot_s[ord][w].occ(),
             tot_s[ord][w].time(), tot_e[ord][w].time() + tot_s[ord][w].time(),
             (tot_e[ord][w].time() + tot_s[ord][w].time()) / (tot_e[BASE][SPEC].time() + tot_s[BASE][SPEC].time()),
             tot_e[ord][w].lanes[0] / std::max(1.0, tot_e[ord][w].steps[0]),
             tot_e[ord][w].lanes[1] / std::max(1.0, tot_e[ord][w].steps[1]),
             tot_s[ord][w].lanes[0] / std::max(1.0, tot_s[ord][w].steps[0]),
             tot_s[ord][w].lanes[1] / std::max(1.0, tot_s[ord][w].steps[1]), tot_e[ord][w].steps[0],
             tot_e[ord][w].steps[1], tot_e[ord][w].steps[2], tot_e[ord][w].lanes[2] / std::max(1.0, tot_e[ord][w].steps[2]),
             tot_e[ord][w].exact_ideal, tot_s[ord][w].steps[0], tot_s[ord][w].steps[1], tot_s[ord][w].steps[2],
             tot_s[ord][w].lanes[2] / std::max(1.0, tot_s[ord][w].steps[2]), tot_s[ord][w].exact_ideal);
  return 0;
}
