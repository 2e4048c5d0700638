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
#include "rtx_device.h"

#include <unordered_map>

#include <mutex>
#include <vector>

namespace rtx {


// SRC_PIXELS: work item = one of Camera#render_at's pre_sample_times samples
// of one pixel (a wave's first fetch covers an 8x8 tile for one sample index);
// the sample's colour and first raise go to p.samples, and k_finalize does the
// mean / variance / extra-sample decision.  SRC_EXTRA: the extra samples of the
// pixels k_finalize listed.  SRC_RAYS: one lane per explicit ray running
// RayTracer#trace_sync (rtx_trace).  SPH: where the sphere walk reads its
// records (SphMode, rtx_launch.h).  BS: threads per workgroup.
template <bool COUNT, int WPS, int SPH, int SRC, int BS, bool PP>
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

  Stack st;
  st.n = 0;
  st.maxs = p.lanes_maxs;
  st.bs = BS;
  st.slots = p.stk_slots;
  st.lds = reinterpret_cast<double*>(lds + p.lds_items) + threadIdx.x;
  st.g = p.stk_glb + ((size_t)blockIdx.x * BS + threadIdx.x) * ((size_t)p.lanes_maxs * GITEM_DOUBLES);
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
        if (highlights(S, cur, sum, err,
                       [&](V3 T, V3 L, double rad, int) { return raises_walk<SPH, BS>(p, lds, T, L, rad); }))
          continue;
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

    // ---- B: the object walk, shared by EXTEND and SHADOW lanes (a SHADOW walk
    // also checks its covers' acos raises, option exact_raises: rtx_device.h xr_band)
    const bool xr = p.exact_raises != 0 && mode == M_SHADOW;
    if (SPH == SPH_LIN_LDS)
      query<COUNT>(S, sph_lds, mode == M_EXTEND, qo, qd, qL, qrad, best, besti, hit, hin, total, err, cnt, xr);
    else if (SPH == SPH_LIN_SCALAR)
      query<COUNT>(S, sph_k, mode == M_EXTEND, qo, qd, qL, qrad, best, besti, hit, hin, total, err, cnt, xr);
    else if (SPH == SPH_BVH_LDS)
      q_resume = !query_bvh<BS, PP>(S, reinterpret_cast<const Bvh4Node*>(lds),
                                reinterpret_cast<const float4*>(lds + p.lds_leaf), S.bvh_sph64, S.bvh_obj, stk,
                                cov_i, cov_v,
                                mode == M_EXTEND, qo, qd, qL, qrad, best, besti, hit, hin, total, err, q_ref, q_sp,
                                q_ncov, q_ovf, q_resume, p.postpone, xr);
    else
      q_resume = !query_bvh<BS, PP>(S, S.bvh, reinterpret_cast<const float4*>(S.bvh_sph32), S.bvh_sph64, S.bvh_obj,
                                stk, cov_i, cov_v,
                                mode == M_EXTEND, qo, qd, qL, qrad, best, besti, hit, hin, total, err, q_ref, q_sp,
                                q_ncov, q_ovf, q_resume, p.postpone, xr);
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
    have = shade_finish(S, cam, p.seed, x, y, sample, besti, hin, hit, delta, n, nn, lc, nl, cur, st, sum,
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
  if (it.depth > 0 && !(vr(it.att) < 0.0001) &&
      !highlights<false>(S, it, sum, err, [&](V3 T, V3 L, double rad, int) {
        return lit_area_raises(S, nullptr, nullptr, nullptr, (int*)nullptr, 0, T, L, rad);   // (ordered linear walk)
      })) {
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
  // phase 1: err is the pre-sample raise (already recorded by phase 0 with the
  // smaller phase-0 key) or else the first extra-sample raise
  if (err) record_error(p.err, err, px_key(x, y, cam.height, phase));
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

// The same for tile lists (rtx_render_multi_plan): rank k's packed row r is
// image row plan[k * per_rank + r / tile_rows] * tile_rows + r % tile_rows.
__global__ void k_unpack_plan(const double* __restrict__ gathered, int w, int h, int tile_rows, int n, int per_rank,
                              const int32_t* __restrict__ plan, double* __restrict__ out, size_t stride) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per_row = (long)w * 3;
  const int rows_per_rank = per_rank * tile_rows;
  if (i >= (long)n * rows_per_rank * per_row) return;
  const int src_row = (int)(i / per_row);
  const int k = src_row / rows_per_rank, r = src_row - k * rows_per_rank;
  const long y = (long)plan[k * per_rank + r / tile_rows] * tile_rows + r % tile_rows;
  if (y >= h) return;                              // padding tiles (index past the bottom)
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
  unsigned long long lv[16];                     // k_level's phases (slots 0-7) from rtx_levels.hip
  if (read_level_stamps(lv, reset) != 0) return -1;
  for (int k = 0; k < 8; k++) out[k] += lv[k];
  for (int k = 8; k < 11; k++) out[k] = lv[k];   // (k_level: lanes with a ray / a walk / a hit)
  if (lv[13])                                     // k_tree_finalize's phases (a levels-engine frame)
    for (int k = 11; k < 15; k++) out[k] = lv[k];
  return 0;
}

int stack_bucket(int need) {
  if (need <= 8) return 8;
  if (need <= 16) return 16;
  if (need <= 32) return 32;
  if (need <= 64) return 64;
  return -1;
}


size_t bvh_lds_bytes(int n_nodes, int n_slots, int bvh_stack) {
  return (size_t)n_nodes * sizeof(Bvh4Node) + (size_t)n_slots * 16 + (size_t)bvh_stack * BS_BVH * 4 +
         (size_t)COVER_K * BS_BVH * 12 + 64;
}
size_t bvh_lds_budget() { return LDS_TOTAL_BYTES; }

int resolve_mode(const SceneDev& S, int mode) {
  if (mode == SPH_BVH_QLDS) {                  // nodes + 16-bit leaf records + 16-bit stacks, when conservative
    const size_t need = (size_t)S.n_nodes * sizeof(Bvh4Node) + (size_t)S.n_slots * 8 +
                        (size_t)S.bvh_stack * BS_BVH * 2 + (size_t)COVER_K * BS_BVH * 12 + 64;
    if (S.q_ok && need <= LDS_TOTAL_BYTES) return mode;
    mode = SPH_BVH_MIX;
  }
  if (mode == SPH_BVH_LDSX) {                  // the staged hierarchy plus its exact records
    const size_t need = bvh_lds_bytes(S.n_nodes, S.n_slots, S.bvh_stack) + (size_t)S.n_slots * (sizeof(Sphere64) + 4) +
                        16 + (size_t)S.n_obj * sizeof(Material) + (size_t)S.n_sphere * sizeof(Sphere64);
    if (need <= LDS_TOTAL_BYTES) return mode;
    mode = SPH_BVH_LDS;
  }
  if (mode == SPH_BVH_MIX) {                   // nodes in LDS, leaves global: needs room for the nodes
    const size_t need = (size_t)S.n_nodes * sizeof(Bvh4Node) + (size_t)S.bvh_stack * BS_BVH * 4 +
                        (size_t)COVER_K * BS_BVH * 12 + 64;
    return need > LDS_TOTAL_BYTES ? SPH_BVH_GLOBAL : SPH_BVH_MIX;
  }
  if (mode == SPH_LIN_LDS && (size_t)(S.n_sphere + 4) * 16 > LDS_SPHERE_BYTES) return SPH_LIN_SCALAR;
  if (mode == SPH_BVH_LDS && bvh_lds_bytes(S.n_nodes, S.n_slots, S.bvh_stack) > LDS_TOTAL_BYTES)
    return SPH_BVH_GLOBAL;
  return mode;
}


static thread_local KernelEvents* g_kev = nullptr;   // set by launch_render for its launches
static thread_local bool g_work_zeroed = false;      // launch_one: the work counter is already zero

// Occupancy of a persistent launch, cached per (kernel, block size, LDS
// bytes, device): CUs and resident blocks per CU, the kernel's dynamic-LDS
// limit raised the first time.  Querying the runtime on every launch cost host
// time per level launch, which small frames (one rank's share) feel.
hipError_t launch_fit(const void* kern, int bs, size_t lds, int& cus, int& per_cu) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  struct Key {
    const void* k;
    int bs, dev;
    size_t lds;
    bool operator==(const Key& o) const { return k == o.k && bs == o.bs && dev == o.dev && lds == o.lds; }
  };
  struct KeyHash {
    size_t operator()(const Key& x) const {
      size_t h = std::hash<const void*>()(x.k);
      h = h * 1000003u ^ std::hash<size_t>()(x.lds);
      return h * 1000003u ^ (size_t)(x.bs * 64 + x.dev);
    }
  };
  static std::mutex mu;
  static std::unordered_map<Key, std::pair<int, int>, KeyHash> cache;   // -> (cus, per_cu)
  const Key key{kern, bs, dev, lds};
  {
    std::lock_guard<std::mutex> g(mu);
    const auto it = cache.find(key);
    if (it != cache.end()) {
      cus = it->second.first;
      per_cu = it->second.second;
      return hipSuccess;
    }
  }
  if (lds > 64 * 1024) (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, bs, lds);
  if (e != hipSuccess) return e;
  if (per_cu < 1) per_cu = 1;
  std::lock_guard<std::mutex> g(mu);
  // the LDS size depends on the scene: a process that uploads very many scene
  // sizes starts over rather than growing without bound
  if (cache.size() >= 4096) cache.clear();
  cache[key] = {cus, per_cu};
  return hipSuccess;
}

// Persistent launch: as many workgroups as can be resident at once (the
// occupancy API; an over-estimate only leaves blocks that start after the
// pool is empty and exit at once), never more than the work needs.
template <bool COUNT, int SPH, int SRC, bool PP = false>
static hipError_t launch_one(KParams p, int maxs, int nwork, hipStream_t s) {
  constexpr int BS = (SPH == SPH_BVH_LDS || SPH == SPH_BVH_GLOBAL) ? BS_BVH : BS_LIN;
  const size_t lds = lds_layout(p, SPH, BS);
  p.lanes_maxs = maxs;
  auto kern = k_render<COUNT, RTX_WPS, SPH, SRC, BS, PP>;
  int cus = 0, per_cu = 0;
  hipError_t e = launch_fit(reinterpret_cast<const void*>(kern), BS, lds, cus, per_cu);
  if (e != hipSuccess) return e;
  const long need = ((long)nwork + BS - 1) / BS;
  long blocks = std::min<long>(need, (long)cus * per_cu);
  blocks = std::min<long>(blocks, (long)p.stk_glb_lanes / BS);   // lanes with a global ray-stack region
  // The re-render of overflowed samples (SRC_LIST) is launched after every
  // batch and is nearly always empty; its grid is capped (option
  // lv_redo_blocks) so that it does not wait for a whole chip's worth of CUs
  // that another stream's level launch holds (the batch's tree reduction
  // waits behind it).
  if (SRC == SRC_LIST && p.lv_redo_blocks > 0) blocks = std::min<long>(blocks, p.lv_redo_blocks);
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

template <bool COUNT, int SRC>
static hipError_t launch_mode(const KParams& p, int mode, int maxs, int nwork, hipStream_t s) {
  switch (mode) {
    case SPH_LIN_LDS: return launch_one<COUNT, SPH_LIN_LDS, SRC>(p, maxs, nwork, s);
    case SPH_LIN_SCALAR: return launch_one<COUNT, SPH_LIN_SCALAR, SRC>(p, maxs, nwork, s);
    case SPH_BVH_LDS:
      if (!COUNT && p.postpone > 0) return launch_one<false, SPH_BVH_LDS, SRC, true>(p, maxs, nwork, s);
      if (!COUNT) return launch_one<false, SPH_BVH_LDS, SRC>(p, maxs, nwork, s);
      break;
    case SPH_BVH_GLOBAL:
      if (!COUNT && p.postpone > 0) return launch_one<false, SPH_BVH_GLOBAL, SRC, true>(p, maxs, nwork, s);
      if (!COUNT) return launch_one<false, SPH_BVH_GLOBAL, SRC>(p, maxs, nwork, s);
      break;
  }
  return hipErrorInvalidValue;
}

// The lane's ray-stack depth (maxs: 8, 16, 32 or 64 entries, sized on the host
// from the camera's tree depth) is a launch parameter, not a template axis.
template <int SRC>
static hipError_t launch_src(const KParams& p, int mode, bool count, int maxs, int nwork, hipStream_t s) {
  if (maxs != 8 && maxs != 16 && maxs != 32 && maxs != 64) return hipErrorInvalidValue;
  return count ? launch_mode<true, SRC>(p, mode, maxs, nwork, s) : launch_mode<false, SRC>(p, mode, maxs, nwork, s);
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
  if (mode == SPH_BVH_MIX || mode == SPH_BVH_LDSX || mode == SPH_BVH_QLDS) mode = SPH_BVH_LDS;   // (the lanes engine stages the whole hierarchy or none)
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


// The lanes engine's re-render of the level-0 items the bounce-level engine
// could not hold (SRC_LIST; k_level_begin already zeroed its work counter).
hipError_t launch_redo(const KParams& q, int mode, int maxs, int n, hipStream_t s) {
  g_work_zeroed = true;
  if (mode == SPH_BVH_MIX || mode == SPH_BVH_LDSX || mode == SPH_BVH_QLDS) mode = resolve_mode(q.scene, SPH_BVH_LDS);   // (see launch_render)
  const hipError_t e = launch_src<SRC_LIST>(q, mode, false, maxs, n, s);
  g_work_zeroed = false;
  return e;
}

hipError_t launch_trace(KParams p, int mode, int maxs, hipStream_t s) {
  if (p.nrays == 0) return hipSuccess;
  if (mode == SPH_BVH_MIX || mode == SPH_BVH_LDSX || mode == SPH_BVH_QLDS) mode = SPH_BVH_LDS;   // (see launch_render)
  mode = resolve_mode(p.scene, mode);
  return launch_src<SRC_RAYS>(p, mode, false, maxs, p.nrays, s);
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

hipError_t launch_unpack_plan(const double* gathered, int w, int h, int tile_rows, int n, int per_rank,
                              const int32_t* d_plan, double* out, size_t stride, hipStream_t s) {
  const long total = (long)n * per_rank * tile_rows * w * 3;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack_plan, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, gathered, w, h, tile_rows,
                     n, per_rank, d_plan, out, stride);
  return hipGetLastError();
}

// The k_tile_cost probe over a whole frame (rtx_tile_probe): the class of every
// 8x8 tile into cls (device, one int per tile).
hipError_t launch_tile_probe(KParams p, int32_t* cls, hipStream_t s) {
  const int tiles = ((p.nx + 7) / 8) * ((p.nrows + 7) / 8);
  if (tiles == 0) return hipSuccess;
  hipLaunchKernelGGL(k_tile_cost, dim3((unsigned)((tiles * 4 + 255) / 256)), dim3(256), 0, s, p, cls);
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
