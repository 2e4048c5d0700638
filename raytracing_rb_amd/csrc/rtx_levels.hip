// rtx_levels.hip — the bounce-level engine on gfx950:
// RayTracer#trace_sync (src/ray_tracer.rb:16-46) breadth-first, one launch per
// ray-tree level (or three: trace / shadow / shade), and Camera#render_at's
// reduction over the stored trees.
#include <vector>

#include "rtx_device.h"

namespace rtx {

// ================================================================= bounce levels
// The bounce-level engine (option "engine" = 1).  Instead of
// one lane walking one sample's whole ray tree (the lanes engine), every ray
// of tree level d is one work item of the level-d launch: the camera samples
// at level 0, their live children at level 1, and so on.  A wave's 64 lanes
// therefore run the same step of rt_map (ray_tracer.rb:50-164) on 64 rays at
// once, and no sample's tree can hold a launch open: a launch's longest item
// is one ray.
//
// Order.  trace_sync pops rays LIFO and drains the leaves FIFO afterwards
// (ray_tracer.rb:31-45): leaves are summed in pre-order of the tree, children
// visited in reverse push order (refraction after its pt siblings, reflection
// last).  Each ray writes a tree record {first raise, leaf count, child mask,
// first child, leaves}; its live children go, contiguous and in slot order,
// to the next level's queue.  k_tree_finalize walks each sample's tree in the
// reference's order and sums the leaves in it: the same additions in the same
// order as the sequential program, so the same bits.
//
// Queues without contended atomics.  One device-scope counter
// word saturates at ~88 atomics/us on MI355X (MI355X_MICROARCH.md, "dequeue"),
// below what one chunk claim plus one child allocation per 64 rays needs.  So
//   * chunks are scheduled statically: wave w of W takes chunks w, w + W, ...;
//   * a level's queue (levels >= 1) is cut into LV_SLICES slices of 2^k slots,
//     each with its own counter on its own 128-B line; a wave allocates its
//     children in slice (wave id mod LV_SLICES) with one atomicAdd (wave prefix
//     count: ballot / mbcnt / shfl).  A consumer wave reads the 64 slice
//     counts (one per lane), scans them, and maps its chunk to (slice, offset)
//     with one ballot; dense ray indices (the record arena) are the slice
//     prefix plus the offset, and k_tree_finalize translates a parent's child
//     slot to the dense index the same way.
//
// Raises.  rt_map's raises happen while the tree is walked, the "color greater
// than 1" of rt_reduce only in the drain after it (:39-45): a record keeps the
// first raise of its ray in rt_map's order (highlights; reflection and
// refraction; local_lights' lit_area; path tracing / local_lighting), the walk
// takes the first in tree order, and a >1 partial sum counts only without one.
//
// Capacity.  Children beyond their slice or tree records beyond the record
// arena are not written; their camera sample is listed (lv_redo_list) and
// re-rendered whole by the lanes engine (SRC_LIST), exact either way.
// Staging ray record (p.lv_ray_dbl doubles per slot):
//   12 (96 B): o, d, att, path, {root item, sample}, {x, y};
//   10 (80 B): o, d, att, {path, root item} as two 32-bit words.  The host
//   picks it when every path of the camera's trees fits 32 bits (path < (pt +
//   3)^trace_depth <= 2^32); the RNG key (x, y, sample), needed only by the
//   path-tracing children of a level >= 1 ray, is then decoded from the root.
constexpr int RAY_DOUBLES = 12;
constexpr int RAY_DOUBLES_SMALL = 10;
constexpr int HIT_DOUBLES = 8;           // split hit record: hit, hit + delta, {ray, object | in}, {slot, raises}
static_assert(RAY_DOUBLES * 8 == (int)RAY_BYTES && HIT_DOUBLES * 8 == (int)LV_HIT_BYTES, "record sizes");

// Diagnostic builds: the level kernels' phases per tree level (levels >= 7
// summed into row 7): 6 phases, chunks, lanes with a hit.
static __device__ unsigned long long rtx_stamps_lv[8 * 8];

int levels_rec_bytes(int n_light) {
  const int nl = n_light > 1 ? n_light : 1;
  return (8 + 24 * nl + 15) & ~15;       // {meta, first child} + one leaf per fired light
}

// slice counter of slice s of a level (own 128-B line)
__device__ __forceinline__ uint32_t* lv_slice_ctr(uint32_t* level_ctrs, int s) { return level_ctrs + s * 32; }

__device__ __forceinline__ void lv_redo(const KParams& p, int root) {
  if (atomicCAS(&p.lv_redo_of[root], -1, -2) == -1) {
    const uint32_t e = atomicAdd(&p.lv_ctl->redo_n, 1u);
    p.lv_redo_list[e] = root;
    p.lv_redo_of[root] = (int)e;
  }
}

// World#high_lights' lit_area (world.rb:92-93), deferred.  Its only effect is
// a raise (Math.acos in Sphere#cover_area, lit_area_raises), and its walk,
// run in the level kernel by the one lane whose ray fired while the wave's
// other lanes wait, cost C2 2.8 % and C4 11 % (r07a).  So a level kernel only
// appends a fired ray {o, d, record, root} to the batch's list (wave-
// aggregated: one atomic per wave) and k_hl_raise re-runs the highlight loop
// of every listed ray with the walk, full waves of them, after the batch's
// levels, rewriting the raise byte of the ray's record.  A ray that finds the
// list full sends its sample to the lanes engine (lv_redo), exact either way.
// All lanes of the wave call it.
constexpr int HLQ_DOUBLES = 8;
template <typename RootFn>
__device__ __forceinline__ void lv_hl_defer(const KParams& p, bool want, const Ray& r, uint32_t rec, RootFn&& root_fn) {
  const uint64_t m = __ballot(want);
  if (!m) return;
  const int lane = (int)__lane_id(), first = __builtin_ctzll(m);
  uint32_t b = 0;
  if (lane == first) b = atomicAdd(&p.lv_ctl->hl_n, (uint32_t)__popcll(m));
  b = (uint32_t)__builtin_amdgcn_readlane((int)b, first);
  if (!want) return;
  const uint32_t e = b + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
  if (e >= p.lv_hlq_cap) {
    lv_redo(p, root_fn());
    return;
  }
  double2* q = reinterpret_cast<double2*>(p.lv_hlq + (size_t)e * HLQ_DOUBLES);
  q[0] = make_double2(r.o.x, r.o.y);
  q[1] = make_double2(r.o.z, r.d.x);
  q[2] = make_double2(r.d.y, r.d.z);
  q[3] = make_double2(__builtin_bit_cast(double, (uint64_t)rec), 0.0);
}

// root: the level-0 item of the ray's tree; (x, y, sample): its RNG key.
__device__ __forceinline__ void lv_store_ray(const KParams& p, double* dst, const Ray& r, V3 att, uint64_t path,
                                             int root, int x, int y, int sample) {
  double2* q = reinterpret_cast<double2*>(dst);
  q[0] = make_double2(r.o.x, r.o.y);
  q[1] = make_double2(r.o.z, r.d.x);
  q[2] = make_double2(r.d.y, r.d.z);
  q[3] = make_double2(att.x, att.y);
  if (p.lv_ray_dbl == RAY_DOUBLES_SMALL) {
    q[4] = make_double2(att.z, __builtin_bit_cast(double, (uint64_t)(uint32_t)path | (uint64_t)(uint32_t)root << 32));
    return;
  }
  q[4] = make_double2(att.z, __builtin_bit_cast(double, path));
  q[5] = make_double2(__builtin_bit_cast(double, (uint64_t)(uint32_t)root | (uint64_t)(uint32_t)sample << 32),
                      __builtin_bit_cast(double, (uint64_t)(uint32_t)x | (uint64_t)(uint32_t)y << 32));
}

// A staged ray's path, root item and RNG key from the record's last 16-B
// words (e = {att.z, .}, f: the 96-B record's last word, unread for 80 B).
__device__ __forceinline__ void lv_ray_tail(const KParams& p, const double2* q, double2 e, uint64_t& path, int& root,
                                            int& x, int& y, int& sample) {
  const uint64_t w = __builtin_bit_cast(uint64_t, e.y);
  if (p.lv_ray_dbl == RAY_DOUBLES_SMALL) {
    path = (uint32_t)w;
    root = (int)(w >> 32);
    x = y = sample = -1;                       // decoded when needed (lv_ray_key)
    return;
  }
  const double2 f = q[5];
  path = w;
  const uint64_t rs = __builtin_bit_cast(uint64_t, f.x), xy = __builtin_bit_cast(uint64_t, f.y);
  root = (int)(uint32_t)rs;
  sample = (int)(rs >> 32);
  x = (int)(uint32_t)xy;
  y = (int)(xy >> 32);
}

// The root item of the staged ray at `q` (its record-arena overflow).
__device__ __forceinline__ int lv_ray_root(const KParams& p, const double2* q) {
  const uint64_t w = __builtin_bit_cast(uint64_t, p.lv_ray_dbl == RAY_DOUBLES_SMALL ? q[4].y : q[5].x);
  return p.lv_ray_dbl == RAY_DOUBLES_SMALL ? (int)(w >> 32) : (int)(uint32_t)w;
}

__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t v) {
  const int lane = (int)__lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)v, off);
    if (lane >= off) v += t;
  }
  return v;
}

// One wave's view of a queue: lane s holds slice s (count clamped to the
// slice capacity, exclusive item prefix, inclusive chunk prefix).  Level 0 is
// one dense slice.  `mult` items per queue entry (the shadow launch: lights).
struct LvQueue {
  uint32_t cnt, pex, cin;      // per lane = per slice
  uint32_t total, chunks;      // wave-uniform
  __device__ __forceinline__ void dense(uint32_t n) {
    const int lane = (int)__lane_id();
    cnt = lane == 0 ? n : 0u;
    pex = lane == 0 ? 0u : n;
    cin = (n + 63u) >> 6;
    total = n;
    chunks = cin;
  }
  __device__ __forceinline__ void sliced(const uint32_t* ctrs, uint32_t cap, uint32_t mult) {
    const int lane = (int)__lane_id();
    uint32_t c = ctrs[lane * 32];
    c = (c < cap ? c : cap) * mult;
    const uint32_t incl = wave_scan_incl(c);
    cnt = c;
    pex = incl - c;
    total = (uint32_t)__shfl((int)incl, 63);
    cin = wave_scan_incl((c + 63u) >> 6);
    chunks = (uint32_t)__shfl((int)cin, 63);
  }
  // chunk c (< chunks) -> this lane's slice s, offset within the slice, dense
  // index; valid false past the slice's count.  All lanes must call it.
  __device__ __forceinline__ bool item(uint32_t c, uint32_t& s, uint32_t& off, uint32_t& dense_i) const {
    return item_k(c, __lane_id(), s, off, dense_i);
  }
  // the same for ray k (< 64) of chunk c instead of the lane's own
  __device__ __forceinline__ bool item_k(uint32_t c, uint32_t k, uint32_t& s, uint32_t& off,
                                         uint32_t& dense_i) const {
    s = (uint32_t)__popcll(__ballot(cin <= c));
    const uint32_t first = s ? (uint32_t)__shfl((int)cin, (int)s - 1) : 0u;
    off = (c - first) * 64u + k;
    dense_i = (uint32_t)__shfl((int)pex, (int)s) + off;
    return off < (uint32_t)__shfl((int)cnt, (int)s);
  }
};

// Level d's first record in the arena (the dense counts of levels < d), from
// the compact layout (lv_level_done).
__device__ __forceinline__ uint32_t lv_base(const KParams& p, int level) { return p.lv_ctl->lay_base[level]; }

// A level's queue: level 0 is one dense slice; levels >= 1 read the compact
// layout the launch that allocated them left (lv_level_done: three coalesced
// 256-B loads, where reading the 64 slice counters, one per 128-B line, cost
// every wave of every launch a 64-line gather from the same hot lines).
__device__ __forceinline__ void lv_in_queue(const KParams& p, int level, LvQueue& q) {
  if (level == 0) {
    q.dense(p.lv_ctl->count0);
    return;
  }
  const int lane = (int)__lane_id();
  q.cnt = p.lv_ctl->lay_cnt[level][lane];
  q.pex = p.lv_ctl->lay_pex[level][lane];
  q.cin = p.lv_ctl->lay_cin[level][lane];
  q.total = (uint32_t)__shfl((int)(q.pex + q.cnt), 63);
  q.chunks = (uint32_t)__shfl((int)q.cin, 63);
}

// Ray binning (option lv_sort).  A level >= 1 holds its rays
// in the order their parents were shaded, so a wave's 64 rays start from
// scattered points in all directions and its lanes walk different parts of the
// hierarchy.  With lv_sort the producer tags every staged ray with a bin (the
// octant of its direction and the cell of its origin in a 16 x 16 x 16 grid
// over the spheres' box, Morton order); before the level's launch k_lv_bin (count)
// / k_lv_bin_scan / k_lv_bin (scatter), one counting-sort pass, list the
// level's rays bin by bin, and the level takes its chunks from that list.
// Only the visiting order changes: every ray writes its record at its dense
// index and allocates its children as before, so the trees, hence the frames,
// are bit-identical (order independence, §3.7).
__device__ __forceinline__ uint32_t lv_ray_bin(const SceneDev& S, const Ray& r, int bits) {
  const float cells = (float)(1 << bits);
  const float o[3] = {(float)r.o.x, (float)r.o.y, (float)r.o.z};
  uint32_t m = 0;
#pragma unroll
  for (int a = 0; a < 3; a++) {
    const float lo = S.root_c[a] - S.root_h[a];
    const float f = (o[a] - lo) * ((0.5f * cells) / fmaxf(S.root_h[a], 1e-30f));   // cells over 2 h
    const uint32_t c = (uint32_t)fminf(fmaxf(f, 0.0f), cells - 1.0f);            // (NaN: cell 0)
#pragma unroll
    for (int b = 0; b < LV_CELL_BITS_MAX; b++) m |= ((c >> b) & 1u) << (3 * b + a);   // Morton order
  }
  const uint32_t oct = (r.d.x < 0 ? 1u : 0u) | (r.d.y < 0 ? 2u : 0u) | (r.d.z < 0 ? 4u : 0u);
  return oct << (3 * bits) | m;
}
static_assert(LV_BINS <= 65536, "bins are 16-bit keys");

__device__ __forceinline__ const double* lv_src(const KParams& p, int level) {
  return p.lv_sorted && p.lv_sort && level >= p.lv_sort ? p.lv_sorted : p.lv_stage[level & 1];
}

// The level's chunks, and chunk c's ray for this lane: its queue slot and
// dense index (binned: from the bin list; else the slices).  All lanes call it.
__device__ __forceinline__ uint32_t lv_chunks(const KParams& p, const LvQueue& in, int level) {
  return p.lv_sort && level >= p.lv_sort ? (in.total + 63u) >> 6 : in.chunks;
}
// With lv_sort_copy the binning pass also moved the records into bin order
// (lv_sorted): the ray's "slot" is then its place k in that order, and
// lv_src gives the array the level's records are read from.
__device__ __forceinline__ bool lv_chunk_item(const KParams& p, const LvQueue& in, int level, uint32_t c,
                                              uint32_t& slot, uint32_t& i) {
  if (p.lv_sort && level >= p.lv_sort) {
    const uint32_t k = c * 64u + (uint32_t)__lane_id();
    slot = i = 0;
    if (k >= in.total) return false;
    const uint2 e = p.lv_perm[k];
    slot = p.lv_sorted ? k : e.x;
    i = e.y;
    return true;
  }
  uint32_t s, off;
  const bool a = in.item(c, s, off, i);
  slot = level == 0 ? i : (s << p.lv_slice_log2) + off;
  return a;
}

// The end of a launch that allocated level e's rays (k_level, k_level_c,
// k_lv_shade of level e - 1): the grid's last wave to finish writes level e's
// compact layout: per slice the ray count (clamped to the slice), the
// exclusive ray prefix and the inclusive 64-ray chunk prefix, and the first
// record of level e + 1.  No barrier (a wave that is done leaves at once and
// frees its SIMD slots) and no fence (a device-scope release fence writes
// back the XCD's L2: 2048 of them cost C2 0.7 ms): wave w counts itself on
// counter w mod LV_DONE (each on its own line), the wave that completes a
// counter counts it on the top counter, and the wave that completes the top
// counter is the last one.  Every slice allocation is a device-scope atomic
// whose value its wave consumed before it got here, and the counts are
// device-scope atomics too, all performed at the same coherence point: the
// last wave's atomic loads see every allocation.  (The ray records are read
// by later launches only: kernel boundaries order them.)
__device__ __forceinline__ void lv_level_done(const KParams& p, int e) {
  if (e > LV_MAXL) return;
  const int lane = (int)__lane_id();
  const uint32_t W = gridDim.x * (blockDim.x >> 6);
  const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint32_t j = w % LV_DONE;
  const uint32_t quota = W / LV_DONE + (j < W % LV_DONE ? 1u : 0u);
  const uint32_t nsub = W < LV_DONE ? W : (uint32_t)LV_DONE;
  uint32_t last = 0;
  if (lane == 0) {
    if (__hip_atomic_fetch_add(&p.lv_ctl->done_sub[e][j * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
        quota - 1)
      last = __hip_atomic_fetch_add(&p.lv_ctl->done[e], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsub - 1;
  }
  if (!__shfl((int)last, 0)) return;
  const uint32_t cap = 1u << p.lv_slice_log2;
  uint32_t c = __hip_atomic_load(&p.lv_ctl->sc[e][lane * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  c = c < cap ? c : cap;
  const uint32_t incl = wave_scan_incl(c);
  p.lv_ctl->lay_cnt[e][lane] = c;
  p.lv_ctl->lay_pex[e][lane] = incl - c;
  p.lv_ctl->lay_cin[e][lane] = wave_scan_incl((c + 63u) >> 6);
  if (lane == 63) p.lv_ctl->lay_base[e + 1] = p.lv_ctl->lay_base[e] + incl;
}

// Chunk schedule of a launch: the first p.lv_static_pct % of the chunks
// static (wave w of the grid's W waves takes chunks w, w + W, ...: no
// atomics, but imbalanced when ray costs vary a lot, C4), the rest dynamic
// over LV_CLAIMS sharded counters, counter j handing out chunks
// S + j, S + j + LV_CLAIMS, ...; a wave starts at its home counter (wave id
// mod LV_CLAIMS) and, once that is exhausted, reads all counters (one load
// per lane, no atomic) and moves to one that is not.
struct LvSched {
  uint32_t* ctrs;              // this launch's claim counters (ctrs[j * 32])
  uint32_t next, step, j, pct;
  __device__ __forceinline__ LvSched(uint32_t* claim_ctrs, int static_pct) : ctrs(claim_ctrs), pct((uint32_t)static_pct) {
    next = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    step = gridDim.x * (blockDim.x >> 6);
    j = next & (LV_CLAIMS - 1);
  }
  __device__ __forceinline__ int wave_id() const { return (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)); }
  __device__ __forceinline__ bool claim(uint32_t chunks, uint32_t& c) {
    const uint32_t S = (uint32_t)(((uint64_t)chunks * pct) / 100);
    if (next < S) {
      c = next;
      next += step;
      return true;
    }
    if (S == chunks) return false;
    const int lane = (int)__lane_id();
    while (true) {
      uint32_t k = 0;
      if (lane == 0) k = atomicAdd(&ctrs[j * 32], 1u);
      c = S + j + LV_CLAIMS * (uint32_t)__shfl((int)k, 0);
      if (c < chunks) return true;
      // counter j is exhausted: look at all of them (plain loads past L1)
      bool open = false;
      if (lane < LV_CLAIMS) {
        const uint32_t v = __hip_atomic_load(&ctrs[lane * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        open = S + (uint32_t)lane + LV_CLAIMS * v < chunks;
      }
      const uint64_t m = __ballot(open);
      if (!m) return false;
      const uint64_t rot = (m >> j) | (m << ((64 - j) & 63));   // the next open counter after j
      j = (j + (uint32_t)__builtin_ctzll(rot)) & (LV_CLAIMS - 1);
    }
  }
};

// Exclusive wave prefix of `cnt` plus one atomicAdd of the wave's total on
// `ctr` (skipped when the total is 0): the lane's first offset.
__device__ __forceinline__ uint32_t lv_wave_alloc(uint32_t* ctr, int cnt) {
  const int incl = (int)wave_scan_incl((uint32_t)cnt);
  const int wtotal = __shfl(incl, 63);
  uint32_t wbase = 0;
  if (wtotal > 0) {
    if (__lane_id() == 0) wbase = atomicAdd(ctr, (uint32_t)wtotal);
    wbase = (uint32_t)__shfl((int)wbase, 0);
  }
  return wbase + (uint32_t)(incl - cnt);
}

// LDS staging of the sphere records / hierarchy of a walk workgroup.
template <int SPH, int BS>
__device__ __forceinline__ void lv_stage_scene(const KParams& p, float4* lds_sph) {
  const SceneDev& S = p.scene;
  char* lds = reinterpret_cast<char*>(lds_sph);
  if (SPH == SPH_LIN_LDS) {
    for (int i = threadIdx.x; i < S.n_sphere + 4; i += BS) lds_sph[i] = reinterpret_cast<const float4*>(S.sph32)[i];
    __syncthreads();
  } else if (SPH == SPH_BVH_LDS || SPH == SPH_BVH_MIX || SPH == SPH_BVH_LDSX || SPH == SPH_BVH_QLDS) {
    const int nn = S.n_nodes * (int)(sizeof(Bvh4Node) / 16);
    for (int i = threadIdx.x; i < nn; i += BS) lds_sph[i] = reinterpret_cast<const float4*>(S.bvh)[i];
    if (SPH == SPH_BVH_QLDS) {
      uint4* q = reinterpret_cast<uint4*>(lds + p.lds_leaf);
      for (int i = threadIdx.x; i < S.n_slots / 2; i += BS) q[i] = reinterpret_cast<const uint4*>(S.bvh_q)[i];
    } else if (SPH != SPH_BVH_MIX) {
      float4* leaf = reinterpret_cast<float4*>(lds + p.lds_leaf);
      for (int i = threadIdx.x; i < S.n_slots; i += BS) leaf[i] = reinterpret_cast<const float4*>(S.bvh_sph32)[i];
    }
    if (SPH == SPH_BVH_LDSX) {
      float4* x = reinterpret_cast<float4*>(lds + p.lds_x64);
      for (int i = threadIdx.x; i < 2 * S.n_slots; i += BS) x[i] = reinterpret_cast<const float4*>(S.bvh_sph64)[i];
      int32_t* o = reinterpret_cast<int32_t*>(lds + p.lds_xobj);
      for (int i = threadIdx.x; i < S.n_slots; i += BS) o[i] = S.bvh_obj[i];
      float4* m = reinterpret_cast<float4*>(lds + p.lds_mat);
      const int nm = S.n_obj * (int)(sizeof(Material) / 16);
      for (int i = threadIdx.x; i < nm; i += BS) m[i] = reinterpret_cast<const float4*>(S.mat)[i];
      float4* sr = reinterpret_cast<float4*>(lds + p.lds_sphr);
      for (int i = threadIdx.x; i < 2 * S.n_sphere; i += BS) sr[i] = reinterpret_cast<const float4*>(S.sph64)[i];
      if (p.lds_lbuf >= 0) {                  // the light buffer (lbuf_stride words per light, a multiple of 8)
        uint4* lb = reinterpret_cast<uint4*>(lds + p.lds_lbuf);
        const int nw = S.lbuf_stride * S.n_light / 8;
        for (int i = threadIdx.x; i < nw; i += BS) lb[i] = reinterpret_cast<const uint4*>(S.lbuf)[i];
      }
      if (p.lds_rgate >= 0) {                 // the raise buffer's gates (rgate_stride 16-bit words per light, a multiple of 8)
        uint4* g = reinterpret_cast<uint4*>(lds + p.lds_rgate);
        const int nw = S.rgate_stride * S.n_light / 8;
        for (int i = threadIdx.x; i < nw; i += BS) g[i] = reinterpret_cast<const uint4*>(S.rgate)[i];
      }
    }
    __syncthreads();
  }
}

// One walk (EXTEND or SHADOW) through the launch's sphere mode.
// xrm (option exact_raises): a SHADOW walk of local_lights
// also checks the covers' acos raises: XR_BUF through the light buffer's cell
// and the raise buffer's lists (a target below the floor: the ordered linear
// walk), XR_WALK with the hierarchy walk widened to the light's cone; XR_NONE
// not.  A kernel variant each (the launcher picks XR_BUF where both buffers
// are in place): the widened walk's registers would cost XR_BUF's kernels.
enum { XR_NONE = 0, XR_BUF = 1, XR_WALK = 2 };
template <int SPH, int BS>
__device__ __forceinline__ bool lv_walk(const KParams& p, char* lds, bool ext, V3 o, V3 d, V3 L, double rad,
                                        double& best, int& besti, V3& hit, bool& hin, double& total, uint32_t& err,
                                        int xrm, int light = -1) {
  const SceneDev& S = p.scene;
  const bool xr = xrm != XR_NONE && !ext;
  // the light buffer's cell (§3.18): staged in LDS with the sphere records
  // (SPH_BVH_LDSX), read from global memory beside C4's 16-bit leaves;
  // exact_raises: the raise buffer's gates, staged in LDS beside the light buffer or global
  const uint16_t* gates = xrm == XR_BUF && S.rgate && light >= 0
                              ? (p.lds_rgate >= 0 ? reinterpret_cast<const uint16_t*>(lds + p.lds_rgate)
                                                  : S.rgate) + (size_t)light * S.rgate_stride
                              : nullptr;
  if (SPH == SPH_BVH_LDSX && !ext && xrm != XR_WALK && light >= 0 && p.lds_lbuf >= 0) {
    int* cov_i = reinterpret_cast<int*>(lds + p.lds_cov) + threadIdx.x;
    double* cov_v = reinterpret_cast<double*>(lds + p.lds_cov + COVER_K * BS * 4) + threadIdx.x;
    const uint16_t* lb = reinterpret_cast<const uint16_t*>(lds + p.lds_lbuf) + (size_t)light * S.lbuf_stride;
    if (query_lbuf<BS>(S, lb, reinterpret_cast<const float4*>(lds + p.lds_leaf),
                       reinterpret_cast<const Sphere64*>(lds + p.lds_x64),
                       reinterpret_cast<const int32_t*>(lds + p.lds_xobj), cov_i, cov_v, o, d, L, rad, best, besti,
                       hit, hin, total, err, xr, light, gates))
      return true;
  }
  if (SPH == SPH_BVH_QLDS && !ext && xrm != XR_WALK && light >= 0 && p.lv_lbuf && S.lbuf) {
    int* cov_i = reinterpret_cast<int*>(lds + p.lds_cov) + threadIdx.x;
    double* cov_v = reinterpret_cast<double*>(lds + p.lds_cov + COVER_K * BS * 4) + threadIdx.x;
    const QLeaf ql = {reinterpret_cast<const uint4*>(lds + p.lds_leaf), S.q_org[0], S.q_org[1], S.q_org[2],
                      S.q_step[0], S.q_step[1], S.q_step[2], S.q_rstep};
    if (query_lbuf<BS>(S, S.lbuf + (size_t)light * S.lbuf_stride, ql, S.bvh_sph64, S.bvh_obj, cov_i, cov_v, o, d, L,
                       rad, best, besti, hit, hin, total, err, xr, light, gates))
      return true;
  }
  if ((SPH == SPH_BVH_LDSX || SPH == SPH_BVH_QLDS) && xrm == XR_BUF && !ext) {
    // XR_BUF whose buffers could not serve this target (below the raise
    // buffer's floor, a degenerate ray): the ordered linear walk, raises checked
    total = 1.0;
    query<false>(S, cptr(S.sph32), false, o, d, L, rad, best, besti, hit, hin, total, err, nullptr, true);
    return true;
  }
  if (SPH == SPH_LIN_LDS) {
    query<false>(S, reinterpret_cast<const float*>(lds), ext, o, d, L, rad, best, besti, hit, hin, total, err,
                 nullptr, xr);
  } else if (SPH == SPH_LIN_SCALAR) {
    query<false>(S, cptr(S.sph32), ext, o, d, L, rad, best, besti, hit, hin, total, err, nullptr, xr);
  } else {
    int* stk = reinterpret_cast<int*>(lds + p.lds_stack) + threadIdx.x;
    int* cov_i = reinterpret_cast<int*>(lds + p.lds_cov) + threadIdx.x;
    double* cov_v = reinterpret_cast<double*>(lds + p.lds_cov + COVER_K * BS * 4) + threadIdx.x;
    int q_ref = BVH_NONE, q_sp = 0, q_ncov = 0;
    bool q_ovf = false;
    if (SPH == SPH_BVH_QLDS) {
      const QLeaf ql = {reinterpret_cast<const uint4*>(lds + p.lds_leaf), S.q_org[0], S.q_org[1], S.q_org[2],
                        S.q_step[0], S.q_step[1], S.q_step[2], S.q_rstep};
      query_bvh<BS, false>(S, reinterpret_cast<const Bvh4Node*>(lds), ql, S.bvh_sph64, S.bvh_obj,
                           qstack(lds, p), cov_i, cov_v, ext, o, d, L, rad, best, besti, hit, hin, total, err, q_ref,
                           q_sp, q_ncov, q_ovf, false, 0, xr);
    } else if (SPH == SPH_BVH_LDS)
      query_bvh<BS, false>(S, reinterpret_cast<const Bvh4Node*>(lds), reinterpret_cast<const float4*>(lds + p.lds_leaf),
                           S.bvh_sph64, S.bvh_obj, stk, cov_i, cov_v, ext, o, d, L, rad, best, besti, hit, hin, total,
                           err, q_ref, q_sp, q_ncov, q_ovf, false, 0, xr);
    else if (SPH == SPH_BVH_LDSX)
      query_bvh<BS, false>(S, reinterpret_cast<const Bvh4Node*>(lds), reinterpret_cast<const float4*>(lds + p.lds_leaf),
                           reinterpret_cast<const Sphere64*>(lds + p.lds_x64),
                           reinterpret_cast<const int32_t*>(lds + p.lds_xobj), stk, cov_i, cov_v, ext, o, d, L, rad,
                           best, besti, hit, hin, total, err, q_ref, q_sp, q_ncov, q_ovf, false, 0, xr);
    else if (SPH == SPH_BVH_MIX)
      query_bvh<BS, false>(S, reinterpret_cast<const Bvh4Node*>(lds), reinterpret_cast<const float4*>(S.bvh_sph32),
                           S.bvh_sph64, S.bvh_obj, stk, cov_i, cov_v, ext, o, d, L, rad, best, besti, hit, hin, total,
                           err, q_ref, q_sp, q_ncov, q_ovf, false, 0, xr);
    else
      query_bvh<BS, false>(S, S.bvh, reinterpret_cast<const float4*>(S.bvh_sph32), S.bvh_sph64, S.bvh_obj, stk, cov_i,
                           cov_v, ext, o, d, L, rad, best, besti, hit, hin, total, err, q_ref, q_sp, q_ncov, q_ovf,
                           false, 0, xr);
  }
  return true;
}

// The ray of a level's queue entry: a camera sample (level 0: `idx` = its
// item, Camera#lens_func) or the staged child at slot `idx`.  `valid` false
// for the padding of an 8x8 tile.
__device__ __forceinline__ void lv_ray(const KParams& p, int level, uint32_t idx, Item& cur, int& root, int& x, int& y,
                                       int& sample, bool& valid) {
  valid = true;
  if (level == 0) {
    root = (int)idx;
    const ItemPos ip = decode_item(p, root);
    x = p.x0 + ip.px;
    y = row_to_y(p, ip.row);
    sample = ip.sample;
    valid = ip.valid;
    if (valid) {
      const CameraDev& cam = *p.cam;
      cur.ray = lens_ray(cam, lens_target(cam, x, y), x, y, sample, p.seed);
      cur.att = v3(1.0, 1.0, 1.0);
      cur.path = 1;
    }
    return;
  }
  const double2* q = reinterpret_cast<const double2*>(lv_src(p, level) + (size_t)idx * p.lv_ray_dbl);
  const double2 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
  cur.ray.o = v3(a.x, a.y, b.x);
  cur.ray.d = v3(b.y, c.x, c.y);
  cur.att = v3(d.x, d.y, e.x);
  lv_ray_tail(p, q, e, cur.path, root, x, y, sample);
}

// The RNG key (x, y, sample) of a ray of tree `root` (lv_ray_tail leaves it
// -1 for an 80-B record): decode_item of the root, as lv_ray does at level 0.
__device__ __forceinline__ void lv_ray_key(const KParams& p, int root, int& x, int& y, int& sample) {
  if (x >= 0) return;
  const ItemPos ip = decode_item(p, root);
  x = p.x0 + ip.px;
  y = row_to_y(p, ip.row);
  sample = ip.sample;
}

// rt_map's tail once the lit areas are known (ray_tracer.rb:80-158): which
// children pass the cutoff (:52) at depth - 1, their slots in the next level
// (slice of this wave), the children in the reference's push order, else the
// local_lighting leaf; then the ray's tree record.  Shared by k_level and
// k_lv_shade; every lane of the wave calls it (the slot allocation is a wave
// operation).  errA/errS/errL/errP: the raises so far, in rt_map's order.
__device__ __forceinline__ void lv_finish(const KParams& p, int level, int slice, bool shade, bool active,
                                          const Item& cur, int root, int x, int y, int sample, int besti, bool hin,
                                          V3 hit, V3 delta, V3 nrm, V3 nn, double c, V3 lc, int nl, char* rec,
                                          int nleaf, uint32_t errA, uint32_t errS, uint32_t errL, uint32_t errP,
                                          const Material* m, bool last = false, bool keys = false) {
  const SceneDev& S = p.scene;
  const CameraDev& cam = *p.cam;
  const int depth = last ? 1 : cam.depth - level;   // last: the batch's last level (every child is cut off)
  const int pt = cam.pt;
  const uint64_t R = (uint64_t)pt + 3;
  uint32_t mask = 0;
  double rate = 0.0;
  bool may_refract = false;
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
  // Room in the next level: this wave's slice, wave prefix count + one
  // atomic.  The atomic is issued here and its value read only after the
  // reflection / refraction rays and the leaf are computed, so its round trip
  // overlaps that arithmetic instead of stalling the wave.
  const uint32_t log2cap = (uint32_t)p.lv_slice_log2, cap = 1u << log2cap;
  const int nch = __popc(mask);
  const int incl = (int)wave_scan_incl((uint32_t)nch);
  const int wtotal = __shfl(incl, 63);
  uint32_t wraw = 0;
  if (wtotal > 0 && __lane_id() == 0) wraw = atomicAdd(lv_slice_ctr(p.lv_ctl->sc[level + 1], slice), (uint32_t)wtotal);
  Ray refl, refr;
  bool has_refr = false;
  if (shade) {
    // intersect_parameters builds both rays for every hit (sphere.rb:88-101,
    // world_object.rb:121-137), and their normalizes can raise.  A child that
    // the cutoff drops (mask bit clear: always at the last level) needs only
    // those raises: the zero-vector test of its normalize (vnorm's own test,
    // sqrt(s) == 0 iff s == 0), not its direction.  The refraction's test
    // needs the reflected direction, so the reflection is built in full then.
    const bool refr_live = (mask & 2u) != 0;
    const bool refr_chk = may_refract && !refr_live && !(sqrt(1.0 - c * c) / rate >= 1);   // refraction()'s TIR test
    if ((mask & 1u) || refr_live || refr_chk) {
      refl = reflection(cur.ray, nn, c, hit, delta, errS);
    } else if (vr(vadd(vsc(nn, 2.0 * c * vr(cur.ray.d)), cur.ray.d)) == 0) {
      if (!errS) errS = ERR_ZERO_VEC;
    }
    if (refr_live) {
      has_refr = refraction(cur.ray, nn, c, hit, refl.d, rate, refr, errS);
    } else if (refr_chk && vr(vadd(refl.d, cur.ray.d)) == 0) {
      if (!errS) errS = ERR_ZERO_VEC;
    }
    if (nl != 0) {
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
      double* leafp = reinterpret_cast<double*>(rec + 8);
      leafp[0] = leaf.x;
      leafp[1] = leaf.y;
      leafp[2] = leaf.z;
      nleaf = 1;
    }
  }
  const uint32_t off0 = (wtotal > 0 ? (uint32_t)__shfl((int)wraw, 0) : 0u) + (uint32_t)(incl - nch);
  const uint32_t child0 = ((uint32_t)slice << log2cap) + off0;   // slot of the first child (k_tree_finalize)
  if (shade) {
    double* __restrict__ outs = p.lv_stage[(level + 1) & 1];
    uint32_t off = off0;
    auto put = [&](const Ray& r, V3 att, uint64_t path) {
      if (off < cap) {
        const uint32_t at = ((uint32_t)slice << log2cap) + off;
        lv_store_ray(p, outs + (size_t)at * p.lv_ray_dbl, r, att, path, root, x, y, sample);
        if (keys) p.lv_key[at] = (uint16_t)lv_ray_bin(S, r, p.lv_cell_bits);   // (the next level's binning)
      } else {
        lv_redo(p, root);
        atomicAdd(&p.lv_ctl->dropped, 1u);
      }
      off++;
    };
    if (mask & 1u) put(refl, vmul(cur.att, v3p(m->refl_att)), cur.path * R + 1);
    if (has_refr) put(refr, vmul(cur.att, v3p(m->refr_att)), cur.path * R + 2);
    if (nl == 0 && (mask >> 2) != 0) {
      // WorldObject#path_tracing (world_object.rb:76-90) from hit + delta.
      // Skipped when every path-tracing child is cut off: its only raise
      // sites (vertical_vector's zero test, the normalize of a vector with a
      // component 1) cannot fire unless n.normalize raised first (errS).
      const V3 att = vmul(cur.att, vdiv(v3p(m->diffuse), (double)pt));
      const V3 left = vnorm(vertical_vector(nrm, errP), errP);
      const V3 up = vcross(nn, left);
      Ray r;
      r.o = vadd(hit, delta);
      lv_ray_key(p, root, x, y, sample);
      for (int k = 0; k < pt; k++) {
        const double theta = rand01(p.seed, x, y, sample, cur.path, 2 * k) * PI / 2.0;
        const double phi = rand01(p.seed, x, y, sample, cur.path, 2 * k + 1) * PI * 2.0;
        double sth, cth, sph, cph;
        RTX_SINCOS(theta, &sth, &cth);
        RTX_SINCOS(phi, &sph, &cph);
        r.d = vadd(vsc(nn, sth), vsc(vadd(vsc(left, cph), vsc(up, sph)), cth));
        if (mask >> (2 + k) & 1u) put(r, att, cur.path * R + 3 + (uint64_t)k);
      }
    }
  }
  if (active) {
    uint32_t err = errA;
    if (!err) err = errS;
    if (!err) err = errL;
    if (!err) err = errP;
    *reinterpret_cast<uint2*>(rec) = make_uint2((err & 0xffu) | ((uint32_t)nleaf << 8) | (mask << 16), child0);
  }
}

// Level `level` (0 .. trace_depth-1) of one batch in one launch (option
// lv_split = 0).  Persistent, static chunk schedule.
template <int SPH, int BS, int XR>
__device__ __forceinline__ void k_level_body(const KParams& p, int level) {
  const SceneDev& S = p.scene;
  extern __shared__ float4 lds_sph[];
  char* lds = reinterpret_cast<char*>(lds_sph);
  LvQueue in;
  lv_in_queue(p, level, in);
  if (in.chunks == 0) return;                 // uniform: before any barrier
  lv_stage_scene<SPH, BS>(p, lds_sph);
  const uint32_t base = lv_base(p, level);
  const int depth = p.cam->depth - level;
  LvSched sched(p.lv_ctl->claim[0][level], p.lv_static_pct);
  const int slice = sched.wave_id() & (LV_SLICES - 1);

  unsigned long long tS[6] = {0, 0, 0, 0, 0, 0}, t0 = 0, t1, nchunks = 0;   // RTX_STAMPS diagnostic build only
  unsigned long long nA = 0, nE = 0, nS = 0;  // lanes with a ray, an EXTEND walk, a hit (per chunk, summed)
#define RTX_LV_STAMP(k)  \
  if (RTX_STAMPS) {      \
    t1 = stamp();        \
    tS[k] += t1 - t0;    \
    t0 = t1;             \
  }
  uint32_t chunk;
  const uint32_t nch = lv_chunks(p, in, level);
  while (sched.claim(nch, chunk)) {
    if (RTX_STAMPS) {
      t0 = stamp();
      nchunks++;
    }
    uint32_t slot, i;
    bool active = lv_chunk_item(p, in, level, chunk, slot, i);   // i: the ray's dense index in the level
    // ---- the ray: a camera sample (level 0) or a staged child
    Item cur;
    int root = 0, x = 0, y = 0, sample = 0;
    bool alive = false;
    if (active) {
      bool valid;
      lv_ray(p, level, slot, cur, root, x, y, sample, valid);
      if (level == 0) p.lv_redo_of[i] = -1;   // no overflow yet (lv_redo)
      active = valid;                         // tile padding: no record
      alive = valid && (level > 0 || !(depth <= 0 || vr(cur.att) < 0.0001));   // rt_map's cutoff (ray_tracer.rb:52)
      if (active && base + i >= p.lv_lcap) {  // no room for this ray's record
        lv_redo(p, root);
        active = alive = false;
      }
    }
    char* rec = p.lv_rec + (size_t)(base + i) * p.lv_rec_bytes;
    double* leafp = reinterpret_cast<double*>(rec + 8);

    // ---- rt_map: highlights (ray_tracer.rb:60-75)
    uint32_t errA = 0, errS = 0, errL = 0, errP = 0;
    int nleaf = 0;
    bool fired = false, hl_defer = false;
    if (alive)
      fired = highlight_leaves(S, cur, [&](V3 c) {
        leafp[3 * nleaf] = c.x;
        leafp[3 * nleaf + 1] = c.y;
        leafp[3 * nleaf + 2] = c.z;
        nleaf++;
      }, errA, [&](V3, V3, double, int) {         // lit_area's raise: deferred to k_hl_raise
        hl_defer = true;
        return false;
      });
    lv_hl_defer(p, hl_defer, cur.ray, base + i, [&] { return root; });
    RTX_LV_STAMP(0)
    // ---- World#intersect (world.rb:37-59)
    const bool ext = alive && !fired;
    double best = S.max_distance, total = 0.0;
    int besti = -1;
    V3 hit = v3(0.0, 0.0, 0.0);
    bool hin = true;
    if (ext) lv_walk<SPH, BS>(p, lds, true, cur.ray.o, cur.ray.d, hit, 0.0, best, besti, hit, hin, total, errL, XR_NONE);
    const bool shade = ext && besti >= 0;
    if (RTX_STAMPS) {
      nA += __popcll(__ballot(active));
      nE += __popcll(__ballot(ext));
      nS += __popcll(__ballot(shade));
    }
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
    // light loop (world_object.rb:51-74): one SHADOW walk per light.
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
      lv_walk<SPH, BS>(p, lds, false, qo, vsub(qL, qo), qL, L.radius, b2, bi2, h2, in2, tot, errL, XR, li);
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
    lv_finish(p, level, slice, shade, active, cur, root, x, y, sample, besti, hin, hit, delta, nrm, nn, c, lc, nl, rec,
              nleaf, errA, errS, errL, errP, shade ? &S.mat[besti] : S.mat, false, p.lv_sort && level + 1 >= p.lv_sort);
    RTX_LV_STAMP(5)
  }
#undef RTX_LV_STAMP
  if (RTX_STAMPS && __lane_id() == 0) {
    for (int k = 0; k < 6; k++) atomicAdd(&rtx_stamps[k], tS[k]);
    atomicAdd(&rtx_stamps[6], nchunks);
    atomicAdd(&rtx_stamps[7], 1ull);
    atomicAdd(&rtx_stamps[8], nA);
    atomicAdd(&rtx_stamps[9], nE);
    atomicAdd(&rtx_stamps[10], nS);
    unsigned long long* lv = rtx_stamps_lv + 8 * (level < 7 ? level : 7);
    for (int k = 0; k < 6; k++) atomicAdd(&lv[k], tS[k]);
    atomicAdd(&lv[6], nchunks);
    atomicAdd(&lv[7], nS);
  }
}

template <int SPH, int BS, int XR>
__global__ __launch_bounds__(BS, RTX_LVL_WPS) void k_level(KParams p, int level) {
  k_level_body<SPH, BS, XR>(p, level);
  lv_level_done(p, level + 1);
}

// ----------------------------------------------------------------- hit compaction
// Option lv_compact.  In k_level the shading half of a chunk
// (intersect_parameters, the shadow walks of local_lights, local_lighting and
// the children) runs on the lanes whose ray hit something, ~64 % of them on
// C2.  k_level_c splits every chunk at that point: each wave first runs the
// highlights and the nearest-hit walk for 64 rays, writes the records of the
// rays that stop there, and parks the hits in its own LDS ring (a ballot rank
// gives each hit its slot); whenever 64 hits are parked it pops them and runs
// the shading half on a full wave.  Every ray sees the same operations on the
// same values as in k_level, so the trees, hence the frames, are bit-identical.
//
// Ring: LV_RING slots per wave, structure of arrays (field f of slot k at
// (f * LV_RING + k) * 8 bytes: consecutive lanes hit consecutive banks); at
// most 63 hits stay parked between chunks, so 63 + 64 < LV_RING never overwrite
// an unread slot.  A parked hit: the hit point, the ray's origin and
// direction, {dense index, queue slot}, {object | :in << 31, raises}.  The
// rest of the ray (attenuation, path, RNG key) is reloaded from the level's
// queue (level 0: the camera sample's item).
//
// A compact ring (RF = 5 fields: the hit point, {dense index, queue slot},
// {object | :in, raises}) is used when the full one does not fit next to the
// walk's LDS (C4's hierarchy): the second half then re-derives the ray's
// origin and direction, the same bits either way (level >= 1: reloaded from
// the queue; level 0: Camera#lens_func re-evaluated for the item's key).
constexpr int LV_RING = 128;
constexpr int LV_RING_FIELDS = 11;
constexpr int LV_RING_FIELDS_SMALL = 5;
constexpr size_t LV_RING_WAVE_BYTES = (size_t)LV_RING * LV_RING_FIELDS * 8;
constexpr size_t LV_RING_WAVE_BYTES_SMALL = (size_t)LV_RING * LV_RING_FIELDS_SMALL * 8;

template <int SPH, int BS, int RF, bool LAST, int XR, bool SORT>
__device__ __forceinline__ void k_level_c_body(const KParams& p, int level) {
  static_assert(RF == LV_RING_FIELDS || RF == LV_RING_FIELDS_SMALL, "ring layout");
  constexpr int FI = RF == LV_RING_FIELDS ? 9 : 3;   // ring field of {dense index, queue slot}
  const SceneDev& S = p.scene;
  extern __shared__ float4 lds_sph[];
  char* lds = reinterpret_cast<char*>(lds_sph);
  LvQueue in;
  lv_in_queue(p, level, in);
  if (in.chunks == 0) return;                 // uniform: before any barrier
  lv_stage_scene<SPH, BS>(p, lds_sph);
  const uint32_t base = lv_base(p, level);
  const int depth = LAST ? 1 : p.cam->depth - level;   // LAST: the batch's last level, compiled apart
  LvSched sched(p.lv_ctl->claim[0][level], p.lv_static_pct);
  const int slice = sched.wave_id() & (LV_SLICES - 1);
  const int lane = (int)__lane_id();
  double* ring = reinterpret_cast<double*>(lds + p.lds_ring + (threadIdx.x >> 6) * ((size_t)LV_RING * RF * 8));
  uint32_t head = 0, pend = 0;                // wave-uniform: first parked slot, parked hits
  bool got = true;
  const uint32_t nch = lv_chunks(p, in, level);

  unsigned long long tS[6] = {0, 0, 0, 0, 0, 0}, t0 = 0, t1, nchunks = 0;   // RTX_STAMPS diagnostic build only
  unsigned long long nA = 0, nE = 0, nS = 0;
#define RTX_LV_STAMP(k)  \
  if (RTX_STAMPS) {      \
    t1 = stamp();        \
    tS[k] += t1 - t0;    \
    t0 = t1;             \
  }
  while (true) {
    {                                         // first half, chunk by chunk, until 64 hits are parked
      uint32_t chunk = 0;
      if (got) got = sched.claim(nch, chunk);   // (never again once exhausted)
      if (RTX_STAMPS) t0 = stamp();
      if (got) {
        if (RTX_STAMPS) nchunks++;
        // ---- first half: the ray, rt_map's cutoff, highlights, World#intersect
        uint32_t slot, i;
        bool active = lv_chunk_item(p, in, level, chunk, slot, i);
        // A staged child's first half needs its origin and direction only: the
        // attenuation is read if a highlight fires, the root if the ray
        // overflows the record arena (the second half reloads the rest), so
        // the walk does not carry them.
        const double2* qs = reinterpret_cast<const double2*>(lv_src(p, level) + (size_t)slot * p.lv_ray_dbl);
        Item cur;
        int root = 0, x = 0, y = 0, sample = 0;
        bool alive = false;
        if (active) {
          bool valid = true;
          if (level == 0) {
            lv_ray(p, level, slot, cur, root, x, y, sample, valid);
            p.lv_redo_of[i] = -1;
          } else {
            const double2 a = qs[0], b = qs[1], c = qs[2];
            cur.ray.o = v3(a.x, a.y, b.x);
            cur.ray.d = v3(b.y, c.x, c.y);
          }
          active = valid;
          alive = valid && (level > 0 || !(depth <= 0 || vr(cur.att) < 0.0001));   // ray_tracer.rb:52
          if (active && base + i >= p.lv_lcap) {
            lv_redo(p, level == 0 ? root : lv_ray_root(p, qs));
            active = alive = false;
          }
        }
        char* rec = p.lv_rec + (size_t)(base + i) * p.lv_rec_bytes;
        double* leafp = reinterpret_cast<double*>(rec + 8);
        uint32_t errA = 0, errL = 0;
        int nleaf = 0;
        bool fired = false, hl_defer = false;
        if (alive)
          fired = highlight_leaves_att(S, cur.ray, [&] {
            if (level == 0) return cur.att;
            const double2 d = qs[3], e = qs[4];
            return v3(d.x, d.y, e.x);
          }, [&](V3 c) {
            leafp[3 * nleaf] = c.x;
            leafp[3 * nleaf + 1] = c.y;
            leafp[3 * nleaf + 2] = c.z;
            nleaf++;
          }, errA, [&](V3, V3, double, int) {         // lit_area's raise: deferred to k_hl_raise
        hl_defer = true;
        return false;
      });
        lv_hl_defer(p, hl_defer, cur.ray, base + i, [&] { return level == 0 ? root : lv_ray_root(p, qs); });
        RTX_LV_STAMP(0)
        const bool ext = alive && !fired;
        double best = S.max_distance, total = 0.0;
        int besti = -1;
        V3 hit = v3(0.0, 0.0, 0.0);
        bool hin = true;
        if (ext) lv_walk<SPH, BS>(p, lds, true, cur.ray.o, cur.ray.d, hit, 0.0, best, besti, hit, hin, total, errL, XR_NONE);
        const bool shade = ext && besti >= 0;
        if (RTX_STAMPS) {
          nA += __popcll(__ballot(active));
          nE += __popcll(__ballot(ext));
          nS += __popcll(__ballot(shade));
        }
        RTX_LV_STAMP(1)
        if (active && !shade) {                 // the ray ends here: its record (k_level's, no children)
          const uint32_t err = errA ? errA : errL;
          *reinterpret_cast<uint2*>(rec) = make_uint2((err & 0xffu) | ((uint32_t)nleaf << 8), 0u);
        }
        // park the hits: slot head + pend + (rank among the wave's hits)
        const uint64_t hm = __ballot(shade);
        if (shade) {
          const uint32_t k = (head + pend + (uint32_t)__popcll(hm & ((1ull << lane) - 1ull))) & (LV_RING - 1);
          double* r = ring + k;
          r[0 * LV_RING] = hit.x;
          r[1 * LV_RING] = hit.y;
          r[2 * LV_RING] = hit.z;
          if (RF == LV_RING_FIELDS) {
            r[3 * LV_RING] = cur.ray.o.x;
            r[4 * LV_RING] = cur.ray.o.y;
            r[5 * LV_RING] = cur.ray.o.z;
            r[6 * LV_RING] = cur.ray.d.x;
            r[7 * LV_RING] = cur.ray.d.y;
            r[8 * LV_RING] = cur.ray.d.z;
          }
          r[FI * LV_RING] = __builtin_bit_cast(double, (uint64_t)i | (uint64_t)slot << 32);
          r[(FI + 1) * LV_RING] = __builtin_bit_cast(
              double, (uint64_t)((uint32_t)besti | (hin ? 0x80000000u : 0u)) | (uint64_t)((errA & 0xffu) | (errL & 0xffu) << 8) << 32);
        }
        pend += (uint32_t)__popcll(hm);
        RTX_LV_STAMP(4)
      }
      if (pend < 64 && (got || pend == 0)) {
        if (!got) break;                        // no chunk left and nothing parked
        continue;                               // not a full wave of hits yet
      }
    }
    // ---- second half on up to 64 parked hits (64, except the final flush)
    const uint32_t take = pend < 64 ? pend : 64u;
    const bool shade = (uint32_t)lane < take;
    Item cur;
    V3 hit = v3(0.0, 0.0, 0.0);
    uint32_t i = 0, errA = 0, errL = 0, errS = 0, errP = 0;
    int besti = 0, root = 0, x = 0, y = 0, sample = 0;
    bool hin = true;
    if (shade) {
      const double* r = ring + ((head + (uint32_t)lane) & (LV_RING - 1));
      hit = v3(r[0 * LV_RING], r[1 * LV_RING], r[2 * LV_RING]);
      if (RF == LV_RING_FIELDS) {
        cur.ray.o = v3(r[3 * LV_RING], r[4 * LV_RING], r[5 * LV_RING]);
        cur.ray.d = v3(r[6 * LV_RING], r[7 * LV_RING], r[8 * LV_RING]);
      }
      const uint64_t is = __builtin_bit_cast(uint64_t, r[FI * LV_RING]);
      const uint64_t be = __builtin_bit_cast(uint64_t, r[(FI + 1) * LV_RING]);
      i = (uint32_t)is;
      besti = (int)((uint32_t)be & 0x7fffffffu);
      hin = ((uint32_t)be >> 31) != 0;
      errA = (uint32_t)(be >> 32) & 0xffu;
      errL = (uint32_t)(be >> 40) & 0xffu;
      if (level == 0) {                       // the camera sample: item i (lv_ray)
        root = (int)i;
        const ItemPos ip = decode_item(p, root);
        x = p.x0 + ip.px;
        y = row_to_y(p, ip.row);
        sample = ip.sample;
        cur.att = v3(1.0, 1.0, 1.0);
        cur.path = 1;
        if (RF != LV_RING_FIELDS) {             // Camera#lens_func again: the same bits (lv_ray)
          const CameraDev& cam = *p.cam;
          cur.ray = lens_ray(cam, lens_target(cam, x, y), x, y, sample, p.seed);
        }
      } else {                                // the staged child at its queue slot (lv_ray)
        const double2* q = reinterpret_cast<const double2*>(lv_src(p, level) + (size_t)(is >> 32) * p.lv_ray_dbl);
        if (RF != LV_RING_FIELDS) {
          const double2 a = q[0], b = q[1], c = q[2];
          cur.ray.o = v3(a.x, a.y, b.x);
          cur.ray.d = v3(b.y, c.x, c.y);
        }
        const double2 d = q[3], e = q[4];
        cur.att = v3(d.x, d.y, e.x);
        lv_ray_tail(p, q, e, cur.path, root, x, y, sample);
      }
    }
    head = (head + take) & (LV_RING - 1);
    pend -= take;
    char* rec = p.lv_rec + (size_t)(base + i) * p.lv_rec_bytes;
    RTX_LV_STAMP(4)
    V3 delta = hit, nrm = hit, nn = hit;
    double c = 0.0;
    // the hit object's material (and sphere record): LDS copies when staged
    // (SPH_BVH_LDSX), so shading's first loads do not queue behind the wave's
    // record and ray stores (vmcnt counts loads and stores in issue order)
    const Material* mats = SPH == SPH_BVH_LDSX ? reinterpret_cast<const Material*>(lds + p.lds_mat) : S.mat;
    const Material* m = shade ? mats + besti : mats;
    if (shade) {
      if (SPH == SPH_BVH_LDSX)
        hit_info_m(S, *m, reinterpret_cast<const Sphere64*>(lds + p.lds_sphr), cur.ray, hit, delta, nrm, hin);
      else
        hit_info(S, besti, cur.ray, hit, delta, nrm, hin);
      nn = vnorm(nrm, errS);                  // n.normalize (world_object.rb:123)
      c = vcos(cur.ray.d, nrm, errS);         // ray.front.cos(-n): same bits as cos(n)
    }
    const V3 qo = vadd(hit, delta);           // the shadow rays' target point (world.rb:76)
    RTX_LV_STAMP(2)
    V3 lc = v3(0.0, 0.0, 0.0);
    int nl = 0;
    for (int li = 0; li < S.n_light; li++) {  // World#local_lights + local_lighting's light loop
      if (!shade) continue;
      const LightDev& L = S.light[li];
      const V3 qL = v3p(L.pos);
      double tot = 1.0;
      double b2 = 0.0;
      int bi2 = -1;
      V3 h2 = qo;
      bool in2 = true;
      lv_walk<SPH, BS>(p, lds, false, qo, vsub(qL, qo), qL, L.radius, b2, bi2, h2, in2, tot, errL, XR, li);
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
    lv_finish(p, level, slice, shade, shade, cur, root, x, y, sample, besti, hin, hit, delta, nrm, nn, c, lc, nl, rec, 0,
              errA, errS, errL, errP, m, LAST, SORT);
    RTX_LV_STAMP(5)
  }
#undef RTX_LV_STAMP
  if (RTX_STAMPS && __lane_id() == 0) {
    for (int k = 0; k < 6; k++) atomicAdd(&rtx_stamps[k], tS[k]);
    atomicAdd(&rtx_stamps[6], nchunks);
    atomicAdd(&rtx_stamps[7], 1ull);
    atomicAdd(&rtx_stamps[8], nA);
    atomicAdd(&rtx_stamps[9], nE);
    atomicAdd(&rtx_stamps[10], nS);
    unsigned long long* lv = rtx_stamps_lv + 8 * (level < 7 ? level : 7);
    for (int k = 0; k < 6; k++) atomicAdd(&lv[k], tS[k]);
    atomicAdd(&lv[6], nchunks);
    atomicAdd(&lv[7], nS);
  }
}

template <int SPH, int BS, int RF, bool LAST, int XR, bool SORT>
__global__ __launch_bounds__(BS, RTX_LVL_WPS) void k_level_c(KParams p, int level) {
  k_level_c_body<SPH, BS, RF, LAST, XR, SORT>(p, level);
  lv_level_done(p, level + 1);
}

// ----------------------------------------------------------------- split phases
// Option lv_split = 1: every level runs as three launches,
// each over a dense queue, so a wave's 64 lanes do the same phase of rt_map:
//   k_lv_trace   every ray of the level: highlights (world.rb:83-98) and the
//                nearest-hit walk (World#intersect, world.rb:37-59).  A ray
//                that stops here (dead, fired, miss) writes its tree record;
//                a hit goes to the level's hit queue (sliced like the ray
//                queues): {hit, hit + delta, ray, object, :in, slot, raises}.
//   k_lv_shadow  every (hit, light) pair: World#lit_area's walk (world.rb:62-80)
//                from hit + delta towards the light -> {1 - covers, raise}.
//   k_lv_shade   every hit: intersect_parameters, local_lights' colour,
//                the children (reflection, refraction, path tracing) into the
//                next level and the local_lighting leaf; the tree record.
// The phases evaluate the same operations on the same values as k_level
// (hit_info re-evaluated from the stored hit gives its bits again), so the
// trees, hence the frames, are bit-identical to the fused kernel's.
#ifndef RTX_LV_WALK_WPS
#define RTX_LV_WALK_WPS 3                 // waves per SIMD k_lv_trace / k_lv_shadow are compiled for
#endif
#ifndef RTX_LV_SHADE_WPS
#define RTX_LV_SHADE_WPS 3                // k_lv_shade (no walk)
#endif
constexpr int BS_SHADE = 256;

template <int SPH, int BS>
__global__ __launch_bounds__(BS, RTX_LV_WALK_WPS) void k_lv_trace(KParams p, int level) {
  const SceneDev& S = p.scene;
  extern __shared__ float4 lds_sph[];
  char* lds = reinterpret_cast<char*>(lds_sph);
  LvQueue in;
  lv_in_queue(p, level, in);
  if (in.chunks == 0) return;                 // uniform: before any barrier
  lv_stage_scene<SPH, BS>(p, lds_sph);
  const uint32_t base = lv_base(p, level);
  const int depth = p.cam->depth - level;
  LvSched sched(p.lv_ctl->claim[0][level], p.lv_static_pct);
  const int slice = sched.wave_id() & (LV_SLICES - 1);
  const uint32_t hlog2 = (uint32_t)p.lv_hslice_log2, hcap = 1u << hlog2;
  uint32_t chunk;
  while (sched.claim(in.chunks, chunk)) {
    uint32_t s, off, i;
    bool active = in.item(chunk, s, off, i);
    const uint32_t slot = level == 0 ? i : (s << p.lv_slice_log2) + off;
    bool alive = false;
    Item cur;
    int root = 0, x = 0, y = 0, sample = 0;
    if (active) {
      bool valid;
      lv_ray(p, level, slot, cur, root, x, y, sample, valid);
      if (level == 0) p.lv_redo_of[i] = -1;   // no overflow yet (lv_redo)
      active = valid;                         // tile padding: no record
      alive = valid && (level > 0 || !(depth <= 0 || vr(cur.att) < 0.0001));   // rt_map's cutoff (ray_tracer.rb:52)
      if (active && base + i >= p.lv_lcap) {  // no room for this ray's record
        lv_redo(p, root);
        active = alive = false;
      }
    }
    char* rec = p.lv_rec + (size_t)(base + i) * p.lv_rec_bytes;
    double* leafp = reinterpret_cast<double*>(rec + 8);
    uint32_t errA = 0, errL = 0;
    int nleaf = 0;
    bool fired = false, hl_defer = false;
    if (alive)
      fired = highlight_leaves(S, cur, [&](V3 c) {
        leafp[3 * nleaf] = c.x;
        leafp[3 * nleaf + 1] = c.y;
        leafp[3 * nleaf + 2] = c.z;
        nleaf++;
      }, errA, [&](V3, V3, double, int) {         // lit_area's raise: deferred to k_hl_raise
        hl_defer = true;
        return false;
      });
    lv_hl_defer(p, hl_defer, cur.ray, base + i, [&] { return root; });
    const bool ext = alive && !fired;
    double best = S.max_distance, total = 0.0;
    int besti = -1;
    V3 hit = v3(0.0, 0.0, 0.0);
    bool hin = true;
    if (ext) lv_walk<SPH, BS>(p, lds, true, cur.ray.o, cur.ray.d, hit, 0.0, best, besti, hit, hin, total, errL, XR_NONE);
    bool shade = ext && besti >= 0;
    V3 delta = hit, nrm = hit;
    if (shade) hit_info(S, besti, cur.ray, hit, delta, nrm, hin);
    const uint32_t h = lv_wave_alloc(lv_slice_ctr(p.lv_ctl->sh[level], slice), shade ? 1 : 0);
    if (shade && h >= hcap) {                 // the hit queue's slice is full
      lv_redo(p, root);
      shade = false;
    }
    if (shade) {
      const V3 qo = vadd(hit, delta);         // the shadow rays' target point (world.rb:76)
      double2* q = reinterpret_cast<double2*>(p.lv_hit + (size_t)(((uint32_t)slice << hlog2) + h) * HIT_DOUBLES);
      q[0] = make_double2(hit.x, hit.y);
      q[1] = make_double2(hit.z, qo.x);
      q[2] = make_double2(qo.y, qo.z);
      q[3] = make_double2(
          __builtin_bit_cast(double, (uint64_t)i | (uint64_t)((uint32_t)besti | (hin ? 0x80000000u : 0u)) << 32),
          __builtin_bit_cast(double, (uint64_t)slot | (uint64_t)((errA & 0xffu) | (errL & 0xffu) << 8) << 32));
    } else if (active) {
      uint32_t err = errA;
      if (!err) err = errL;
      *reinterpret_cast<uint2*>(rec) = make_uint2((err & 0xffu) | ((uint32_t)nleaf << 8), 0u);
    }
  }
}

template <int SPH, int BS>
__global__ __launch_bounds__(BS, RTX_LV_WALK_WPS) void k_lv_shadow(KParams p, int level) {
  const SceneDev& S = p.scene;
  extern __shared__ float4 lds_sph[];
  char* lds = reinterpret_cast<char*>(lds_sph);
  const uint32_t nL = (uint32_t)S.n_light;
  const uint32_t hlog2 = (uint32_t)p.lv_hslice_log2;
  LvQueue in;
  in.sliced(p.lv_ctl->sh[level], 1u << hlog2, nL);
  if (in.chunks == 0) return;
  lv_stage_scene<SPH, BS>(p, lds_sph);
  LvSched sched(p.lv_ctl->claim[1][level], p.lv_static_pct);
  uint32_t chunk;
  while (sched.claim(in.chunks, chunk)) {
    uint32_t s, off, t;
    if (in.item(chunk, s, off, t)) {          // (lanes past their slice idle until the next chunk)
      const uint32_t hs = (s << hlog2) + off / nL, li = off % nL;   // hit slot, light
      const double* q = p.lv_hit + (size_t)hs * HIT_DOUBLES;
      const double2 a = *reinterpret_cast<const double2*>(q + 2), b = *reinterpret_cast<const double2*>(q + 4);
      const V3 qo = v3(a.y, b.x, b.y);
      const LightDev& L = S.light[li];
      const V3 qL = v3p(L.pos);
      double tot = 1.0, b2 = 0.0;
      int bi2 = -1;
      V3 h2 = qo;
      bool in2 = true;
      uint32_t err = 0;
      lv_walk<SPH, BS>(p, lds, false, qo, vsub(qL, qo), qL, L.radius, b2, bi2, h2, in2, tot, err,
                       p.exact_raises != 0 ? XR_WALK : XR_NONE);   // (split phases: the widened walk, at run time)
      reinterpret_cast<double2*>(p.lv_area)[(size_t)hs * nL + li] =
          make_double2(tot, __builtin_bit_cast(double, (uint64_t)err));
    }
  }
}

__device__ __forceinline__ void k_lv_shade_body(const KParams& p, int level) {
  const SceneDev& S = p.scene;
  const uint32_t hlog2 = (uint32_t)p.lv_hslice_log2;
  LvQueue in;
  in.sliced(p.lv_ctl->sh[level], 1u << hlog2, 1u);
  if (in.chunks == 0) return;
  const uint32_t base = lv_base(p, level);
  const int nL = S.n_light;
  LvSched sched(p.lv_ctl->claim[2][level], p.lv_static_pct);
  const int slice = sched.wave_id() & (LV_SLICES - 1);
  uint32_t chunk;
  while (sched.claim(in.chunks, chunk)) {
    uint32_t s, off, t;
    const bool shade = in.item(chunk, s, off, t);
    const uint32_t hs = (s << hlog2) + off;   // hit slot
    V3 hit = v3(0.0, 0.0, 0.0);
    uint32_t i = 0, errA = 0, errL = 0, errS = 0, errP = 0;
    int besti = 0;
    bool hin = true;
    Item cur;
    int root = 0, x = 0, y = 0, sample = 0;
    if (shade) {
      const double2* q = reinterpret_cast<const double2*>(p.lv_hit + (size_t)hs * HIT_DOUBLES);
      const double2 a = q[0], b = q[1], d = q[3];
      hit = v3(a.x, a.y, b.x);
      const uint64_t ib = __builtin_bit_cast(uint64_t, d.x), se = __builtin_bit_cast(uint64_t, d.y);
      i = (uint32_t)ib;
      besti = (int)((uint32_t)(ib >> 32) & 0x7fffffffu);
      hin = (ib >> 63) != 0;
      errA = (uint32_t)(se >> 32) & 0xffu;
      errL = (uint32_t)(se >> 40) & 0xffu;
      bool valid;
      lv_ray(p, level, (uint32_t)se, cur, root, x, y, sample, valid);
    }
    char* rec = p.lv_rec + (size_t)(base + i) * p.lv_rec_bytes;
    V3 delta = hit, nrm = hit, nn = hit;
    double c = 0.0;
    if (shade) {
      hit_info(S, besti, cur.ray, hit, delta, nrm, hin);   // the bits k_lv_trace computed
      nn = vnorm(nrm, errS);                  // n.normalize (world_object.rb:123)
      c = vcos(cur.ray.d, nrm, errS);         // ray.front.cos(-n): same bits as cos(n)
    }
    // World#local_lights' areas (k_lv_shadow) into local_lighting's light loop
    V3 lc = v3(0.0, 0.0, 0.0);
    int nl = 0;
    for (int li = 0; li < nL; li++) {
      if (!shade) continue;
      const double2 ar = reinterpret_cast<const double2*>(p.lv_area)[(size_t)hs * nL + li];
      seterr(errL, (uint32_t)__builtin_bit_cast(uint64_t, ar.y));
      const double tot = ar.x;
      const double area = tot > 0 ? tot : 0.0;
      if (area > 0) {
        const LightDev& L = S.light[li];
        nl++;
        const double pw = S.sse_is_two ? area * area : rx_pow(area, S.sse);
        const V3 lcol = vsc(v3p(L.color), pw / (double)nL);
        const V3 ll = vnorm(vsub(v3p(L.pos), hit), errP);
        double ldn = vdot(ll, nn);
        if (ldn > 1) ldn = 1.0;
        else if (ldn < 0) ldn = 0.0;
        lc = vadd(lc, vsc(lcol, ldn));
      }
    }
    lv_finish(p, level, slice, shade, shade, cur, root, x, y, sample, besti, hin, hit, delta, nrm, nn, c, lc, nl, rec,
              0, errA, errS, errL, errP, shade ? &S.mat[besti] : S.mat);
  }
}

__global__ __launch_bounds__(BS_SHADE, RTX_LV_SHADE_WPS) void k_lv_shade(KParams p, int level) {
  k_lv_shade_body(p, level);
  lv_level_done(p, level + 1);
}

// ----------------------------------------------------------------- tree reduction
// The batch's level layout for the reductions: base[d] = first record of level
// d, pex[d * 64 + s] = dense index of slice s's first ray at level d (d >= 1).
// Block 0 also adds the batch's level statistics to lv_acc (rtx_level_stats):
// every level launch of the batch has ended.
__device__ __forceinline__ void lv_layout(const KParams& p, int nlev, uint32_t* base, uint32_t* pex) {
  const int t = (int)threadIdx.x;
  for (int w = t; w < nlev * 64; w += (int)blockDim.x)
    if (w >= 64) pex[w] = p.lv_ctl->lay_pex[w >> 6][w & 63];
  if (t <= nlev && t <= LV_MAXL) base[t] = p.lv_ctl->lay_base[t];
  if (blockIdx.x == 0 && p.lv_acc) {
    // atomic: the two halves of a two-stream render add into the same totals
    if (t == 0) atomicAdd(&p.lv_acc[0], (unsigned long long)p.lv_ctl->redo_n);
    if (t == 1) atomicAdd(&p.lv_acc[1], (unsigned long long)p.lv_ctl->dropped);
    if (t < nlev)
      atomicAdd(&p.lv_acc[2 + t], (unsigned long long)(p.lv_ctl->lay_base[t + 1] - p.lv_ctl->lay_base[t]));
  }
  __syncthreads();
}

// Sum of one camera sample's tree (level-0 item `root`) in trace_sync's
// order: pre-order, children in reverse slot order.  Returns the first raise
// (rt_map's first, else rt_reduce's).  The walk keeps one pending child range
// per level below the root in lo[k * st] / hi[k * st], k < sd (LDS, word-major
// over the block's threads, or a private array with st = 1).
__device__ __forceinline__ V3 lv_tree_sum(const KParams& p, const uint32_t* base, const uint32_t* pex, int root,
                                          int nlev, uint32_t* lo, uint32_t* hi, int st, int sd, uint32_t& err_out,
                                          uint32_t& nvis) {
  int sp = 0;
  V3 sum = v3(0.0, 0.0, 0.0);
  uint32_t err = 0, pf = 0;
  bool gt1 = false;
  int lev = 0;
  uint32_t q = (uint32_t)root;
  const uint32_t log2cap = (uint32_t)p.lv_slice_log2;
  while (true) {
    const char* rec = p.lv_rec + (size_t)(base[lev] + q) * p.lv_rec_bytes;
    nvis++;                                    // (rays of the tile: rtx_tile_rays)
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
      // the children's slot -> their dense index at level lev + 1
      const uint32_t c0 = pex[(lev + 1) * 64 + (hdr.y >> log2cap)] + (hdr.y & ((1u << log2cap) - 1u));
      lo[sp * st] = c0;
      hi[sp * st] = c0 + nch;
      sp++;
      // the children's records (contiguous, slot order) are fetched now, all
      // at once: the walk's dependent chain becomes the tree's depth, not
      // its size (the loads' values are consumed only at the end)
      const char* r0 = p.lv_rec + (size_t)(base[lev + 1] + c0) * p.lv_rec_bytes;
      pf += *reinterpret_cast<const uint32_t*>(r0) +
            *reinterpret_cast<const uint32_t*>(r0 + (size_t)(nch - 1) * p.lv_rec_bytes);
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

// One camera sample's colour and first raise: its tree, or the lanes engine's
// record when the sample overflowed the level buffers.
__device__ __forceinline__ V3 lv_sample(const KParams& p, const uint32_t* base, const uint32_t* pex, int item,
                                        int nlev, uint32_t* lo, uint32_t* hi, int st, int sd, uint32_t& e,
                                        uint32_t& nvis) {
  const int r = p.lv_redo_of[item];
  if (r >= 0) {
    const double* q = p.lv_redo_smp + (size_t)r * 4;
    e = (uint32_t)__builtin_bit_cast(uint64_t, q[3]);
    return v3(q[0], q[1], q[2]);
  }
  return lv_tree_sum(p, base, pex, item, nlev, lo, hi, st, sd, e, nvis);
}

// render_at's per-pixel stage of pass 0 (camera.rb:70-99) once a tile's
// 64 x pre sample colours / raises are in LDS (scol, serr): 64 threads, one
// per pixel of the tile.
__device__ __forceinline__ void lv_tile_pixels(const KParams& p, const double* scol, const uint32_t* serr, int slot) {
  const int pre = p.pre;
  const int l = (int)threadIdx.x;
  if (l >= 64) return;
  const int tiles_x = (p.nx + 7) >> 3;
  const int tile = p.lv_t0 + slot * p.lv_tstride;
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

// Camera#render_at's reduction (camera.rb:70-99) of pass 0: one 256-thread
// block per 8x8 tile of the batch.  The block's threads sum the tile's
// 64 x pre sample trees (item order (pixel, sample): a wave's trees are
// neighbours), park colour and raise in LDS, then 64 threads do the pixels:
// mean in sample order, the variance test, then the pixel or (max_sample_times
// > pre) an extra-list entry with the pre mean parked in the output.
// Dynamic LDS: nlev * 64 slice offsets, SD * 2 words of walk stack per thread,
// then 64 * pre samples.
template <int SD>
__global__ __launch_bounds__(256) void k_tree_finalize(KParams p, int nlev) {
  __shared__ uint32_t base[LV_MAXL + 1];
  extern __shared__ uint32_t lds_fin[];
  uint32_t* pex = lds_fin;
  const unsigned long long ts0 = RTX_STAMPS ? stamp() : 0ull;   // RTX_STAMPS diagnostic build only
  __shared__ uint32_t trays;                   // the tile's rays (rtx_tile_rays)
  if (threadIdx.x == 0) trays = 0;             // (lv_layout's barrier orders it before every add)
  lv_layout(p, nlev, base, pex);               // once per block: every tile of the batch shares it
  const unsigned long long ts1 = RTX_STAMPS ? stamp() : 0ull;
  const int pre = p.pre;
  uint32_t* lo = lds_fin + nlev * 64 + threadIdx.x;
  uint32_t* hi = lo + SD * 256;
  double* scol = reinterpret_cast<double*>(lds_fin + nlev * 64 + (SD > 16 ? 0 : 2 * SD * 256));   // 64 * pre * 3
  uint32_t* serr = reinterpret_cast<uint32_t*>(scol + 64 * pre * 3);
  uint32_t lo_p[SD > 16 ? LV_MAXL : 1], hi_p[SD > 16 ? LV_MAXL : 1];  // deep trees: private stack
  const int n_items = 64 * pre;
  // one block per tile, or (lv_fin_tiles > gridDim.x) a grid-stride loop over
  // the batch's tiles, so the layout above is read once per block
  const int n_tiles = p.lv_fin_tiles > (int)gridDim.x ? p.lv_fin_tiles : (int)gridDim.x;
  for (int slot = blockIdx.x; slot < n_tiles; slot += gridDim.x) {
    const int item0 = slot * n_items;
    uint32_t nvis = 0;
    for (int it = (int)threadIdx.x; it < n_items; it += 256) {
      const ItemPos ip = decode_item(p, item0 + it);
      if (!ip.valid) continue;
      uint32_t e = 0;
      const V3 c = SD > 16 ? lv_sample(p, base, pex, item0 + it, nlev, lo_p, hi_p, 1, LV_MAXL, e, nvis)
                           : lv_sample(p, base, pex, item0 + it, nlev, lo, hi, 256, SD, e, nvis);
      scol[3 * it] = c.x;
      scol[3 * it + 1] = c.y;
      scol[3 * it + 2] = c.z;
      serr[it] = e;
    }
    if (p.tile_rays) atomicAdd(&trays, nvis);
    __syncthreads();
    if (p.tile_rays && threadIdx.x == 0) {    // rtx_tile_rays
      p.tile_rays[p.lv_t0 + slot * p.lv_tstride] = trays;
      trays = 0;
    }
    lv_tile_pixels(p, scol, serr, slot);
    __syncthreads();                           // scol / serr / trays are reused by the next tile
  }
  if (RTX_STAMPS) {                           // layout / walks + pixels (wave lifetime parts), waves
    const unsigned long long ts2 = stamp();
    if (__lane_id() == 0) {
      atomicAdd(&rtx_stamps[11], ts1 - ts0);
      atomicAdd(&rtx_stamps[12], ts2 - ts1);
      atomicAdd(&rtx_stamps[13], 1ull);
    }
  }
}

// Pass 1: one thread per extra-list entry of the batch: (pre mean * pre +
// the extra samples in order) / max_sample_times.
template <int SD>
__global__ __launch_bounds__(256) void k_tree_finalize_extra(KParams p, int nlev) {
  __shared__ uint32_t base[LV_MAXL + 1];
  extern __shared__ uint32_t lds_fin[];
  uint32_t* pex = lds_fin;
  lv_layout(p, nlev, base, pex);
  uint32_t* lo = lds_fin + nlev * 64 + threadIdx.x;
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
    uint32_t e = 0, nv = 0;
    const int item = t * n_extra + j;
    cv = vadd(cv, SD > 16 ? lv_sample(p, base, pex, item, nlev, lo_p, hi_p, 1, LV_MAXL, e, nv)
                          : lv_sample(p, base, pex, item, nlev, lo, hi, 256, SD, e, nv));
    if (!err) err = e;
  }
  const V3 r = vdiv(vadd(vsc(avg, (double)pre), cv), (double)p.max_samples);
  o[0] = r.x;
  o[1] = r.y;
  o[2] = r.z;
  // an extra sample's raise: after any pre-sample raise of this pixel, which
  // pass 0 recorded with phase 0 (render_at traces the pre samples first)
  if (err) record_error(p.err, err, px_key(x, y, cam.height, 1));
}

// The batch's deferred highlight rays (lv_hl_defer): each thread re-runs
// World#high_lights for one listed ray, now with lit_area_raises for every
// light that fires (in light order, after that light's own cos raise, as
// rt_map meets them), and rewrites the raise byte of the ray's record.  The
// walk reads the hierarchy from LDS when the launcher staged it (`stage` 1:
// small hierarchies) or from global memory (L2-resident), its stack in LDS
// (bvh_stack words per thread).  `stage` 2 (scenes of at most 256 spheres,
// C2): one wave per listed ray instead, its lanes testing the spheres side by
// side (lit_area raises iff some sphere's cover_area does, whatever the
// order), which replaces a lane's walk over the whole cone by a few ballots.
// Grid-stride over the device-side counts; workgroups with no entry leave.
__device__ __forceinline__ bool lit_area_raises_wave(const SceneDev& S, V3 T, V3 L, double radius) {
  if (!(radius > 0.0) || S.n_sphere == 0) return false;   // as lit_area_raises
  const V3 lt = vsub(L, T);
  for (int b = 0; b < S.n_sphere; b += 64) {
    const int i = b + (int)__lane_id();
    bool r = false;
    if (i < S.n_sphere) {
      const Sphere64 sp = S.sph64[i];
      r = penumbra_raises(v3p(sp.c), sp.r, T, lt, radius);
    }
    if (__ballot(r)) return true;
  }
  return false;
}

__global__ __launch_bounds__(256) void k_hl_raise(KParams p, int stage) {
  extern __shared__ int lds_hl[];
  const SceneDev& S = p.scene;
  const uint32_t n = p.lv_ctl->hl_n < p.lv_hlq_cap ? p.lv_ctl->hl_n : p.lv_hlq_cap;
  if (stage == 2) {                           // one wave per entry (every lane loads it: uniform flow)
    const uint32_t w0 = blockIdx.x * 4u + (threadIdx.x >> 6), nw = gridDim.x * 4u;
    for (uint32_t e = w0; e < n; e += nw) {
      const double2* q = reinterpret_cast<const double2*>(p.lv_hlq + (size_t)e * HLQ_DOUBLES);
      const double2 a = q[0], b = q[1], c = q[2], d = q[3];
      Ray r;
      r.o = v3(a.x, a.y, b.x);
      r.d = v3(b.y, c.x, c.y);
      const uint32_t rec = (uint32_t)__builtin_bit_cast(uint64_t, d.x);
      uint32_t err = 0;
      highlight_leaves_att(S, r, [] { return v3(0.0, 0.0, 0.0); }, [](V3) {}, err,
                           [&](V3 T, V3 L, double rad, int) { return lit_area_raises_wave(S, T, L, rad); });
      if (__lane_id() == 0) {
        uint32_t* h = reinterpret_cast<uint32_t*>(p.lv_rec + (size_t)rec * p.lv_rec_bytes);
        *h = (*h & ~0xffu) | (err & 0xffu);
      }
    }
    return;
  }
  if (blockIdx.x * 256u >= n) return;          // uniform per workgroup
  const Bvh4Node* nodes = S.bvh_root != BVH_NONE ? S.bvh : nullptr;
  const float4* leaf4 = reinterpret_cast<const float4*>(S.bvh_sph32);
  int* stk = lds_hl + threadIdx.x;
  if (stage == 1 && nodes) {
    float4* l = reinterpret_cast<float4*>(lds_hl);
    const int nn = S.n_nodes * (int)(sizeof(Bvh4Node) / 16);
    for (int k = threadIdx.x; k < nn; k += 256) l[k] = reinterpret_cast<const float4*>(S.bvh)[k];
    for (int k = threadIdx.x; k < S.n_slots; k += 256) l[nn + k] = leaf4[k];
    __syncthreads();
    nodes = reinterpret_cast<const Bvh4Node*>(l);
    leaf4 = l + nn;
    stk += (nn + S.n_slots) * 4;
  }
  for (uint32_t e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
    const double2* q = reinterpret_cast<const double2*>(p.lv_hlq + (size_t)e * HLQ_DOUBLES);
    const double2 a = q[0], b = q[1], c = q[2], d = q[3];
    Ray r;
    r.o = v3(a.x, a.y, b.x);
    r.d = v3(b.y, c.x, c.y);
    const uint32_t rec = (uint32_t)__builtin_bit_cast(uint64_t, d.x);
    uint32_t err = 0;
    highlight_leaves_att(S, r, [] { return v3(0.0, 0.0, 0.0); }, [](V3) {}, err, [&](V3 T, V3 L, double rad, int li) {
      // the light and raise buffers when built, else / below their floor the walk
      if (stage == 3) {
        const int b = lit_area_raises_lbuf(S, li, T, L, rad);
        if (b >= 0) return b != 0;
      }
      return lit_area_raises(S, nodes, leaf4, S.bvh_sph64, stk, 256, T, L, rad);
    });
    uint32_t* h = reinterpret_cast<uint32_t*>(p.lv_rec + (size_t)rec * p.lv_rec_bytes);
    *h = (*h & ~0xffu) | (err & 0xffu);
  }
}

static hipError_t launch_hl_raise(const KParams& q, hipStream_t s) {
  if (q.scene.n_light == 0 || !q.lv_hlq) return hipSuccess;
  // up to 256 spheres: a wave per entry over the spheres (C2); else the walk, the
  // hierarchy staged in LDS when small (every workgroup with entries copies it)
  const size_t hier = (size_t)q.scene.n_nodes * sizeof(Bvh4Node) + (size_t)q.scene.n_slots * 16;
  // (stage 3: larger scenes with the light and raise buffers: their lists, the global hierarchy as fallback)
#ifndef RTX_HL_BUF_SMALL
#define RTX_HL_BUF_SMALL 1
#endif
  const bool bufs = q.scene.lbuf && q.scene.rbuf;
  const int stage = bufs && (RTX_HL_BUF_SMALL || q.scene.n_sphere > 256) ? 3
                    : q.scene.n_sphere <= 256                                ? 2
                    : q.scene.bvh_root != BVH_NONE && hier <= 16 * 1024      ? 1 : 0;
  const size_t lds = stage == 2 ? 0 : (stage == 1 ? hier : 0) + (size_t)std::max(1, q.scene.bvh_stack) * 256 * 4;
  int cus = 0, per_cu = 0;
  hipError_t e = launch_fit(reinterpret_cast<const void*>(k_hl_raise), 256, lds, cus, per_cu);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_hl_raise, dim3((unsigned)std::max(1, cus * std::min(per_cu, 4))), dim3(256), lds, s, q,
                     stage);
  return hipGetLastError();
}

// Per batch: the control block (count0 = the batch's level-0 items, pass 1:
// from the device-side extra count; the slice counters of levels 1..nlev),
// the lanes engine's work counter (the re-render launch); the call's first
// batch also the extra-list count and the level statistics.  (Every level-0
// lane sets its item's redo slot to -1.)  Grid-stride over the words.
__global__ __launch_bounds__(256) void k_level_begin(KParams p, int n0_max, int first, int nlev) {
  const int t = blockIdx.x * 256 + (int)threadIdx.x;
  const int nt = gridDim.x * 256;
  if (t == 0) {
    *p.work = 0;
    uint32_t v;
    if (p.lv_pass == 0) {
      v = (uint32_t)n0_max;
    } else {
      const int left = *p.extra_count - p.lv_e0;
      const int ent = left < 0 ? 0 : (left < p.lv_entries ? left : p.lv_entries);
      v = (uint32_t)(ent * (p.max_samples - p.pre));
    }
    p.lv_ctl->count0 = v;
    p.lv_ctl->redo_n = 0;
    p.lv_ctl->dropped = 0;
    p.lv_ctl->hl_n = 0;
    p.lv_ctl->lay_base[0] = 0;
    p.lv_ctl->lay_base[1] = v;
  }
  if (t < LV_MAXL + 2) p.lv_ctl->done[t] = 0;
  const int dwords = (nlev + 1 < LV_MAXL + 1 ? nlev + 1 : LV_MAXL + 1) * LV_DONE * 32;
  for (int w = t; w < dwords; w += nt) (&p.lv_ctl->done_sub[0][0])[w] = 0;
  if (first) {
    if (t == 0) *p.extra_count = 0;
    if (p.lv_acc && t < LV_MAXL + 3) p.lv_acc[t] = 0;
  }
  const int words = (nlev + 1 < LV_MAXL + 1 ? nlev + 1 : LV_MAXL + 1) * LV_SLICES * 32;
  for (int w = t; w < words; w += nt) {
    (&p.lv_ctl->sc[0][0])[w] = 0;
    (&p.lv_ctl->sh[0][0])[w] = 0;
  }
  if (p.lv_sort)
    for (int w = t; w < (8 << (3 * p.lv_cell_bits)); w += nt) p.lv_bins[w] = 0;   // (k_lv_bin_scan zeroes them after each level)
  const int cwords = (nlev < LV_MAXL + 1 ? nlev : LV_MAXL + 1) * LV_CLAIMS * 32;
  for (int w = t; w < cwords; w += nt)
    for (int k = 0; k < 3; k++) (&p.lv_ctl->claim[k][0][0])[w] = 0;
}

// ----------------------------------------------------------------- ray binning
// One counting-sort pass over a level's rays by bin (option lv_sort; lv_ray_bin
// above): counts, exclusive prefix (k_lv_bin_scan), scatter into lv_perm.  The
// producing level wrote each staged ray's bin beside it (lv_key, by queue
// slot).  Workgroup g takes a contiguous range of the level's chunks (the
// queue order, LvQueue), counts its rays per bin in LDS and then touches each
// bin it saw once in global memory: the count adds its range's count, the
// scatter reserves its range's places and, in a second pass over the range,
// places each ray (LDS cursors).  A popular bin's counter word takes one
// atomic per workgroup: one per wave and distinct bin measured 0.5 ms per C2
// level (r10b), one per 1,024 rays 0.1 ms (r10c).  The order inside a bin is
// the workgroups' order, which cannot change a result.
constexpr int BIN_UNROLL = 4;              // chunks a wave has in flight
constexpr int BIN_BS = 1024;               // one workgroup per CU: the counts take 128 KB of LDS
constexpr int BIN_WAVES = BIN_BS / 64;
template <bool SCATTER>
__global__ __launch_bounds__(BIN_BS) void k_lv_bin(KParams p, int level) {
  extern __shared__ uint32_t hist[];        // [nb] the range's count per bin (scatter: then its next place)
  const int nb = 8 << (3 * p.lv_cell_bits);
  LvQueue in;
  lv_in_queue(p, level, in);
  const int t = (int)threadIdx.x, wv = t >> 6;
  const uint16_t* key = p.lv_key;
  const uint32_t per = (in.chunks + gridDim.x - 1) / gridDim.x;
  const uint32_t c0 = blockIdx.x * per, c1 = c0 + per < in.chunks ? c0 + per : in.chunks;
  for (int k = t; k < nb; k += BIN_BS) hist[k] = 0u;
  __syncthreads();
  // chunks c0 + wv + W (u + BIN_UNROLL k): each wave BIN_UNROLL chunks at a time
  auto sweep = [&](auto&& fn) {
    for (uint32_t c = c0 + (uint32_t)wv; c < c1; c += (uint32_t)(BIN_WAVES * BIN_UNROLL)) {
      uint32_t slot[BIN_UNROLL], idx[BIN_UNROLL], bin[BIN_UNROLL];
      bool ok[BIN_UNROLL];
#pragma unroll
      for (int u = 0; u < BIN_UNROLL; u++) {
        const uint32_t cu = c + (uint32_t)(BIN_WAVES * u);     // (uniform per wave)
        uint32_t s = 0, off = 0, i = 0;
        ok[u] = cu < c1 && in.item(cu, s, off, i);
        slot[u] = (s << p.lv_slice_log2) + off;
        idx[u] = i;
        bin[u] = ok[u] ? key[slot[u]] & (uint32_t)(nb - 1) : 0u;   // (written for this resolution: < nb)
      }
#pragma unroll
      for (int u = 0; u < BIN_UNROLL; u++)
        if (ok[u]) fn(bin[u], slot[u], idx[u]);
    }
  };
  sweep([&](uint32_t b, uint32_t, uint32_t) { atomicAdd(&hist[b], 1u); });
  __syncthreads();
  for (int k = t; k < nb; k += BIN_BS) {
    const uint32_t n = hist[k];
    if (!n) continue;
    if (SCATTER) hist[k] = atomicAdd(&p.lv_bins[LV_BINS + k], n);   // this range's first place in bin k
    else atomicAdd(&p.lv_bins[k], n);
  }
  if (!SCATTER) return;
  __syncthreads();
  // (lv_sort_copy: each record moves to its place too, read in queue order, written in bin order)
  double* dst = p.lv_sorted;
  sweep([&](uint32_t b, uint32_t slot, uint32_t i) {
    const uint32_t at = atomicAdd(&hist[b], 1u);
    p.lv_perm[at] = make_uint2(slot, i);
    if (dst) {
      const double2* s2 = reinterpret_cast<const double2*>(p.lv_stage[level & 1] + (size_t)slot * p.lv_ray_dbl);
      double2* d2 = reinterpret_cast<double2*>(p.lv_sorted + (size_t)at * p.lv_ray_dbl);
      for (int w = 0; w < p.lv_ray_dbl / 2; w++) d2[w] = s2[w];
    }
  });
}

// The bins' exclusive prefix into the cursors; the counts zeroed for the next
// level.  One workgroup of 1024 threads, nb / 1024 consecutive bins each
// (4 or 32), all loaded at once: one memory round trip instead of one per bin
// (the loop over a run-time count issued them one at a time: 71 us per C4
// level, r11v).
__global__ __launch_bounds__(1024) void k_lv_bin_scan(KParams p, int level) {
  constexpr int PMAX = (8 << (3 * LV_CELL_BITS_MAX)) / 1024;   // (32,768 bins)
  const int per = (8 << (3 * p.lv_cell_bits)) / 1024;
  __shared__ uint32_t part[16];
  const int t = (int)threadIdx.x, lane = t & 63, wv = t >> 6;
  uint32_t v[PMAX];
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < PMAX; k++) {
    v[k] = k < per ? p.lv_bins[per * t + k] : 0u;
    sum += v[k];
  }
  const uint32_t incl = wave_scan_incl(sum);
  if (lane == 63) part[wv] = incl;
  __syncthreads();
  uint32_t pre = incl - sum;
  for (int k = 0; k < wv; k++) pre += part[k];
#pragma unroll
  for (int k = 0; k < PMAX; k++) {
    if (k >= per) break;
    p.lv_bins[LV_BINS + per * t + k] = pre;
    p.lv_bins[per * t + k] = 0u;
    pre += v[k];
  }
}

// Diagnostic builds: this unit's stamps (k_level), added by rtxdbg_read_stamps.
int read_level_stamps(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rtx_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rtx_stamps), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}

int levels_auto_mode(const SceneDev& S, int mode, int compact, int split) {
  if (mode != SPH_BVH_LDS || compact == 0 || split) return mode;
  const size_t waves = BS_BVH / 64;
  const size_t walk = (size_t)S.bvh_stack * BS_BVH * 4 + (size_t)COVER_K * BS_BVH * 12 + 64;
  const size_t nodes = (size_t)S.n_nodes * sizeof(Bvh4Node), leaves = (size_t)S.n_slots * 16;
  const size_t exact = (size_t)S.n_slots * (sizeof(Sphere64) + 4) + 16 + (size_t)S.n_obj * sizeof(Material) +
                       (size_t)S.n_sphere * sizeof(Sphere64);   // + shading's materials and sphere records
  // C2: the exact test's records staged too (r05d: 4.91-4.94 -> 4.85 ms, same bits)
  if (nodes + leaves + exact + walk + waves * LV_RING_WAVE_BYTES <= LDS_TOTAL_BYTES) return SPH_BVH_LDSX;
  if (nodes + leaves + walk + waves * LV_RING_WAVE_BYTES <= LDS_TOTAL_BYTES) return mode;   // LDS + full ring
  if (nodes + leaves + walk + waves * LV_RING_WAVE_BYTES_SMALL <= LDS_TOTAL_BYTES) return mode;   // + compact ring
  // C4: the leaves as 16-bit records, 16-bit stacks (+ alignment)
  const size_t walk16 = (size_t)S.bvh_stack * BS_BVH * 2 + (size_t)COVER_K * BS_BVH * 12 + 64;
  if (S.q_ok && nodes + (size_t)S.n_slots * 8 + walk16 + 32 + waves * LV_RING_WAVE_BYTES_SMALL <= LDS_TOTAL_BYTES)
    return SPH_BVH_QLDS;
  if (nodes + walk + waves * LV_RING_WAVE_BYTES_SMALL <= LDS_TOTAL_BYTES) return SPH_BVH_MIX;
  return mode;
}

extern "C" int rtxdbg_read_walkstats(unsigned long long* out, int reset) {   // diagnostic builds (levels unit)
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rtx_walkstats), sizeof(unsigned long long) * 8) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rtx_walkstats), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}

extern "C" int rtxdbg_read_level_stamps(unsigned long long* out, int reset) {   // diagnostic builds: [8 levels][8]
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rtx_stamps_lv), sizeof(unsigned long long) * 64) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[64] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(rtx_stamps_lv), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}

// ----------------------------------------------------------------- bounce-level launchers
static hipError_t cus_and_fit(const void* kern, int bs, size_t lds, int& cus, int& per_cu) {
  return launch_fit(kern, bs, lds, cus, per_cu);   // cached (rtx_kernels.hip)
}

template <typename K>
static hipError_t launch_timed(K kern, long blocks, int bs, size_t lds, hipStream_t s, KernelEvents* kev,
                               const KParams& q, int level) {
  if (blocks < 1) blocks = 1;
  const bool ev = kev && kev->n < kev->max;
  if (ev) (void)hipEventRecord(kev->ev[2 * kev->n], s);
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(bs), lds, s, q, level);
  const hipError_t e = hipGetLastError();
  if (ev) {
    (void)hipEventRecord(kev->ev[2 * kev->n + 1], s);
    kev->n++;
  }
  return e;
}

// k_level_c for a level: the batch's last level compiled apart; with ray
// binning (lv_sort) the other levels write their children's bins (SORT: a
// kernel of its own, the key's registers would cost the default one spills).
// xrm: XR_NONE / XR_BUF / XR_WALK (lv_walk); XR_BUF is instantiated only for
// the sphere modes with a light buffer (the others take XR_WALK).
template <int SPH, int BS, int RF, bool LAST, bool SORT>
static void (*level_c_xr(int xrm))(KParams, int) {
  constexpr bool BUF = SPH == SPH_BVH_LDSX || SPH == SPH_BVH_QLDS;
  if (xrm == XR_NONE) return k_level_c<SPH, BS, RF, LAST, XR_NONE, SORT>;
  if constexpr (BUF) if (xrm == XR_BUF) return k_level_c<SPH, BS, RF, LAST, XR_BUF, SORT>;
  return k_level_c<SPH, BS, RF, LAST, XR_WALK, SORT>;
}
template <int SPH, int BS, int RF>
static void (*level_c_kernel(bool last, int xrm, bool sort))(KParams, int) {
  if (last) return level_c_xr<SPH, BS, RF, true, false>(xrm);
  if (sort) return level_c_xr<SPH, BS, RF, false, true>(xrm);
  return level_c_xr<SPH, BS, RF, false, false>(xrm);
}

#ifndef RTX_LV_FUSED_BS
#define RTX_LV_FUSED_BS 0                  // k_level's block size (0: BS_LIN / BS_BVH)
#endif
template <int SPH>
constexpr int fused_bs() { return RTX_LV_FUSED_BS ? RTX_LV_FUSED_BS : (sph_is_bvh(SPH) ? BS_BVH : BS_LIN); }

// kind: 0 k_level (fused), 1 k_lv_trace, 2 k_lv_shadow.  Persistent: as many
// workgroups as fit at once, never more than cap_items need.
template <int SPH, int BS>
static hipError_t launch_level_bs(const KParams& p, int kind, int level, long cap_items, hipStream_t s,
                                  KernelEvents* kev) {
  KParams q = p;
  q.stk_slots_max = 0;                         // no ray stack in this engine
  size_t lds = lds_layout(q, SPH, BS);
  // exact_raises (the default) compiles the shadow walks' raise check in (k_level / k_level_c <..., XR>):
  // XR_BUF through the light and raise buffers where both serve this launch (the LDS-staged light
  // buffer of SPH_BVH_LDSX, the global one of SPH_BVH_QLDS), else XR_WALK; exact_raises = 0: XR_NONE
  const bool xr = q.exact_raises != 0;
  bool bufs = false;                           // (SPH_BVH_LDSX: settled below, once the rings are placed)
  if constexpr (SPH == SPH_BVH_QLDS) bufs = q.lv_lbuf && q.scene.lbuf && q.scene.rbuf;
  int xrm = !xr ? XR_NONE : bufs ? XR_BUF : XR_WALK;
  auto kern = kind == 0 ? (xrm == XR_NONE ? k_level<SPH, BS, XR_NONE> : k_level<SPH, BS, XR_WALK>)
              : kind == 1 ? k_lv_trace<SPH, BS> : k_lv_shadow<SPH, BS>;
  // hit compaction when the rings fit next to the walk's LDS (k_level_c is
  // instantiated for the fused kernel's block size only)
  int ring_fields = 0;
  if constexpr (BS == fused_bs<SPH>()) if (kind == 0 && q.lv_compact != 0) {
    constexpr bool BVH = sph_is_bvh(SPH);
    const size_t ring = (lds + 15) & ~(size_t)15, budget = BVH ? LDS_TOTAL_BYTES : LDS_LIN_BLOCK_BYTES;
    const size_t need = ring + (size_t)(BS / 64) * LV_RING_WAVE_BYTES;
    const size_t need_small = ring + (size_t)(BS / 64) * LV_RING_WAVE_BYTES_SMALL;
    if (need <= budget && q.lv_compact != 2) { // the full ring
      q.lds_ring = (int32_t)ring;
      lds = need;
      ring_fields = LV_RING_FIELDS;
    } else if (BVH && need_small <= budget) {  // the compact ring (C4-sized hierarchies)
      q.lds_ring = (int32_t)ring;
      lds = need_small;
      ring_fields = LV_RING_FIELDS_SMALL;
    }
  }
  // the light buffer (§3.18) after the rings, when it fits: the shadow walks read their cell's leaves;
  // with exact_raises the raise buffer's gates after it (§2.4), in LDS when they fit too
  if constexpr (SPH == SPH_BVH_LDSX) if (kind == 0 && q.lv_lbuf && q.scene.lbuf) {
    const size_t at = (lds + 15) & ~(size_t)15, bytes = (size_t)q.scene.lbuf_stride * q.scene.n_light * 2;
    if (at + bytes <= LDS_TOTAL_BYTES) {
      q.lds_lbuf = (int32_t)at;
      lds = at + bytes;
      if (xr && q.scene.rbuf) {
        xrm = XR_BUF;
        const size_t ga = (lds + 15) & ~(size_t)15, gb = (size_t)q.scene.rgate_stride * q.scene.n_light * 2;
        if (ga + gb <= LDS_TOTAL_BYTES) {
          q.lds_rgate = (int32_t)ga;
          lds = ga + gb;
        }
      }
    }
  }
  if constexpr (BS == fused_bs<SPH>()) {
    const bool last = level == q.lv_last_level, sort = q.lv_sort && level + 1 >= q.lv_sort;
    if (ring_fields == LV_RING_FIELDS) kern = level_c_kernel<SPH, BS, LV_RING_FIELDS>(last, xrm, sort);
    else if (ring_fields == LV_RING_FIELDS_SMALL) kern = level_c_kernel<SPH, BS, LV_RING_FIELDS_SMALL>(last, xrm, sort);
    else if (kind == 0 && xrm == XR_BUF) {     // (no ring: k_level, which walks the widened hierarchy)
      xrm = XR_WALK;
      q.lds_lbuf = q.lds_rgate = -1;
      kern = k_level<SPH, BS, XR_WALK>;
    }
  }
  int cus = 0, per_cu = 0;                     // (also raises the kernel's dynamic-LDS limit once)
  const hipError_t e = cus_and_fit(reinterpret_cast<const void*>(kern), BS, lds, cus, per_cu);
  if (e != hipSuccess) return e;
  const long grid = std::max<long>(1, (long)cus * per_cu / std::max(1, q.lv_grid_div));
  return launch_timed(kern, std::min<long>((cap_items + BS - 1) / BS, grid), BS, lds, s, kev, q, level);
}

// The fused kernel runs the engine's block sizes (BS_LIN / BS_BVH, 2 waves per
// SIMD).  The split walk kernels (3 waves per SIMD) take 256-thread blocks
// when three of them fit a CU's LDS, else the hierarchy's 512.
template <int SPH>
static hipError_t launch_level(const KParams& p, int kind, int level, long cap_items, hipStream_t s,
                               KernelEvents* kev) {
  constexpr bool BVH = sph_is_bvh(SPH);
  constexpr int FBS = fused_bs<SPH>();
  if (kind == 0) return launch_level_bs<SPH, FBS>(p, kind, level, cap_items, s, kev);
  if (BVH) {
    KParams q = p;
    q.stk_slots_max = 0;
    if (3 * lds_layout(q, SPH, 256) > LDS_TOTAL_BYTES)
      return launch_level_bs<SPH, BS_BVH>(p, kind, level, cap_items, s, kev);
  }
  return launch_level_bs<SPH, 256>(p, kind, level, cap_items, s, kev);
}

static hipError_t launch_level_mode(const KParams& p, int mode, int kind, int level, long cap, hipStream_t s,
                                    KernelEvents* kev) {
  switch (mode) {
    case SPH_LIN_LDS: return launch_level<SPH_LIN_LDS>(p, kind, level, cap, s, kev);
    case SPH_LIN_SCALAR: return launch_level<SPH_LIN_SCALAR>(p, kind, level, cap, s, kev);
    case SPH_BVH_LDS: return launch_level<SPH_BVH_LDS>(p, kind, level, cap, s, kev);
    case SPH_BVH_GLOBAL: return launch_level<SPH_BVH_GLOBAL>(p, kind, level, cap, s, kev);
    case SPH_BVH_MIX: return launch_level<SPH_BVH_MIX>(p, kind, level, cap, s, kev);
    case SPH_BVH_LDSX: return launch_level<SPH_BVH_LDSX>(p, kind, level, cap, s, kev);
    case SPH_BVH_QLDS: return launch_level<SPH_BVH_QLDS>(p, kind, level, cap, s, kev);
  }
  return hipErrorInvalidValue;
}

static hipError_t launch_shade(const KParams& p, int level, long cap_items, hipStream_t s, KernelEvents* kev) {
  int cus = 0, per_cu = 0;
  const hipError_t e = cus_and_fit(reinterpret_cast<const void*>(k_lv_shade), BS_SHADE, 0, cus, per_cu);
  if (e != hipSuccess) return e;
  return launch_timed(k_lv_shade, std::min<long>((cap_items + BS_SHADE - 1) / BS_SHADE, (long)cus * per_cu), BS_SHADE,
                      0, s, kev, p, level);
}

// A level's binning (option lv_sort): count, prefix, scatter; grids sized for
// the level's capacity (cap rays): one workgroup per CU, each a contiguous range of chunks.
static hipError_t launch_bins(const KParams& q, int level, long cap, hipStream_t s) {
  const size_t lds = (size_t)(8 << (3 * q.lv_cell_bits)) * 4;
  int cus = 0, per_cu = 0;                     // (also raises the kernels' dynamic-LDS limit)
  hipError_t e = cus_and_fit(reinterpret_cast<const void*>(k_lv_bin<false>), BIN_BS, lds, cus, per_cu);
  if (e == hipSuccess) e = cus_and_fit(reinterpret_cast<const void*>(k_lv_bin<true>), BIN_BS, lds, cus, per_cu);
  if (e != hipSuccess) return e;
  const long grid = std::max<long>(1, std::min<long>(cap / 4096, (long)cus * std::max(1, per_cu)));
  hipLaunchKernelGGL(k_lv_bin<false>, dim3((unsigned)grid), dim3(BIN_BS), lds, s, q, level);
  hipLaunchKernelGGL(k_lv_bin_scan, dim3(1), dim3(1024), 0, s, q, level);
  hipLaunchKernelGGL(k_lv_bin<true>, dim3((unsigned)grid), dim3(BIN_BS), lds, s, q, level);
  return hipGetLastError();
}

template <int SD>
static hipError_t launch_finalize_sd(const KParams& q, int nlev, int n, hipStream_t s) {
  const size_t stack = (size_t)nlev * 64 * 4 + (SD > 16 ? 0 : (size_t)SD * 2 * 256 * 4);
  if (q.lv_pass == 0) {                        // n = tiles of the batch
    const size_t lds = ((stack + 7) & ~(size_t)7) + (size_t)64 * q.pre * 28;
    KParams r = q;
    long grid = n;
    if (q.lv_fin_tiles > 0) {                  // lv_fin_grid blocks per CU, grid-stride over the tiles
      int dev = 0, cus = 0;
      if (hipGetDevice(&dev) == hipSuccess &&
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
        grid = std::min<long>(n, (long)cus * q.lv_fin_tiles);
    }
    r.lv_fin_tiles = n;
    hipLaunchKernelGGL(k_tree_finalize<SD>, dim3((unsigned)grid), dim3(256), lds, s, r, nlev);
  } else {                                     // n = extra-list entries of the batch
    hipLaunchKernelGGL(k_tree_finalize_extra<SD>, dim3((unsigned)((n + 255) / 256)), dim3(256), stack, s, q, nlev);
  }
  return hipGetLastError();
}

static hipError_t launch_finalize(const KParams& q, int nlev, int n, hipStream_t s) {
  // a walk keeps one pending child range per level below the root: nlev - 1
  // entries; the smaller stack lets 8 blocks share a CU (C2, depth 5) instead of 6
  if (nlev <= 5) return launch_finalize_sd<4>(q, nlev, n, s);
  if (nlev <= 8) return launch_finalize_sd<8>(q, nlev, n, s);
  if (nlev <= 16) return launch_finalize_sd<16>(q, nlev, n, s);
  return launch_finalize_sd<64>(q, nlev, n, s);
}

// One batch: reset, the levels, the lanes-engine re-render of overflowed
// samples (exits at once when there are none), the tree reduction.  A level's
// launches size their grids for its capacity (level 0: the batch's items;
// deeper levels: LV_SLICES full slices).
// One batch as a sequence of launch steps (step 0: k_level_begin; 1..nlev:
// the levels, each with its binning passes or split phases; then the deferred
// highlight checks, the lanes-engine re-render and the tree reduction), so
// that launch_levels can issue the steps of several parts' batches in turn
// (the host's launch cost otherwise delays part 1 by all of part 0's
// launches: 55 us of a 0.83 ms C2 1/8 share, r11j).
struct LevelBatch {
  KParams q;
  int mode, maxs, nlev, n0_max, fin_threads;
  hipStream_t s;
  KernelEvents* kev;
  bool first;
  hipEvent_t after_begin;
  int step = 0;
  bool done() const { return step > nlev + 1; }
  hipError_t next() {
    hipError_t e = hipSuccess;
    if (step == 0) {
      const int words = std::min(nlev + 1, LV_MAXL + 1) * LV_SLICES * 32;
      hipLaunchKernelGGL(k_level_begin, dim3((unsigned)std::min(64, (words + 255) / 256)), dim3(256), 0, s, q, n0_max,
                         first ? 1 : 0, nlev);
      e = hipGetLastError();
      if (e == hipSuccess && after_begin) e = hipEventRecord(after_begin, s);
    } else if (step <= nlev) {
      const int d = step - 1;
      const long scap = (long)LV_SLICES << q.lv_slice_log2, hcap = (long)LV_SLICES << q.lv_hslice_log2;
      const long cap = d == 0 ? (long)n0_max : scap;
      if (!q.lv_split) {
        if (q.lv_sort && d >= q.lv_sort) e = launch_bins(q, d, cap, s);
        if (e == hipSuccess) e = launch_level_mode(q, mode, 0, d, cap, s, kev);
      } else {
        const long hits = std::min(cap, hcap);
        e = launch_level_mode(q, mode, 1, d, cap, s, kev);
        if (e == hipSuccess && q.scene.n_light > 0)
          e = launch_level_mode(q, mode, 2, d, hits * q.scene.n_light, s, kev);
        if (e == hipSuccess) e = launch_shade(q, d, hits, s, kev);
      }
    } else {
      e = launch_hl_raise(q, s);
      if (e == hipSuccess) e = launch_redo(q, mode, maxs, n0_max, s);
      if (e == hipSuccess && fin_threads > 0) e = launch_finalize(q, nlev, fin_threads, s);
    }
    step++;
    return e;
  }
};

static hipError_t level_batch(KParams q, int mode, int maxs, int nlev, int n0_max, int fin_threads, hipStream_t s,
                              KernelEvents* kev, bool first, hipEvent_t after_begin = nullptr) {
  LevelBatch b{q, mode, maxs, nlev, n0_max, fin_threads, s, kev, first, after_begin};
  hipError_t e = hipSuccess;
  while (!b.done() && e == hipSuccess) e = b.next();
  return e;
}

hipError_t launch_levels(KParams p, int mode, int maxs, int nlev, int batch_tiles, hipStream_t s,
                         KernelEvents* kev, const LvAux* aux) {
  const int tiles = ((p.nx + 7) / 8) * ((p.nrows + 7) / 8);
  if (tiles == 0) return hipSuccess;
  mode = resolve_mode(p.scene, mode);
  batch_tiles = std::max(1, std::min(batch_tiles, tiles));
  const int per_tile = 64 * p.pre;
  p.tile_order = nullptr;
  if (aux && tiles < aux->parts) aux = nullptr;
  // The parts interleave tiles (tile t in part t mod P): neighbouring tiles
  // cost alike, so the parts are balanced and each one's tail overlaps the
  // others' work.
  const int stride = aux ? aux->parts : 1;
  hipError_t e = hipSuccess;                   // (the first batch's k_level_begin zeroes the extra count)
  // part j: the batches of the tiles j + stride * k (k < n_j) with the buffers of
  // its KParams on its stream; the parts' launch steps are issued in turn (one
  // step of each part, then the next), each part's in its own order
  const int parts = aux ? aux->parts : 1;
  std::vector<std::vector<LevelBatch>> seq(parts);
  for (int j = 0; j < parts; j++) {
    const KParams& base = j == 0 ? p : aux->pb[j - 1];
    const hipStream_t st = j == 0 ? s : aux->s2[j - 1];
    const int n = (tiles - j + stride - 1) / stride;
    for (int k0 = 0; k0 < n; k0 += batch_tiles) {
      KParams q = base;
      q.lv_pass = 0;
      q.lv_t0 = j + stride * k0;
      q.lv_tstride = stride;
      q.lv_tiles = std::min(batch_tiles, n - k0);
      q.lv_e0 = q.lv_entries = 0;
      const bool first = j == 0 && k0 == 0;
      seq[j].push_back(LevelBatch{q, mode, maxs, nlev, q.lv_tiles * per_tile, q.lv_tiles, st, kev, first,
                                  first && aux ? aux->ev_first : nullptr});
    }
  }
  std::vector<size_t> at(parts, 0);
  for (bool more = true; more && e == hipSuccess;) {
    more = false;
    for (int j = 0; j < parts && e == hipSuccess; j++) {
      if (at[j] >= seq[j].size()) continue;
      LevelBatch& b = seq[j][at[j]];
      // part j >= 1 starts after part 0's first k_level_begin has zeroed the shared totals
      if (j > 0 && at[j] == 0 && b.step == 0) e = hipStreamWaitEvent(aux->s2[j - 1], aux->ev_first, 0);
      if (e == hipSuccess) e = b.next();
      if (b.done()) at[j]++;
      more = more || at[j] < seq[j].size();
    }
  }
  for (int j = 1; aux && j < aux->parts && e == hipSuccess; j++) e = hipEventRecord(aux->ev_done[j - 1], aux->s2[j - 1]);
  for (int j = 1; aux && j < aux->parts && e == hipSuccess; j++) e = hipStreamWaitEvent(s, aux->ev_done[j - 1], 0);
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
    q.lv_tstride = 1;
    e = level_batch(q, mode, maxs, nlev, q.lv_entries * n_extra, q.lv_entries, s, kev, false);
  }
  return e;
}

}  // namespace rtx
