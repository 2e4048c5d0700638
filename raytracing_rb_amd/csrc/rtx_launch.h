// rtx_launch.h — kernel parameter block and launchers shared by the C-ABI
// (rtx_capi.cpp) and the kernels (rtx_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "rtx_scene.h"

namespace rtx {

// Reference raise sites recorded by the device (codes: ERR_* in rtx_vec3.h).
struct ErrState {
  unsigned int flags;              // bit (1 << code) for every code raised
  unsigned int pad;
  unsigned long long first[5];     // per ERR_ code (rtx_vec3.h): min key (pixels: (x*H + y)*2 + phase, render_sync order; rays: index)
};

// Bounce-level engine: one launch per tree level (or three,
// option lv_split).  The ray queue of every level >= 1 (and the hit queue of
// the split phases) is cut into LV_SLICES slices of 2^k slots, each with its
// own allocation counter on its own 128-B line (no contended device atomics).
constexpr int LV_MAXL = 64;                     // levels (= trace_depth) the engine supports
constexpr int LV_SLICES = 64;                   // slices per queue (one per lane of a consumer wave)
constexpr int LV_CLAIMS = 16;                   // sharded chunk-claim counters per launch
constexpr int LV_DONE = 16;                     // wave-completion counters per level launch (lv_level_done)
constexpr int LV_CELL_BITS_MAX = 4;             // ray bins (option lv_sort): origin cells per axis = 2^lv_cell_bits
constexpr int LV_BINS = 8 << (3 * LV_CELL_BITS_MAX); // x 8 direction octants: at most 32,768 bins
struct LevelCtl {
  uint32_t count0;                              // level-0 items of the batch
  uint32_t redo_n;                              // level-0 items handed to the lanes engine (capacity overflow)
  uint32_t dropped;                             // child rays that found no room (diagnostic)
  uint32_t hl_n;                                // highlight rays whose lit_area raise check is deferred (k_hl_raise)
  uint32_t pad[27];                             // (pad[0]: the lanes-engine work counter of parts 1..)
  uint32_t sc[LV_MAXL + 1][LV_SLICES * 32];     // rays allocated in slice s of level d: sc[d][32 s]
  uint32_t sh[LV_MAXL + 1][LV_SLICES * 32];     // split phases: hits of level d in slice s
  uint32_t claim[3][LV_MAXL + 1][LV_CLAIMS * 32]; // chunk claims: [launch kind: fused/trace, shadow, shade][level][j * 32]
  // compact layout of level d (written by the last workgroup of the launch that allocated it)
  uint32_t lay_cnt[LV_MAXL + 2][LV_SLICES];     // rays in slice s (clamped to the slice)
  uint32_t lay_pex[LV_MAXL + 2][LV_SLICES];     // exclusive ray prefix of slice s
  uint32_t lay_cin[LV_MAXL + 2][LV_SLICES];     // inclusive 64-ray chunk prefix of slice s
  uint32_t lay_base[LV_MAXL + 2];               // first record of level d in the arena
  uint32_t done[LV_MAXL + 2];                   // completed done_sub counters of the launch allocating level d
  uint32_t done_sub[LV_MAXL + 1][LV_DONE * 32]; // finished waves w (w mod LV_DONE = j) of that launch: [d][32 j]
};

struct KParams {
  SceneDev scene;                  // by value: read by scalar loads from the kernarg segment
  const CameraDev* cam;            // device copy (uploaded by rtx_camera_set)
  uint64_t seed;
  int32_t x0, nx, nrows;           // columns [x0, x0+nx); packed output rows
  int32_t y0, tile_rows, rank, nranks;   // tile_rows == 0: rows y0 .. y0+nrows-1
  const int32_t* row_tiles;        // non-null: packed tile k is image tile row_tiles[k] (rtx_render_tile_list_device)
  uint32_t* tile_rays;             // non-null (whole-frame level renders): rays per 8x8 tile, written by the reduction
  double* out;
  size_t stride;                   // doubles per output row
  ErrState* err;
  unsigned long long* counts;      // RTX_NCOUNT counters (counting launches only)
  int* work;                       // work-item counter of this launch (zeroed by the launcher)
  const double* rays;              // SRC_RAYS (rtx_trace): 6 doubles per ray, keys (x, y, sample)
  const int32_t* keys;
  int32_t nrays;
  // dynamic LDS layout (bytes), filled by launch_render/launch_trace
  int32_t lds_leaf, lds_stack, lds_cov, lds_items;
  int32_t lds_x64, lds_xobj;       // SPH_BVH_LDSX: staged Sphere64 records / object indices per leaf slot
  int32_t lds_lbuf;                // the light buffer staged in LDS (byte offset), or -1: shadow walks use the hierarchy
  int32_t lds_rgate;               // the raise buffer's gates staged in LDS (byte offset), or -1: read from global memory
  int32_t lds_mat, lds_sphr;       // SPH_BVH_LDSX: staged materials (per object) / Sphere64 records (per sphere)
  int32_t stk_slots;               // ray-stack entries per lane kept in LDS (set by the launcher)
  int32_t stk_slots_max;           // cap (option "lds_stack"; the stack bucket by default)
  double* stk_glb;                 // per-lane regions: lanes_maxs * 12 doubles of ray stack
  int32_t lanes_maxs;              // lanes engine: ray-stack entries per lane (8, 16, 32 or 64; set by the launcher)
  int32_t stk_glb_lanes;           // lanes the buffer holds (the launcher caps the grid to it)
  // Camera#render_at in two steps (launch_render): per (pixel, sample) records
  // of 4 doubles {r, g, b, first raise} at samples[(pixel * max(pre, max) + j) * 4]
  // (pixel = row * nx + column of the region), and the list of pixels whose
  // variance asks for the extra samples.
  int32_t pre, max_samples;        // camera pre_sample_times / max_sample_times
  int32_t postpone;                // query_bvh: postpone walks when fewer lanes than this still walk (0: never)
  double* samples;
  int32_t* extra_list;             // nx * nrows entries
  int32_t* extra_count;
  // SRC_PIXELS: tile visiting order (k_tile_cost + k_tile_sort), null = natural
  int32_t* tile_order;
  int32_t* tile_cls;
  // bounce-level engine: one batch = pass 0 (the pre samples of the pixels of
  // tiles lv_t0 + k * lv_tstride, k < lv_tiles) or pass 1 (the extra samples of extra-list
  // entries [lv_e0, lv_e0 + lv_entries)); level-0 item k of the batch is
  // decode_item(k); trees are stored per level in lv_rec (lv_rec_bytes each).
  int32_t lv_pass, lv_t0, lv_tiles, lv_e0, lv_entries;
  int32_t lv_tstride;              // 1, or 2 for the interleaved halves of a two-stream render
  uint32_t lv_scap;                // ray records per staging buffer (levels >= 1): LV_SLICES << lv_slice_log2
  int32_t lv_slice_log2;           // slots per slice of a level's ray queue (log2)
  int32_t lv_hslice_log2;          // split phases: slots per slice of a level's hit queue (log2)
  uint32_t lv_lcap;                // tree records in lv_rec
  int32_t lv_rec_bytes;
  LevelCtl* lv_ctl;
  double* lv_stage[2];             // level d reads lv_stage[d & 1], writes lv_stage[(d + 1) & 1]
  char* lv_rec;
  int32_t* lv_redo_of;             // per level-0 item: -1, or its entry in lv_redo_list
  int32_t* lv_redo_list;           // level-0 items re-rendered by the lanes engine (SRC_LIST)
  double* lv_redo_smp;             // their sample records {r, g, b, first raise}
  unsigned long long* lv_acc;      // per call: {redo_n, dropped, count[0..LV_MAXL]} summed over batches (or null)
  int32_t lv_split;                // 1: three phase launches per level (k_lv_trace / k_lv_shadow / k_lv_shade)
  int32_t lv_static_pct;           // % of a level launch's chunks scheduled statically (the rest: sharded claims)
  double* lv_hit;                  // split: hit queue, LV_HIT_BYTES per hit, LV_SLICES << lv_hslice_log2 slots
  double* lv_area;                 // split: {1 - covers, raise} per (hit, light)
  int32_t lv_compact;              // k_level: park hits in an LDS ring, shade full waves (-1 auto, 0 off, 1 on, 2 compact ring)
  int32_t lds_ring;                // k_level (compacting): LDS byte offset of the per-wave hit rings
  int32_t lv_last_level;           // trace_depth - 1 (-1 if trace_depth < 1): the level whose children are all
                                   // cut off, run by a k_level_c compiled for it
  int32_t lv_grid_div;             // level launches: persistent grid = resident workgroups / this (option lv_grid_div)
  int32_t lv_fin_tiles;            // tree reduction pass 0: tiles of the batch (grid-stride loop when the grid is smaller)
  int32_t lv_redo_blocks;          // the lanes-engine re-render of overflowed samples: at most this many workgroups (0: all resident)
  int32_t lv_ray_dbl;              // staged ray record, doubles: 10 (80 B: path < 2^32, RNG key decoded from the root) or 12
  int32_t exact_raises;            // 1: every shadow walk (local_lights) also checks its covers' acos raises (option exact_raises)
  uint32_t lv_hlq_cap;             // entries of lv_hlq
  double* lv_hlq;                  // highlight rays of the batch whose lit_area raise k_hl_raise checks (8 doubles each)
  // ray binning (option lv_sort): a level >= 1 is processed in the order of its
  // rays' bins (lv_ray_bin: direction octant, origin cell), records still at
  // their dense index
  int32_t lv_sort;                 // 0, or the first level binned before its launch (option lv_sort_from)
  int32_t lv_cell_bits;            // origin cells per axis of a bin = 2^lv_cell_bits (3 or 4: 4,096 or 32,768 bins)
  int32_t lv_lbuf;                 // 1: the fused level kernels' shadow walks use the light buffer when staged (option lbuf)
  uint16_t* lv_key;                // bin of each staged ray of the level being binned, by queue slot (k_lv_bin)
  uint2* lv_perm;                  // the level's rays in bin order: {queue slot, dense index}
  double* lv_sorted;               // lv_sort_copy: the binned level's ray records in bin order (k_lv_bin), or null
  uint32_t* lv_bins;               // LV_BINS counts, LV_BINS cursors (the first 8 << 3 lv_cell_bits used)
};

// Where the sphere walk reads its records:
enum SphMode : int {
  SPH_LIN_LDS = 0,       // ordered linear walk, float32 pre-test records staged in LDS
  SPH_LIN_SCALAR = 1,    // ordered linear walk, records by scalar loads
  SPH_BVH_LDS = 2,       // four-wide ball hierarchy, nodes + leaf records staged in LDS
  SPH_BVH_GLOBAL = 3,    // four-wide ball hierarchy, nodes + leaf records by scalar loads
  SPH_BVH_MIX = 4,       // four-wide ball hierarchy, nodes staged in LDS, leaf records from global memory
                         // (bounce-level engine only: room for the hit rings of k_level_c; the lanes
                         // engine walks it as SPH_BVH_LDS)
  SPH_BVH_LDSX = 5,      // as SPH_BVH_LDS, and the binary64 sphere records of the exact test with their
                         // object indices staged too (bounce-level engine only, small hierarchies: no
                         // global load inside the walk; the lanes engine walks it as SPH_BVH_LDS)
  SPH_BVH_QLDS = 6,      // four-wide ball hierarchy, nodes + 16-bit quantized leaf records (SceneDev::bvh_q)
                         // in LDS, 16-bit traversal stacks (bounce-level engine only, hierarchies too big for
                         // SPH_BVH_LDS next to a hit ring, e.g. C4; the lanes engine walks it as SPH_BVH_LDS)
};


// Sphere modes that walk the ball hierarchy.
constexpr bool sph_is_bvh(int m) {
  return m == SPH_BVH_LDS || m == SPH_BVH_GLOBAL || m == SPH_BVH_MIX || m == SPH_BVH_LDSX || m == SPH_BVH_QLDS;
}

// HIP event pairs recorded on the launch stream around every ray-tree kernel
// launch of one render call (option "kernel_events", rtx_kernel_time).
struct KernelEvents {
  hipEvent_t* ev;                  // 2 * max events: start, end of launch k at ev[2k], ev[2k+1]
  int n, max;
};

int stack_bucket(int need);
// Persistent-launch occupancy (CUs, resident blocks per CU) of `kern`, cached
// per (kernel, block size, dynamic LDS bytes, device); raises the kernel's
// dynamic-LDS limit on first use.
hipError_t launch_fit(const void* kern, int bs, size_t lds, int& cus, int& per_cu);
// mode: SphMode; a linear mode whose records exceed the LDS budget falls back to
// SPH_LIN_SCALAR, a BVH mode to SPH_BVH_GLOBAL.  Counting launches always walk
// linearly (the counters are the reference's brute-force events).
hipError_t launch_render(KParams p, int mode, bool count, int maxs, hipStream_t s, KernelEvents* kev = nullptr);
hipError_t launch_trace(KParams p, int mode, int maxs, hipStream_t s);
// Camera#render_at over the region of `p` with the bounce-level engine: nlev =
// trace_depth level launches per batch of `batch_tiles` 8x8 tiles (pass 0) or
// of batch_tiles * 64 * pre / (max - pre) extra-list entries (pass 1).  The
// lv_* buffers of `p` are the caller's: lv_redo_of / lv_rec / staging sized for
// batch_tiles * 64 * pre level-0 items; lanes-engine buffers (stk_glb) too, for
// the overflow re-render.
// Parts at once (option lv_streams = P > 1): pass 0's tiles interleaved over
// P parts, tile t in part t mod P; part 0 on `s` with the buffers of `p`,
// part j > 0 on s2[j - 1] with the buffers of pb[j - 1] (own level buffers,
// work counter and lanes-engine stacks; the extra-sample list and the
// statistics shared with `p`).  The parts j > 0 start after the first reset
// on `s` (ev_first); `s` waits for all of them (ev_done) before the extra
// samples (pass 1), which run on `s` alone.
constexpr int LV_MAX_PARTS = 4;
struct LvAux {
  int parts;                       // P (2 .. LV_MAX_PARTS)
  KParams pb[LV_MAX_PARTS - 1];
  hipStream_t s2[LV_MAX_PARTS - 1];
  hipEvent_t ev_first, ev_done[LV_MAX_PARTS - 1];
};
hipError_t launch_levels(KParams p, int mode, int maxs, int nlev, int batch_tiles, hipStream_t s,
                         KernelEvents* kev = nullptr, const LvAux* aux = nullptr);
// Tree-record bytes for a scene with n_light lights (one leaf per fired light).
int levels_rec_bytes(int n_light);
// The bounce-level engine's sphere mode for sphere_src auto: SPH_BVH_LDSX
// when the hierarchy, its exact records and the full hit ring fit LDS (C2);
// SPH_BVH_MIX when the staged hierarchy leaves no LDS for a hit ring while
// the hierarchy's nodes alone with the compact ring fit (C4); else SPH_BVH_LDS.
int levels_auto_mode(const SceneDev& S, int mode, int compact, int split);
constexpr size_t RAY_BYTES = 96;                // staged ray record of the bounce-level engine (at most)
constexpr size_t LV_HIT_BYTES = 64;             // split phases: hit-queue record
constexpr int LV_SPLIT_MAX_LIGHTS = 16;         // split phases only up to this many lights (shadow results per hit)
hipError_t launch_path_trace(KParams p, hipStream_t s);
// The lanes engine's re-render of the level-0 items listed in lv_redo_list
// (SRC_LIST; exits at once when the list is empty).
hipError_t launch_redo(const KParams& q, int mode, int maxs, int n, hipStream_t s);
int read_level_stamps(unsigned long long* out, int reset);   // diagnostic builds
int resolve_mode(const SceneDev& S, int mode);
// LDS bytes a hierarchy workgroup needs (nodes + leaf records + traversal
// stacks + cover lists) and the budget SPH_BVH_LDS has.
size_t bvh_lds_bytes(int n_nodes, int n_slots, int bvh_stack);
size_t bvh_lds_budget();
hipError_t launch_quantize(const double* rgb, int w, int h, size_t stride, int blend, uint8_t* out,
                           hipStream_t s);
// Rank-major packed tiles (n ranks x rows_per_rank rows x w x 3) -> frame rows.
hipError_t launch_unpack(const double* gathered, int w, int h, int tile_rows, int n, int rows_per_rank,
                         double* out, size_t stride, hipStream_t s);
hipError_t launch_unpack_plan(const double* gathered, int w, int h, int tile_rows, int n, int per_rank,
                              const int32_t* d_plan, double* out, size_t stride, hipStream_t s);
hipError_t launch_tile_probe(KParams p, int32_t* cls, hipStream_t s);

}  // namespace rtx
