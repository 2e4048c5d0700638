// rtx_capi.cpp — the C-ABI of librtx (include/rtx.h): scene/camera upload,
// render entry points, Vec3 helpers.  Host code; kernels in rtx_kernels.hip.
//
// Scene preparation restates the constructors of the reference
// (src/world.rb:15-34, src/objects/{sphere,plane,box,texture}.rb,
// src/camera.rb:26-34,129-151) with the same operation order, so every
// constant the device uses has the bits the Ruby code would compute.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <math.h>

#include <cmath>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <string>
#include <vector>

#include "../../include/rtx.h"
#include "rtx_launch.h"
#include "rtx_scene.h"
#include "rtx_vec3.h"

using namespace rtx;

#ifndef RTX_BVH_SAH
#define RTX_BVH_SAH 1                         // default hierarchy splits: 1 binned SAH, 0 median
#endif
#ifndef RTX_SAH_PUSHES
#define RTX_SAH_PUSHES 12                     // SAH only while <= this many traversal-stack entries sit above
#endif

constexpr unsigned RTX_WORK_RING = 256;
#ifndef RTX_POSTPONE_NODES
#define RTX_TILE_ORDER_SPHERES 512             // auto tile_order up to this many spheres
#define RTX_POSTPONE_NODES 64                 // hierarchy nodes from which walks are postponed by default
#endif

struct rtx_context {
  int device = 0;
  std::string err;
  // device scene
  std::vector<void*> d_bufs;         // every device allocation of the scene
  SceneDev scene{};
  SceneDev* d_scene = nullptr;
  bool have_scene = false;
  // camera
  CameraDev cam{};
  CameraDev* d_cam = nullptr;
  bool have_cam = false;
  // work buffers
  ErrState* d_err = nullptr;
  unsigned long long* d_counts = nullptr;
  double* d_scratch = nullptr;
  size_t scratch_bytes = 0;
  double* d_stk = nullptr;           // per-lane global ray-stack regions
  size_t stk_bytes = 0;
  double* d_stk2[LV_MAX_PARTS - 1] = {};   // the same for parts 1.. of a multi-stream level render
  size_t stk2_bytes[LV_MAX_PARTS - 1] = {};
  hipStream_t aux[LV_MAX_PARTS - 1] = {};  // bounce levels: the streams of parts 1.. (lv_streams)
  hipEvent_t lv_ev[LV_MAX_PARTS] = {};     // ... after the first batch's reset / after each part
  int* d_work = nullptr;             // ring of per-launch work counters (launches on different streams)
  unsigned work_seq = 0;
  int64_t opt_force_stack = 0;
  int64_t opt_bvh = 1;               // 0: ordered linear walk; 1: hierarchy from opt_bvh_min spheres; 2: always
  int64_t opt_bvh_sah = RTX_BVH_SAH;  // hierarchy splits: 1 binned SAH, 0 median (applies at the next upload)
  int64_t opt_bvh_min = 32;         // C2 (64 spheres): hierarchy 16.0 ms vs ordered walk 17.8 ms
  int64_t opt_sphere_src = -1;       // 0: LDS staging (measured faster), 1: scalar loads, 2: nodes LDS + leaves global,
                                     // 3: + exact records in LDS, 4: quantized leaves in LDS, -1 auto
  int64_t opt_postpone = -1;         // query_bvh postponing threshold in lanes (-1: auto by hierarchy size)
  int64_t opt_tile_order = -1;       // 1: expensive tiles first (k_tile_cost/k_tile_sort), 0: natural order, -1: auto
  int64_t opt_lds_stack = 0;         // ray-stack entries per lane in LDS (-1: as many as fit; 0 measured fastest)
  int64_t opt_engine = 1;            // 0: persistent lanes (per-lane LIFO ray tree), 1: bounce levels (default: faster, same bits)
  int64_t opt_lv_batch = 1 << 24;    // bounce levels: level-0 items (camera samples) per batch (C4: 2^23 -> 2^24
                                     // 358.0 -> 352.8 ms, half the level launches and their tails, r08k)
  int64_t opt_lv_stage_pct = 300;    // bounce levels: ray records per staging buffer, % of the batch items
  int64_t opt_lv_rec_pct = 1600;      // bounce levels: tree records of a batch (all levels), % of the batch items
  int64_t opt_lv_floor = 1 << 20;    // bounce levels: at least this many staging and 4x this many tree records
  int64_t opt_lv_split = 0;          // bounce levels: 1 = three phase launches per level (trace / shadow / shade)
  int64_t opt_lv_static = -1;        // bounce levels: % of a launch's chunks scheduled statically (-1 auto)
  int64_t opt_lv_compact = -1;       // bounce levels: 1 = park hits in an LDS ring and shade full waves, -1 auto (when it fits)
  int64_t opt_lv_grid_div = 1;       // bounce levels: persistent level grids = resident workgroups / this
  int64_t opt_lv_fin_grid = 0;       // bounce levels: tree reduction blocks per CU (grid-stride over tiles), 0 = one block per tile
  int64_t opt_lv_redo_blocks = 8;    // bounce levels: workgroups of the overflow re-render launch (0: all resident)
  int64_t opt_lv_streams = 2;        // bounce levels: P = the region's tiles in P interleaved parts on P streams at once
  int64_t opt_lv_ray_bytes = 0;      // bounce levels: staged ray record, 0 auto (80 B when every path fits 32 bits), 80, 96
  int64_t opt_lv_hl_cap = 0;         // bounce levels: deferred highlight-check list entries (0 auto)
  int64_t opt_exact_raises = 1;      // 1 (default): local_lights' shadow walks also check the acos raises of the covers they skip (§2.4)
                                     // (C2 +10 %, C4 +108 %, r09c; so not the default)
  int64_t opt_lv_sort = -1;          // bounce levels: 1 = levels visited bin by bin (direction octant, origin cell), 0 off,
                                     // -1 auto = on
  int64_t opt_lv_sort_from = 0;      // bounce levels: the first level binned; 0 auto: level 1 above 512 spheres (C4 354 ->
                                     // 307 ms), else the last level only (C2 4.60 -> 4.57 ms; all levels 4.65 -> 4.88, r10d/r10k)
  int64_t opt_lv_sort_bits = 0;      // bounce levels: 2^bits origin cells per axis (3 or 4); 0 auto: 4 above 512 spheres, else 3
  int64_t opt_lv_sort_copy = 0;      // bounce levels: 1 = binning copies the rays' records into bin order (r11i: C4 296 -> 342 ms, off)
  int64_t opt_lbuf = 1;              // bounce levels: 1 = shadow walks through the light buffer where it is staged (§3.18)
  int n_cus = 0;                     // compute units of the device (hipDeviceAttributeMultiprocessorCount)
  unsigned long long* d_lvstats = nullptr;   // rtx_level_stats of the last bounce-level render call
  int64_t last_sort_levels = 0;              // levels per batch the last bounce-level render binned (lv_sort_last)
  uint32_t* d_tile_rays = nullptr;   // rtx_tile_rays: rays per 8x8 tile of the last whole-frame level render
  size_t tile_rays_n = 0;
  int32_t* d_rowtiles = nullptr;     // rtx_render_tile_list_device: the tile list on the device
  std::vector<int32_t> rowtiles;     // ... and the list it holds
  size_t rowtiles_cap = 0;
  int64_t opt_kernel_events = 0;     // 1: HIP events around the ray-tree kernel launches (rtx_kernel_time)
  bool err_keys_rays = false;        // the device error keys of the last launch are ray indices (rtx_trace)
  // rtx_render_multi: this context's packed tiles; on the call's first context
  // also the gathered tiles + frame, and the RCCL clique over the call's devices
  double* d_multi = nullptr;
  size_t multi_bytes = 0;
  double* d_gather = nullptr;
  size_t gather_bytes = 0;
  std::vector<int> comm_devs;
  std::vector<ncclComm_t> comms;
  // rtx_kernel_time: event pairs around each ray-tree kernel launch of the last render call
  static constexpr int MAX_EV = 128;
  hipEvent_t ev[2 * MAX_EV] = {};
  int n_ev = 0;
};

static rtx_status fail(rtx_context* c, rtx_status s, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return s;
}

#define HIPCHK(c, expr)                                                                     \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(c, RTX_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

static void free_scene(rtx_context* c) {
  for (void* b : c->d_bufs) (void)hipFree(b);
  c->d_bufs.clear();
  c->have_scene = false;
}

#include "rtx_bvh_build.h"

extern "C" {

int32_t rtx_abi_version(void) { return RTX_ABI_VERSION; }

#ifndef RTX_SOURCE_SHA
#define RTX_SOURCE_SHA "unknown"
#endif
const char* rtx_build_id(void) { return RTX_SOURCE_SHA; }

const char* rtx_status_string(rtx_status s) {
  switch (s) {
    case RTX_OK: return "ok";
    case RTX_EZERO_VEC: return "zero vector detected";
    case RTX_ECOLOR_GT1: return "color greater than 1";
    case RTX_EDOMAIN: return "domain error";
    case RTX_EHIP: return "HIP error";
    case RTX_ERCCL: return "RCCL error";
    case RTX_EINVAL: return "invalid argument";
    case RTX_ENOMEM: return "out of memory";
    case RTX_ETYPE: return "TypeError: nil can't be coerced into Integer";
  }
  return "unknown";
}

const char* rtx_last_error(const rtx_context* c) { return c ? c->err.c_str() : "null context"; }

rtx_status rtx_context_create(int32_t device, rtx_context** out) {
  if (!out) return RTX_EINVAL;
  *out = nullptr;
  rtx_context* c = new rtx_context();
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(&c->d_err, sizeof(ErrState));
  if (e == hipSuccess) e = hipMalloc(&c->d_counts, sizeof(unsigned long long) * RTX_NCOUNT);
  if (e == hipSuccess) e = hipMalloc(&c->d_scene, sizeof(SceneDev));
  if (e == hipSuccess) e = hipMalloc(&c->d_cam, sizeof(CameraDev));
  if (e == hipSuccess) e = hipMalloc(&c->d_work, sizeof(int) * RTX_WORK_RING);
  if (e == hipSuccess) e = hipMemset(c->d_err, 0, sizeof(unsigned int) * 2);
  if (e == hipSuccess) e = hipMemset(((char*)c->d_err) + 8, 0xFF, sizeof(ErrState) - 8);
  if (e == hipSuccess) {           // keep render_region's stream-ordered buffers pooled between frames
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
      uint64_t keep = UINT64_MAX;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    fprintf(stderr, "rtx_context_create: %s\n", hipGetErrorString(e));
    delete c;
    return RTX_EHIP;
  }
  *out = c;
  return RTX_OK;
}

void rtx_context_destroy(rtx_context* c) {
  if (!c) return;
  hipSetDevice(c->device);
  free_scene(c);
  hipFree(c->d_err);
  hipFree(c->d_counts);
  hipFree(c->d_scene);
  hipFree(c->d_cam);
  hipFree(c->d_scratch);
  hipFree(c->d_stk);
  for (int j = 0; j < LV_MAX_PARTS - 1; j++) {
    hipFree(c->d_stk2[j]);
    if (c->aux[j]) (void)hipStreamDestroy(c->aux[j]);
  }
  for (hipEvent_t ev : c->lv_ev)
    if (ev) (void)hipEventDestroy(ev);
  hipFree(c->d_work);
  hipFree(c->d_lvstats);
  hipFree(c->d_tile_rays);
  hipFree(c->d_rowtiles);
  hipFree(c->d_multi);
  hipFree(c->d_gather);
  for (size_t k = 0; k < c->comms.size(); k++) {
    hipSetDevice(c->comm_devs[k]);
    ncclCommDestroy(c->comms[k]);
  }
  hipSetDevice(c->device);
  for (hipEvent_t ev : c->ev)
    if (ev) (void)hipEventDestroy(ev);
  delete c;
}

static bool levels_engine(const rtx_context* c);
static bool lv_paths32(const rtx_context* c);
static int sph_mode(const rtx_context* c);

static int lv_sort_from(const rtx_context* c, size_t n0);
static size_t lv_frame_items(const rtx_context* c);

rtx_status rtx_get_option(rtx_context* c, const char* key, int64_t* value) {
  if (!c || !key || !value) return RTX_EINVAL;
  if (!strcmp(key, "engine_effective")) {   // read-only: the engine the next render of this camera runs
    *value = c->have_cam && c->have_scene ? (levels_engine(c) ? 1 : 0) : c->opt_engine;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_sort_last")) {         // read-only: levels per batch the last bounce-level render binned
    *value = c->last_sort_levels;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_sort_effective")) {    // read-only: whether the next whole-frame bounce-level render bins its levels
    *value = c->have_cam && lv_sort_from(c, lv_frame_items(c)) > 0 ? 1 : 0;
    return RTX_OK;
  }
  if (!strcmp(key, "sph_mode_effective")) {   // read-only: the SphMode of the next bounce-level render's walks
    if (!c->have_scene) return fail(c, RTX_EINVAL, "sph_mode_effective: no scene uploaded");
    const int m = c->opt_sphere_src == -1
                      ? levels_auto_mode(c->scene, sph_mode(c), (int)c->opt_lv_compact, (int)c->opt_lv_split)
                      : sph_mode(c);
    *value = resolve_mode(c->scene, m);
    return RTX_OK;
  }
  if (!strcmp(key, "lv_ray_bytes_effective")) {   // read-only: the staged ray record of the next level render
    *value = c->opt_lv_ray_bytes == 96 || (c->have_cam && !lv_paths32(c)) ? 96 : 80;
    return RTX_OK;
  }
  const struct { const char* k; int64_t v; } tab[] = {
      {"engine", c->opt_engine},       {"force_stack", c->opt_force_stack}, {"bvh", c->opt_bvh},
      {"bvh_sah", c->opt_bvh_sah},     {"bvh_min", c->opt_bvh_min},         {"postpone", c->opt_postpone},
      {"lds_stack", c->opt_lds_stack}, {"tile_order", c->opt_tile_order},   {"sphere_src", c->opt_sphere_src},
      {"kernel_events", c->opt_kernel_events}, {"lv_batch", c->opt_lv_batch},
      {"lv_stage_pct", c->opt_lv_stage_pct}, {"lv_rec_pct", c->opt_lv_rec_pct}, {"lv_floor", c->opt_lv_floor},
      {"lv_split", c->opt_lv_split}, {"lv_static", c->opt_lv_static}, {"lv_compact", c->opt_lv_compact},
      {"lv_streams", c->opt_lv_streams}, {"lv_grid_div", c->opt_lv_grid_div},
      {"lv_redo_blocks", c->opt_lv_redo_blocks},
      {"lv_fin_grid", c->opt_lv_fin_grid}, {"lv_ray_bytes", c->opt_lv_ray_bytes},
      {"exact_raises", c->opt_exact_raises}, {"lv_hl_cap", c->opt_lv_hl_cap}, {"lv_sort", c->opt_lv_sort},
      {"lv_sort_from", c->opt_lv_sort_from}, {"lv_sort_bits", c->opt_lv_sort_bits}, {"lbuf", c->opt_lbuf},
      {"lv_sort_copy", c->opt_lv_sort_copy}};
  for (const auto& t : tab)
    if (!strcmp(key, t.k)) {
      *value = t.v;
      return RTX_OK;
    }
  return fail(c, RTX_EINVAL, "unknown option '%s'", key);
}

rtx_status rtx_set_option(rtx_context* c, const char* key, int64_t value) {
  if (!c || !key) return RTX_EINVAL;
  if (!strcmp(key, "engine")) {            // 0: persistent lanes (one ray tree per lane), 1: bounce levels
    if (value < 0 || value > 1) return fail(c, RTX_EINVAL, "engine must be 0 or 1");
    c->opt_engine = value;
    return RTX_OK;
  }
  if (!strcmp(key, "force_stack")) {
    c->opt_force_stack = value;
    return RTX_OK;
  }
  if (!strcmp(key, "bvh")) {               // 0: linear ordered walk; 1: auto (>= bvh_min spheres); 2: always
    if (value < 0 || value > 2) return fail(c, RTX_EINVAL, "bvh must be 0, 1 or 2");
    c->opt_bvh = value;
    return RTX_OK;
  }
  if (!strcmp(key, "bvh_sah")) {           // hierarchy splits: 1 binned SAH, 0 median (at the next upload)
    c->opt_bvh_sah = value != 0;
    return RTX_OK;
  }
  if (!strcmp(key, "bvh_min")) {           // sphere count from which bvh=1 uses the hierarchy
    if (value < 0) return fail(c, RTX_EINVAL, "bvh_min must be >= 0");
    c->opt_bvh_min = value;
    return RTX_OK;
  }
  if (!strcmp(key, "postpone")) {          // lanes below which hierarchy walks are postponed (-1 auto, 0 never)
    if (value < -1 || value > 64) return fail(c, RTX_EINVAL, "postpone must be in [-1, 64]");
    c->opt_postpone = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lds_stack")) {         // ray-stack entries per lane kept in LDS (-1: as many as fit)
    if (value < -1 || value > 64) return fail(c, RTX_EINVAL, "lds_stack must be in [-1, 64]");
    c->opt_lds_stack = value;
    return RTX_OK;
  }
  if (!strcmp(key, "tile_order")) {        // 1: expensive tiles first; 0: natural (row-major) tile order
    if (value < -1 || value > 1) return fail(c, RTX_EINVAL, "tile_order must be -1, 0 or 1");
    c->opt_tile_order = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_batch")) {          // bounce levels: camera samples per batch
    if (value < 1 || value > (1 << 28)) return fail(c, RTX_EINVAL, "lv_batch must be in [1, 2^28]");
    c->opt_lv_batch = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_stage_pct") || !strcmp(key, "lv_rec_pct")) {   // bounce-level buffer capacities
    if (value < 1 || value > 10000) return fail(c, RTX_EINVAL, "%s must be in [1, 10000]", key);
    (!strcmp(key, "lv_stage_pct") ? c->opt_lv_stage_pct : c->opt_lv_rec_pct) = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_floor")) {          // bounce levels: minimum buffer records (small frames, deep trees)
    if (value < 0 || value > (1 << 26)) return fail(c, RTX_EINVAL, "lv_floor must be in [0, 2^26]");
    c->opt_lv_floor = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_split")) {          // bounce levels: 0 one fused launch per level, 1 trace / shadow / shade
    if (value < 0 || value > 1) return fail(c, RTX_EINVAL, "lv_split must be 0 or 1");
    c->opt_lv_split = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_static")) {         // bounce levels: % of chunks scheduled statically, -1 auto
    if (value < -1 || value > 100) return fail(c, RTX_EINVAL, "lv_static must be in [-1, 100]");
    c->opt_lv_static = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_grid_div")) {       // bounce levels: level grids = resident workgroups / this
    if (value < 1 || value > 8) return fail(c, RTX_EINVAL, "lv_grid_div must be in [1, 8]");
    c->opt_lv_grid_div = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_fin_grid")) {       // bounce levels: reduction blocks per CU (grid-stride), 0 = one per tile
    if (value < 0 || value > 64) return fail(c, RTX_EINVAL, "lv_fin_grid must be in [0, 64]");
    c->opt_lv_fin_grid = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_hl_cap")) {         // bounce levels: deferred highlight-check list entries, 0 auto
    if (value < 0 || value > (1 << 26)) return fail(c, RTX_EINVAL, "lv_hl_cap must be in [0, 2^26]");
    c->opt_lv_hl_cap = value;
    return RTX_OK;
  }
  if (!strcmp(key, "exact_raises")) {      // every shadow walk also checks the skipped covers' acos raises
    if (value != 0 && value != 1) return fail(c, RTX_EINVAL, "exact_raises must be 0 or 1");
    c->opt_exact_raises = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_sort")) {           // bounce levels: bin each level's rays before its launch (same bits)
    if (value < -1 || value > 1) return fail(c, RTX_EINVAL, "lv_sort must be -1, 0 or 1");
    c->opt_lv_sort = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_sort_from")) {      // bounce levels: the first level binned (with lv_sort), 0 auto
    if (value < 0 || value > LV_MAXL) return fail(c, RTX_EINVAL, "lv_sort_from must be in [0, %d]", LV_MAXL);
    c->opt_lv_sort_from = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_sort_copy")) {      // bounce levels: binning moves the records into bin order (same bits)
    if (value < 0 || value > 1) return fail(c, RTX_EINVAL, "lv_sort_copy must be 0 or 1");
    c->opt_lv_sort_copy = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_sort_bits")) {      // bounce levels: 2^bits origin cells per axis of a ray bin, 0 auto
    if (value != 0 && value != 3 && value != 4) return fail(c, RTX_EINVAL, "lv_sort_bits must be 0, 3 or 4");
    c->opt_lv_sort_bits = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lbuf")) {              // bounce levels: shadow walks through the light buffer (same bits)
    if (value != 0 && value != 1) return fail(c, RTX_EINVAL, "lbuf must be 0 or 1");
    c->opt_lbuf = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_ray_bytes")) {      // bounce levels: staged ray record size (0 auto)
    if (value != 0 && value != 80 && value != 96) return fail(c, RTX_EINVAL, "lv_ray_bytes must be 0, 80 or 96");
    c->opt_lv_ray_bytes = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_redo_blocks")) {    // bounce levels: overflow re-render grid cap, 0 = all resident
    if (value < 0 || value > (1 << 20)) return fail(c, RTX_EINVAL, "lv_redo_blocks must be in [0, 2^20]");
    c->opt_lv_redo_blocks = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_streams")) {        // bounce levels: tiles in this many interleaved parts on as many streams
    if (value < 1 || value > LV_MAX_PARTS) return fail(c, RTX_EINVAL, "lv_streams must be in [1, %d]", LV_MAX_PARTS);
    c->opt_lv_streams = value;
    return RTX_OK;
  }
  if (!strcmp(key, "lv_compact")) {        // bounce levels: hit compaction in k_level, -1 auto, 2 compact ring
    if (value < -1 || value > 2) return fail(c, RTX_EINVAL, "lv_compact must be -1, 0, 1 or 2");
    c->opt_lv_compact = value;
    return RTX_OK;
  }
  if (!strcmp(key, "kernel_events")) {     // 1: HIP events around the ray-tree launches (rtx_kernel_time)
    c->opt_kernel_events = value != 0;
    return RTX_OK;
  }
  if (!strcmp(key, "sphere_src")) {        // 0: LDS staging; 1: scalar loads; 2: hierarchy nodes in LDS, leaves global;
                                           // 3: + exact records in LDS; 4: quantized leaf records in LDS; -1 auto
    if (value < -1 || value > 4) return fail(c, RTX_EINVAL, "sphere_src must be -1, 0, 1, 2, 3 or 4");
    c->opt_sphere_src = value;
    return RTX_OK;
  }
  return fail(c, RTX_EINVAL, "unknown option '%s'", key);
}

// ------------------------------------------------------------------ scene
static void put3(std::vector<double>& g, V3 v) {
  g.push_back(v.x);
  g.push_back(v.y);
  g.push_back(v.z);
}
static void set3(double* d, V3 v) {
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
}

// Plane record (plane.rb:21-23 reinit + get_uv's re-normalizations :82-83).
static void put_plane(std::vector<double>& g, V3 P, V3 F, V3 U, double uu, double vu, uint32_t& err) {
  V3 left = vnorm(vcross(F, U), err);
  put3(g, P);
  put3(g, F);
  put3(g, vnorm(left, err));
  put3(g, vnorm(U, err));
  g.push_back(uu);
  g.push_back(vu);
}

rtx_status rtx_scene_upload(rtx_context* c, const rtx_scene_desc* sd) {
  if (!c || !sd) return fail(c, RTX_EINVAL, "null argument");
  if (sd->n_objects < 0 || sd->n_lights < 0 || sd->n_textures < 0)
    return fail(c, RTX_EINVAL, "negative counts");
  if (sd->n_lights > 32) return fail(c, RTX_EINVAL, "at most 32 lights are supported");
  if ((sd->n_objects && !sd->objects) || (sd->n_lights && !sd->lights) || (sd->n_textures && !sd->textures))
    return fail(c, RTX_EINVAL, "null array with nonzero count");
  hipSetDevice(c->device);
  uint32_t err = 0;
  std::vector<Run> runs;
  std::vector<Material> mat(sd->n_objects);
  std::vector<Sphere64> sph64;
  std::vector<float> sph32;
  std::vector<int32_t> sph_obj;
  std::vector<double> planes, boxes;
  float sph_scale = 0.0f;
  for (int i = 0; i < sd->n_objects; i++) {
    const rtx_object_desc& o = sd->objects[i];
    Material& m = mat[i];
    memset(&m, 0, sizeof m);
    set3(m.diffuse, v3p(o.diffuse_rate));
    set3(m.ambient, v3p(o.ambient));
    set3(m.refl_att, v3p(o.reflective_attenuation));
    set3(m.refr_att, v3p(o.refractive_attenuation));
    m.rr = o.refractive_rate;
    m.has_rr = o.has_refractive_rate != 0;
    m.tex = o.texture_id;
    m.hs = o.texture_horizontal_scale;
    m.vs = o.texture_vertical_scale;
    m.type = o.type;
    if (o.texture_id >= sd->n_textures) return fail(c, RTX_EINVAL, "object %d: bad texture id", i);
    if (o.type != RTX_SPHERE && o.type != RTX_PLANE && o.type != RTX_BOX)
      return fail(c, RTX_EINVAL, "object %d: unknown type %d", i, o.type);
    if (runs.empty() || runs.back().type != o.type) {
      Run r;
      r.type = o.type;
      r.obj0 = i;
      r.count = 0;
      r.rec0 = o.type == RTX_SPHERE ? (int)sph64.size()
             : o.type == RTX_PLANE ? (int)(planes.size() / PLANE_GEO) : (int)(boxes.size() / BOX_GEO);
      runs.push_back(r);
    }
    runs.back().count++;
    if (o.type == RTX_SPHERE) {
      if (!o.has_refractive_rate) return fail(c, RTX_EINVAL, "object %d: sphere needs refractive_rate", i);
      m.rec = (int)sph64.size();
      sph_obj.push_back(i);
      Sphere64 sp;
      set3(sp.c, v3p(o.center));
      sp.r = o.radius;
      sph64.push_back(sp);
      // float32 pre-test record {cx, cy, cz, R^2}; scale = max(|C|_1 + R) (exact culls)
      sph32.push_back((float)o.center[0]);
      sph32.push_back((float)o.center[1]);
      sph32.push_back((float)o.center[2]);
      sph32.push_back((float)(o.radius * o.radius));
      const double sc = fabs(o.center[0]) + fabs(o.center[1]) + fabs(o.center[2]) + fabs(o.radius);
      const float scf = (float)(sc * (1.0 + 1e-6));
      if (scf > sph_scale) sph_scale = scf;
      m.u_off = o.texture_u_offset;
      m.v_off = o.texture_v_offset;
      if (o.texture_id >= 0) {                     // sphere.rb:18, 113-115
        const V3 north = v3p(o.north_pole_vec), gw = v3p(o.greenwich_vec);
        set3(m.gw_n, vnorm(gw, err));
        set3(m.east_n, vnorm(vcross(north, gw), err));
        set3(m.north_n, vnorm(north, err));
      }
    } else if (o.type == RTX_PLANE) {
      m.rec = (int)(planes.size() / PLANE_GEO);
      put_plane(planes, v3p(o.point), v3p(o.front), v3p(o.up), o.u_unit, o.v_unit, err);
    } else {                                         // box.rb:15-73
      m.rec = (int)(boxes.size() / BOX_GEO);
      m.tex = -1;                                    // loaded, never used for shading
      const V3 P = v3p(o.point), F = v3p(o.front), U = v3p(o.up);
      const double wf = o.width_front, wu = o.width_up, wl = o.width_left;
      const V3 left = vnorm(vcross(F, U), err);
      put_plane(boxes, vadd(P, vsc(vsc(U, wu), 0.5)), U, left, wf, wl, err);
      put_plane(boxes, vsub(P, vsc(vsc(U, wu), 0.5)), vneg(U), left, wf, wl, err);
      put_plane(boxes, vadd(P, vsc(vsc(F, wf), 0.5)), F, U, wl, wu, err);
      put_plane(boxes, vsub(P, vsc(vsc(F, wf), 0.5)), vneg(F), U, wl, wu, err);
      put_plane(boxes, vadd(P, vsc(vsc(left, wl), 0.5)), left, U, wf, wu, err);
      put_plane(boxes, vsub(P, vsc(vsc(left, wl), 0.5)), vneg(left), U, wf, wu, err);
    }
  }
  if (err) return fail(c, RTX_EZERO_VEC, "zero vector detected while building the scene");
  if (!std::isfinite(sph_scale)) return fail(c, RTX_EINVAL, "non-finite sphere coordinates");
  // bounding-ball hierarchy (before the padding records are appended)
  std::vector<BSph> bs(sph64.size());
  for (size_t k = 0; k < sph64.size(); k++) {
    for (int a = 0; a < 3; a++) bs[k].c[a] = sph64[k].c[a];
    bs[k].r = sph64[k].r;
    bs[k].rec = (int)k;
  }
  // SAH splits unless their tree would not fit the LDS of a hierarchy
  // workgroup while the median tree does (C4: the SAH tree spills to global
  // memory and renders 10 % slower; C2: SAH 1.3 % faster).
  const std::vector<BSph> bs_in = bs;
  auto bbp = std::make_unique<Bvh4Builder>(Bvh4Builder{bs, sph64, sph32, sph_obj});
  bbp->sah = c->opt_bvh_sah != 0;
  int32_t bvh_root = bs.empty() ? BVH_NONE : bbp->build(0, (int)bs.size(), 0);
  if (bbp->sah && !bs.empty() &&
      bvh_lds_bytes((int)bbp->nodes.size(), (int)bbp->slot_obj.size(), bbp->stack + 1) > bvh_lds_budget()) {
    bs = bs_in;
    auto med = std::make_unique<Bvh4Builder>(Bvh4Builder{bs, sph64, sph32, sph_obj});
    med->sah = false;
    const int32_t r = med->build(0, (int)bs.size(), 0);
    if (bvh_lds_bytes((int)med->nodes.size(), (int)med->slot_obj.size(), med->stack + 1) <= bvh_lds_budget()) {
      bbp = std::move(med);
      bvh_root = r;
    }
  }
  const Bvh4Builder& bb = *bbp;
  const QuantLeaves ql = quantize_leaves(bb, sph_scale);
  for (int k = 0; k < 16; k++) sph32.push_back(0.0f);   // 4 padding records: group loads stay in bounds
  std::vector<LightDev> lights(sd->n_lights);
  for (int i = 0; i < sd->n_lights; i++) {
    const rtx_light_desc& l = sd->lights[i];
    LightDev& d = lights[i];
    memset(&d, 0, sizeof d);
    set3(d.pos, v3p(l.position));
    set3(d.color, v3p(l.color));
    d.radius = l.radius;
    d.hl_rate = l.high_light_rate;
    d.hl_angle_rad = l.high_light_angle / 180.0 * 3.141592653589793;   // world.rb:91
    const double th = d.hl_angle_rad;
    if (!(th > 0)) {
      d.hl_mode = 2;                                 // acos(c) >= 0 can never be < th
    } else if (th < 1e-6 || th > 1.5) {
      d.hl_mode = 1;
    } else {
      const double ct = cos(th), lo = ct - 1e-7, hi = ct + 1e-7;
      d.hl_mode = (hi >= 1.0 || lo <= 0.0) ? 1 : 0;
      d.cos_lo2 = lo * lo;
      d.cos_hi2 = hi * hi;
    }
  }
  std::vector<TexDev> tex(sd->n_textures);
  std::vector<uint8_t> texels;
  for (int i = 0; i < sd->n_textures; i++) {
    const rtx_texture_desc& t = sd->textures[i];
    if (t.width <= 0 || t.height <= 0 || !t.rgb) return fail(c, RTX_EINVAL, "texture %d: empty", i);
    tex[i].w = t.width;
    tex[i].h = t.height;
    tex[i].off = (int64_t)texels.size();
    texels.insert(texels.end(), t.rgb, t.rgb + (size_t)t.width * t.height * 3);
  }
  free_scene(c);
  auto up = [&](const void* src, size_t bytes, void** dst) -> hipError_t {
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e != hipSuccess) return e;
    c->d_bufs.push_back(p);
    if (bytes) e = hipMemcpy(p, src, bytes, hipMemcpyHostToDevice);
    *dst = p;
    return e;
  };
  SceneDev& S = c->scene;
  memset(&S, 0, sizeof S);
  void* ptr;
  HIPCHK(c, up(runs.data(), runs.size() * sizeof(Run), &ptr));           S.runs = (const Run*)ptr;
  HIPCHK(c, up(sph64.data(), sph64.size() * sizeof(Sphere64), &ptr));    S.sph64 = (const Sphere64*)ptr;
  HIPCHK(c, up(sph32.data(), sph32.size() * sizeof(float), &ptr));       S.sph32 = (const float*)ptr;
  HIPCHK(c, up(planes.data(), planes.size() * sizeof(double), &ptr));    S.planes = (const double*)ptr;
  HIPCHK(c, up(boxes.data(), boxes.size() * sizeof(double), &ptr));      S.boxes = (const double*)ptr;
  HIPCHK(c, up(mat.data(), mat.size() * sizeof(Material), &ptr));        S.mat = (const Material*)ptr;
  HIPCHK(c, up(bb.nodes.data(), bb.nodes.size() * sizeof(Bvh4Node), &ptr)); S.bvh = (const Bvh4Node*)ptr;
  HIPCHK(c, up(bb.slot32.data(), bb.slot32.size() * sizeof(float), &ptr)); S.bvh_sph32 = (const float*)ptr;
  HIPCHK(c, up(bb.slot64.data(), bb.slot64.size() * sizeof(Sphere64), &ptr)); S.bvh_sph64 = (const Sphere64*)ptr;
  HIPCHK(c, up(ql.rec.data(), ql.rec.size() * sizeof(uint32_t), &ptr)); S.bvh_q = (const uint32_t*)ptr;
  HIPCHK(c, up(bb.slot_obj.data(), bb.slot_obj.size() * sizeof(int32_t), &ptr)); S.bvh_obj = (const int32_t*)ptr;
  HIPCHK(c, up(sph_obj.data(), sph_obj.size() * sizeof(int32_t), &ptr)); S.sph_obj = (const int32_t*)ptr;
  HIPCHK(c, up(lights.data(), lights.size() * sizeof(LightDev), &ptr));  S.light = (const LightDev*)ptr;
  HIPCHK(c, up(tex.data(), tex.size() * sizeof(TexDev), &ptr));          S.tex = (const TexDev*)ptr;
  HIPCHK(c, up(texels.data(), texels.size(), &ptr));                     S.texels = (const uint8_t*)ptr;
  S.n_obj = sd->n_objects;
  S.n_light = sd->n_lights;
  S.n_sphere = (int)sph64.size();
  S.n_plane = (int)(planes.size() / PLANE_GEO);
  S.n_box = (int)(boxes.size() / BOX_GEO);
  S.n_runs = (int)runs.size();
  S.n_nodes = (int)bb.nodes.size();
  S.n_slots = (int)bb.slot_obj.size();
  S.bvh_root = bvh_root;
  S.bvh_stack = bb.stack + 1;
  {                                                  // the light buffer (scenes whose records the level kernels stage)
    std::vector<double> lp(3 * (size_t)std::max(1, sd->n_lights));
    for (int i = 0; i < sd->n_lights; i++)
      for (int a = 0; a < 3; a++) lp[3 * i + a] = lights[i].pos[a];
    // small scenes: a table for LDS (<= 16 KB); larger ones: a finer one read
    // from global memory (<= 512 KB, L2-resident; C4: 160 cells per face side,
    // 251 ms per frame against 253 ms with 128 and 256 ms with 96, r10t)
#ifndef RTX_LBUF_GLOBAL_N
#define RTX_LBUF_GLOBAL_N 160
#endif
    std::vector<double> lrad(std::max(1, sd->n_lights), 0.0);
    for (int i = 0; i < sd->n_lights; i++) lrad[i] = lights[i].radius;
    LightBuffer lb;
    const bool small = sph64.size() <= 512;
    if (sd->n_lights > 0 && !sph64.empty())
      for (int n : small ? std::vector<int>{24, 16, 12, 8} : std::vector<int>{RTX_LBUF_GLOBAL_N, 128, 96, 64, 48, 32, 24}) {
        lb = build_light_buffer(bb, bvh_root, reinterpret_cast<const double(*)[3]>(lp.data()), sd->n_lights, n,
                                small ? LBUF_MAX_WORDS : LBUF_MAX_WORDS_GLOBAL, lrad.data());
        if (lb.n) break;
      }
    if (lb.n) {
      HIPCHK(c, up(lb.words.data(), lb.words.size() * sizeof(uint16_t), &ptr));
      S.lbuf = (const uint16_t*)ptr;
      S.lbuf_n = lb.n;
      S.lbuf_stride = lb.stride;
      // the raise buffer (exact_raises): its cells nest in the
      // light buffer's (small scenes: 12 per face side for C2's 24, gates staged
      // in LDS; larger: 160, as C4's light buffer), read from global memory; each light's floor
      // is 0.99 of the distance to the nearest object surface (targets of
      // World#local_lights lie on surfaces; nearer ones walk the hierarchy)
      std::vector<double> lfloor(std::max(1, sd->n_lights), 0.0);
      for (int li = 0; li < sd->n_lights; li++) {
        const double* L = lights[li].pos;
        double fl = HUGE_VAL;
        for (int k = 0; k < sd->n_objects; k++) {
          const rtx_object_desc& o = sd->objects[k];
          auto dist = [&](const double* p) {
            return std::sqrt((L[0] - p[0]) * (L[0] - p[0]) + (L[1] - p[1]) * (L[1] - p[1]) + (L[2] - p[2]) * (L[2] - p[2]));
          };
          auto norm = [](const double* v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); };
          if (o.type == RTX_SPHERE) {
            fl = std::min(fl, dist(o.center) - std::fabs(o.radius));
          } else if (o.type == RTX_PLANE) {
            const double fn = norm(o.front);
            fl = std::min(fl, std::fabs((L[0] - o.point[0]) * o.front[0] + (L[1] - o.point[1]) * o.front[1] +
                                        (L[2] - o.point[2]) * o.front[2]) / fn);
          } else {                                    // a box: within this ball of its point (box.rb:15-73)
            const double rb = 0.5 * (std::fabs(o.width_front) * (1.0 + norm(o.front)) +
                                     std::fabs(o.width_up) * (1.0 + norm(o.up)) + 2.0 * std::fabs(o.width_left));
            fl = std::min(fl, dist(o.point) - rb);
          }
        }
        lfloor[li] = std::isfinite(fl) ? std::max(0.0, 0.99 * fl) : 0.0;
      }
      // (the finest nesting resolution up to 12 / 160 cells per face side whose lists fit at the
      // lights' own floors; only if none does, a coarse one with the floors raised until it fits)
#ifndef RTX_RBUF_GLOBAL_N
#define RTX_RBUF_GLOBAL_N 160      // C4: 294.5 / 285.6 / 283.7 ms per frame at 40 / 80 / 160 (r11y; r11ab: 285.4 / 283.2 at 80 / 160; 77 MB)
#endif
      RaiseBuffer rb;
      const int want = small ? 12 : RTX_RBUF_GLOBAL_N;
      const size_t rb_max = small ? RBUF_MAX_WORDS : RBUF_MAX_WORDS_GLOBAL;
      int coarse = 0;
      for (int nc = std::min(want, lb.n); nc >= 1 && !rb.n; nc--) {
        if (lb.n % nc) continue;
        coarse = nc;
        if (nc < 4) break;
        rb = build_raise_buffer(bb, bvh_root, reinterpret_cast<const double(*)[3]>(lp.data()), lrad.data(),
                                lfloor.data(), sd->n_lights, nc, rb_max, nullptr, !small, 0);
      }
      if (!rb.n && coarse)
        rb = build_raise_buffer(bb, bvh_root, reinterpret_cast<const double(*)[3]>(lp.data()), lrad.data(),
                                lfloor.data(), sd->n_lights, coarse, rb_max, nullptr, !small);
      if (rb.n) {
        // per light: floor^2 (rounded up) and log2 floor^2 (float bits, 2 words each), 4 words of
        // padding, a gate word per cell (rtx_device.h raise_qa)
        const std::vector<uint16_t> g = raise_gates(rb, sd->n_lights);
        const int cells = 6 * rb.n * rb.n, gs = (8 + cells + 7) & ~7;
        std::vector<uint16_t> gw((size_t)gs * sd->n_lights, 0);
        for (int li = 0; li < sd->n_lights; li++) {
          const float hw[2] = {raise_floor2(rb, li), raise_lf2(rb, li)};
          memcpy(&gw[(size_t)gs * li], hw, 8);
          std::copy(g.begin() + (size_t)cells * li, g.begin() + (size_t)cells * (li + 1), gw.begin() + (size_t)gs * li + 8);
        }
        HIPCHK(c, up(rb.words.data(), rb.words.size() * sizeof(uint32_t), &ptr));
        S.rbuf = (const uint32_t*)ptr;
        HIPCHK(c, up(gw.data(), gw.size() * sizeof(uint16_t), &ptr));
        S.rgate = (const uint16_t*)ptr;
        for (int li = 0; li < sd->n_lights; li++) {   // (raise_qa reads them with the light's data)
          lights[li].raise_f2 = raise_floor2(rb, li);
          lights[li].raise_lf2 = raise_lf2(rb, li);
        }
        HIPCHK(c, hipMemcpy((void*)S.light, lights.data(), lights.size() * sizeof(LightDev), hipMemcpyHostToDevice));
        S.rbuf_n = rb.n;
        S.rbuf_stride = rb.stride;
        S.rgate_stride = gs;
        S.rbuf_inv_m = (float)rb.n / (float)lb.n;   // (exact enough: (i + 0.5) m' stays 0.5 / m from an integer)
        S.rbuf_sphere = small ? 0 : 1;              // larger scenes: per-sphere entries (fewer band tests per walk)
      }
    }
  }
  S.max_distance = sd->max_distance;
  S.sse = sd->soft_shadow_exponent;
  S.sph_scale = sph_scale;
  S.sse_is_two = sd->soft_shadow_exponent == 2.0;     // glibc pow(x, 2.0) == x*x
  for (int a = 0; a < 3; a++) S.q_org[a] = ql.org[a], S.q_step[a] = ql.step[a];
  S.q_rstep = ql.rstep;
  S.q_ok = ql.ok && S.n_nodes <= 32767 && (int64_t)S.n_slots <= 32767;   // references fit int16 stack entries
  // a decoded center lies within max_err of the true one; a decoded radius within max_err + 2 rstep of R
  // (ceil to the step, at most one more step: quantize_leaves)
  S.q_err = (float)((ql.max_err + 2.0 * (double)ql.rstep) * 1.01 + 1e-9 * ql.max_r);
  {                                                  // the spheres' box, float32, rounded outwards
    double mn[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, mx[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
    for (const Sphere64& sp : sph64)
      for (int a = 0; a < 3; a++) {
        mn[a] = std::min(mn[a], sp.c[a] - fabs(sp.r));
        mx[a] = std::max(mx[a], sp.c[a] + fabs(sp.r));
      }
    for (int a = 0; a < 3; a++) {
      if (!(mn[a] <= mx[a])) {                       // no spheres: an empty box far away
        S.root_c[a] = 3e38f;
        S.root_h[a] = 0.0f;
        continue;
      }
      const float cf = (float)(0.5 * (mn[a] + mx[a]));
      const double h = std::max(mx[a] - (double)cf, (double)cf - mn[a]);
      S.root_c[a] = cf;
      S.root_h[a] = f32_up(h * (1.0 + 1e-9) + 1e-30);
    }
  }
  HIPCHK(c, hipMemcpy(c->d_scene, &S, sizeof S, hipMemcpyHostToDevice));
  c->have_scene = true;
  return RTX_OK;
}

rtx_status rtx_camera_set(rtx_context* c, const rtx_camera_desc* d) {
  if (!c || !d) return fail(c, RTX_EINVAL, "null argument");
  if (d->width <= 0 || d->height <= 0) return fail(c, RTX_EINVAL, "width/height must be positive");
  if (d->pre_sample_times < 1 || d->pre_sample_times > 16)
    return fail(c, RTX_EINVAL, "pre_sample_times must be in [1, 16]");
  if (d->max_sample_times < 0) return fail(c, RTX_EINVAL, "max_sample_times must be >= 0");
  {
    // device work items are 32-bit: every (8x8-padded) pixel x sample of the frame must fit
    const size_t padded = (size_t)((d->width + 7) / 8) * (size_t)((d->height + 7) / 8) * 64;
    const size_t ms = (size_t)std::max(d->pre_sample_times, d->max_sample_times);
    if (padded * ms > (size_t)INT32_MAX)
      return fail(c, RTX_EINVAL, "%dx%d pixels x %zu samples exceed 2^31 work items", d->width, d->height, ms);
  }
  if (d->trace_depth < 0 || d->trace_depth > 1000) return fail(c, RTX_EINVAL, "bad trace_depth");
  if (d->monte_carlo_diffusion_times < 1) return fail(c, RTX_EINVAL, "monte_carlo_diffusion_times must be >= 1");
  uint32_t err = 0;
  CameraDev& k = c->cam;
  memset(&k, 0, sizeof k);
  const V3 pos = v3p(d->position), up = v3p(d->up), front = v3p(d->front);
  const V3 left = vnorm(vcross(up, front), err);                       // camera.rb:130
  set3(k.pos, pos);
  set3(k.left, left);
  set3(k.left_n, vnorm(left, err));                                    // :136
  set3(k.up_n, vnorm(up, err));                                        // :134,136
  set3(k.front, front);
  set3(k.retina_center, vsub(pos, vsc(vnorm(front, err), d->image_distance)));   // :131
  const double od = d->focal_distance * d->image_distance / (d->image_distance - d->focal_distance);  // :139
  set3(k.pofp, vadd(pos, vsc(vnorm(front, err), od)));                // :142
  k.retina_width = d->retina_width;
  k.retina_height = d->retina_height;
  k.aperture_radius = d->aperture_radius;
  k.variant_threshold = d->variant_threshold;
  k.width = d->width;
  k.height = d->height;
  k.pre = d->pre_sample_times;
  k.max_samples = d->max_sample_times;
  k.depth = d->trace_depth;
  k.pt = d->monte_carlo_diffusion_times;
  if (err) return fail(c, RTX_EZERO_VEC, "zero vector detected while building the camera");
  HIPCHK(c, hipMemcpy(c->d_cam, &k, sizeof k, hipMemcpyHostToDevice));
  c->have_cam = true;
  return RTX_OK;
}

// ------------------------------------------------------------------ render
static int required_stack(const rtx_context* c) {
  // LIFO depth-first walk: a node at depth d >= 2 pushes <= 2 + pt children.
  const long need = 1 + (long)(c->cam.depth > 1 ? c->cam.depth - 1 : 0) * (1 + c->cam.pt);
  if (c->opt_force_stack) return stack_bucket((int)c->opt_force_stack);
  return need > 64 ? -1 : stack_bucket((int)need);
}

// Sphere walk of the next launch (SphMode); the launchers fall back to scalar
// loads when the records exceed the LDS budget.
static int sph_mode(const rtx_context* c) {
  const bool bvh = c->opt_bvh == 2 || (c->opt_bvh == 1 && c->scene.n_sphere >= c->opt_bvh_min);
  if (bvh && c->scene.bvh_root != BVH_NONE)
    return c->opt_sphere_src == 4   ? SPH_BVH_QLDS
           : c->opt_sphere_src == 3 ? SPH_BVH_LDSX
           : c->opt_sphere_src == 2 ? SPH_BVH_MIX
           : c->opt_sphere_src == 1 ? SPH_BVH_GLOBAL
                                    : SPH_BVH_LDS;
  return c->opt_sphere_src == 1 ? SPH_LIN_SCALAR : SPH_LIN_LDS;
}

// Global per-lane regions (ray-stack entries beyond LDS) for every lane a persistent launch can keep resident (512 per CU at
// 256 VGPRs; room for 1024).
static rtx_status ensure_stack(rtx_context* c, KParams& p, int maxs) {
  int cus = 0;
  HIPCHK(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
  const size_t lanes = (size_t)(cus > 0 ? cus : 1) * 1024;
  const size_t per_lane = (size_t)maxs * 12 * sizeof(double);
  const size_t bytes = lanes * per_lane;
  if (bytes > c->stk_bytes) {
    hipFree(c->d_stk);
    c->d_stk = nullptr;
    c->stk_bytes = 0;
    HIPCHK(c, hipMalloc(&c->d_stk, bytes));
    c->stk_bytes = bytes;
  }
  p.stk_glb = c->d_stk;
  p.stk_glb_lanes = (int32_t)(c->stk_bytes / per_lane);
  return RTX_OK;
}

static rtx_status prep(rtx_context* c, KParams& p, uint64_t seed) {
  // The context's device first: every allocation below and in ensure_stack /
  // ensure_scratch, and every launch, must land on it whatever device the
  // calling thread had selected.
  HIPCHK(c, hipSetDevice(c->device));
  if (!c->have_scene) return fail(c, RTX_EINVAL, "no scene uploaded");
  if (!c->have_cam) return fail(c, RTX_EINVAL, "no camera set");
  memset(&p, 0, sizeof p);
  p.scene = c->scene;
  p.cam = c->d_cam;
  p.seed = seed;
  p.err = c->d_err;
  p.counts = c->d_counts;
  p.work = c->d_work + (c->work_seq++ % RTX_WORK_RING);
  p.stk_slots_max = c->opt_lds_stack < 0 ? 64 : (int32_t)c->opt_lds_stack;
  p.pre = c->cam.pre;
  p.max_samples = c->cam.max_samples;
  // Postponing long walks pays when walks are long (C4, 341 nodes: 550 -> 507 ms)
  // and costs when they are short (C2, a few nodes: 9.0 -> 9.3 ms).
  p.exact_raises = (int32_t)c->opt_exact_raises;
  p.postpone = c->opt_postpone >= 0 ? (int32_t)c->opt_postpone : (c->scene.n_nodes >= RTX_POSTPONE_NODES ? 16 : 0);
  return RTX_OK;
}

// launch_render with its per-launch sample records and extra-sample list,
// allocated stream-ordered (the device's default pool keeps the memory, so
// after the first frame this costs no hipMalloc) and freed after the launch,
// so launches of one context on different streams never share them.
static size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

// The bounce-level engine can take this camera: its levels and child slots.
// 80-B ray records when a ray's path id fits 32 bits at every level: path
// < (pt + 3)^trace_depth (the path ids of rtx_device.h emit / lv_finish).
// lv_ray_bytes 80 asked for a camera whose paths do not fit is refused, not
// truncated.
static bool lv_paths32(const rtx_context* c) {
  uint64_t v = 1;
  for (int l = 0; l < c->cam.depth; l++) {
    v *= (uint64_t)c->cam.pt + 3;
    if (v > (1ull << 32)) return false;
  }
  return true;
}

// ray binning (option lv_sort) for the fused level launches
// The first level binned (0: none) and the bins' resolution.  Large scenes
// bin every level >= 1 (C4 354 -> 307 ms); small ones only the last, where the
// rays are most incoherent and most numerous (C2: binning every level costs
// more than it gains, r10d; the last level alone gains 0.5 %, r10k).
// n0: the camera samples of a batch (the last level of a small scene is binned
// only from 2^22 of them: a 1/8 or 1/4 share of the C2 frame lost 4-5 % to the
// binning passes' fixed cost, half of it neither gained nor lost, r10p).
static int lv_sort_from(const rtx_context* c, size_t n0) {
  const bool split = c->opt_lv_split != 0 && c->scene.n_light <= LV_SPLIT_MAX_LIGHTS;
  if (c->opt_lv_sort == 0 || split) return 0;
  const bool large = c->scene.n_sphere > 512;
  if (c->opt_lv_sort == -1 && c->opt_lv_sort_from == 0 && !large && n0 < ((size_t)1 << 22)) return 0;
  const int from = c->opt_lv_sort_from > 0 ? (int)c->opt_lv_sort_from : large ? 1 : c->cam.depth - 1;
  return from >= 1 && from < c->cam.depth ? from : 0;
}
// the camera samples of a whole-frame render's batch (lv_sort_effective): the
// arithmetic of render_levels' n0, with the frame's tiles split in lv_streams
// parts (the default two parts give C2 4,147,200 samples per batch,
// below the 2^22 of lv_sort_from, so a single C2 frame bins nothing; the
// bench's frames in flight render one part of 8.3 M)
static size_t lv_frame_items(const rtx_context* c) {
  const int64_t tiles = (int64_t)((c->cam.width + 7) / 8) * ((c->cam.height + 7) / 8);
  const int64_t per_tile = 64 * (int64_t)std::max(1, c->cam.pre);
  const int64_t parts = std::max<int64_t>(1, std::min<int64_t>(c->opt_lv_streams, tiles));
  const int64_t batch_tiles = std::max<int64_t>(1, std::min<int64_t>(c->opt_lv_batch / per_tile, (tiles + parts - 1) / parts));
  return std::max<size_t>((size_t)(batch_tiles * per_tile), (size_t)std::max(0, c->cam.max_samples - c->cam.pre));
}
static int lv_sort_bits(const rtx_context* c) {
  return c->opt_lv_sort_bits ? (int)c->opt_lv_sort_bits : c->scene.n_sphere > 512 ? 4 : 3;
}

static bool levels_engine(const rtx_context* c) {
  return c->opt_engine == 1 && c->cam.depth <= LV_MAXL && c->cam.pt + 2 <= 16 && c->scene.n_light <= 255;
}

// render_region for the bounce-level engine: batches of
// 8x8 tiles, one launch per tree level, the trees reduced by k_tree_finalize.
// Buffers for one batch, stream-ordered from the device pool like the lanes
// engine's: staging (2 x lv_stage_pct % of the batch items x 96 B), tree
// records (lv_rec_pct % x 32 B with one light), the re-render list.
static rtx_status render_levels(rtx_context* c, KParams& p, int maxs, hipStream_t stream) {
  const size_t npx = (size_t)p.nx * p.nrows;
  const int tiles = ((p.nx + 7) / 8) * ((p.nrows + 7) / 8);
  const int per_tile = 64 * p.pre;
  const int parts = (int)std::max<int64_t>(1, std::min<int64_t>(c->opt_lv_streams, tiles));   // lv_streams (below)
  const int batch_tiles =
      (int)std::max<int64_t>(1, std::min<int64_t>(c->opt_lv_batch / per_tile, (tiles + parts - 1) / parts));
  // level-0 items of one batch: pass 0 (tiles) or pass 1 (>= one pixel's extra samples)
  const size_t n0 = std::max((size_t)batch_tiles * per_tile, (size_t)std::max(0, p.max_samples - p.pre));
  const size_t fl = (size_t)c->opt_lv_floor;
  const size_t want = std::max<size_t>(std::max<size_t>(64, fl), n0 * (size_t)c->opt_lv_stage_pct / 100);
  const size_t lcap = std::max<size_t>(std::max(n0, 4 * fl), n0 * (size_t)c->opt_lv_rec_pct / 100);
  // queues of levels >= 1: LV_SLICES slices of 2^k slots (k rounded up)
  int slog2 = 0;
  while (((size_t)LV_SLICES << slog2) < want) slog2++;
  const size_t scap = (size_t)LV_SLICES << slog2;
  if (scap > UINT32_MAX / 2 || lcap > UINT32_MAX / 2)
    return fail(c, RTX_EINVAL, "bounce-level buffers exceed 2^31 records: lower lv_batch");
  const bool path32 = lv_paths32(c);
  if (c->opt_lv_ray_bytes == 80 && !path32)
    return fail(c, RTX_EINVAL, "lv_ray_bytes 80: this camera's ray paths need 64 bits ((pt + 3)^trace_depth > 2^32)");
  const int rec_bytes = levels_rec_bytes(c->scene.n_light);
  // deferred highlight checks (k_hl_raise): room for 1/256 of the batch's tree
  // records (rays; C2 fires on ~0.1 % of them); a ray that finds the list full
  // has its sample re-rendered by the lanes engine (option lv_hl_cap: the size)
  const size_t hlcap = c->opt_lv_hl_cap > 0 ? (size_t)c->opt_lv_hl_cap : std::max<size_t>(4096, lcap / 256);
  const size_t sz_hlq = al256(hlcap * 64);
  const size_t sz_ctl = al256(sizeof(LevelCtl)), sz_redo = al256(n0 * 4), sz_smp = al256(n0 * 32),
               sz_stage = al256(scap * RAY_BYTES), sz_rec = al256(lcap * (size_t)rec_bytes),
               sz_extra = al256((npx + 64) * 4);
  // split phases: the hit queue of a level (at most its rays) and its shadow results
  const bool split = c->opt_lv_split != 0 && c->scene.n_light <= LV_SPLIT_MAX_LIGHTS;
  int hlog2 = 0;
  while (((size_t)LV_SLICES << hlog2) < std::max(n0, scap)) hlog2++;
  const size_t hcap = (size_t)LV_SLICES << hlog2;
  const size_t sz_hit = split ? al256(hcap * LV_HIT_BYTES) : 0,
               sz_area = split ? al256(hcap * (size_t)std::max(1, c->scene.n_light) * 16) : 0;
  // ray binning (lv_sort, fused levels only): a bin per staged slot, the
  // level's bin list, the bin counts and cursors
  const int sort_from = lv_sort_from(c, n0);
  const bool sort = sort_from > 0;
  c->last_sort_levels = sort ? std::max(0, c->cam.depth - sort_from) : 0;   // (read-only option lv_sort_last)
  const size_t sz_key = sort ? al256(scap * 2) : 0, sz_perm = sort ? al256(scap * 8) : 0,
               sz_bins = sort ? al256((size_t)LV_BINS * 8) : 0;
  // One buffer set per part: with lv_streams = P the region's tiles are
  // rendered in P interleaved parts at once, parts 1.. on the context's aux
  // streams (one part's level tails, launch gaps and reductions overlap the
  // others' levels).  The extra-sample list and the statistics are shared
  // (appended / added atomically); each part has its own level buffers, its
  // own lanes-engine work counter and ray stacks for its overflow re-render.
  // (lv_sort_copy: the binned level's records in bin order, a third staging buffer)
  const bool sort_copy = sort && c->opt_lv_sort_copy == 1;
  const size_t sz_sorted = sort_copy ? sz_stage : 0;
  const size_t set = sz_ctl + 2 * sz_redo + sz_smp + 2 * sz_stage + sz_rec + sz_hit + sz_area + sz_hlq + sz_key +
                     sz_perm + sz_bins + sz_sorted;
  const size_t total = parts * set + sz_extra;
  if (!c->d_lvstats) HIPCHK(c, hipMalloc(&c->d_lvstats, sizeof(unsigned long long) * (LV_MAXL + 3)));
  char* buf = nullptr;
  HIPCHK(c, hipMallocAsync((void**)&buf, total, stream));
  auto carve = [&](KParams& k, char* q) {
    k.lv_ctl = (LevelCtl*)q;                  q += sz_ctl;
    k.lv_redo_of = (int32_t*)q;               q += sz_redo;
    k.lv_redo_list = (int32_t*)q;             q += sz_redo;
    k.lv_redo_smp = (double*)q;               q += sz_smp;
    k.lv_stage[0] = (double*)q;               q += sz_stage;
    k.lv_stage[1] = (double*)q;               q += sz_stage;
    k.lv_rec = q;                             q += sz_rec;
    k.lv_hit = split ? (double*)q : nullptr;  q += sz_hit;
    k.lv_area = split ? (double*)q : nullptr; q += sz_area;
    k.lv_hlq = (double*)q;                    q += sz_hlq;
    k.lv_hlq_cap = (uint32_t)hlcap;
    k.lv_key = sort ? (uint16_t*)q : nullptr;      q += sz_key;
    k.lv_perm = sort ? (uint2*)q : nullptr;        q += sz_perm;
    k.lv_bins = sort ? (uint32_t*)q : nullptr;     q += sz_bins;
    k.lv_sorted = sort_copy ? (double*)q : nullptr; q += sz_sorted;
    k.lv_sort = sort_from;
    k.lv_cell_bits = lv_sort_bits(c);
    k.lv_lbuf = (int32_t)c->opt_lbuf;
  };
  carve(p, buf);
  p.lv_split = split ? 1 : 0;
  p.lv_compact = (int32_t)c->opt_lv_compact;
  p.lv_grid_div = (int32_t)c->opt_lv_grid_div;
  p.lv_redo_blocks = (int32_t)c->opt_lv_redo_blocks;
  p.lv_fin_tiles = (int32_t)c->opt_lv_fin_grid;   // (blocks per CU here; the launcher sets the tile count)
  // Static chunks cost no atomics; dynamic claims balance rays of very
  // different cost.  Auto: all static while the sphere records fit one walk
  // workgroup's LDS with room to spare (C2: 5.35 vs 5.9 ms at 50 %), half
  // static for large hierarchies (C4: 437 vs 518 ms all static).
  p.lv_static_pct = c->opt_lv_static >= 0 ? (int32_t)c->opt_lv_static : (c->scene.n_sphere <= 512 ? 100 : 50);
  p.extra_count = (int32_t*)(buf + parts * set);
  p.extra_list = p.extra_count + 64;
  p.lv_scap = (uint32_t)scap;
  p.lv_slice_log2 = slog2;
  p.lv_hslice_log2 = hlog2;
  p.lv_lcap = (uint32_t)lcap;
  p.lv_rec_bytes = rec_bytes;
  p.lv_ray_dbl = (c->opt_lv_ray_bytes == 96 || !path32) ? 12 : 10;
  p.lv_last_level = c->cam.depth >= 1 ? c->cam.depth - 1 : -1;
  p.lv_acc = c->d_lvstats;
  p.samples = nullptr;
  LvAux aux{};
  if (parts > 1) {
    aux.parts = parts;
    for (hipEvent_t& ev : c->lv_ev)
      if (!ev) HIPCHK(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    aux.ev_first = c->lv_ev[0];
    const size_t stk = (size_t)p.stk_glb_lanes * (size_t)maxs * 12 * sizeof(double);
    for (int j = 0; j < parts - 1; j++) {
      if (!c->aux[j]) HIPCHK(c, hipStreamCreateWithFlags(&c->aux[j], hipStreamNonBlocking));
      if (stk > c->stk2_bytes[j]) {
        hipFree(c->d_stk2[j]);
        c->d_stk2[j] = nullptr;
        c->stk2_bytes[j] = 0;
        HIPCHK(c, hipMalloc(&c->d_stk2[j], stk));
        c->stk2_bytes[j] = stk;
      }
      KParams& q = aux.pb[j];
      q = p;
      carve(q, buf + (size_t)(j + 1) * set);
      q.work = reinterpret_cast<int*>(&q.lv_ctl->pad[0]);   // zeroed by its part's k_level_begin
      q.stk_glb = c->d_stk2[j];
      aux.s2[j] = c->aux[j];
      aux.ev_done[j] = c->lv_ev[j + 1];
    }
  }
  KernelEvents kev{c->ev, 0, rtx_context::MAX_EV};
  if (c->opt_kernel_events && !c->ev[0])
    for (int k = 0; k < 2 * rtx_context::MAX_EV; k++) HIPCHK(c, hipEventCreate(&c->ev[k]));
  // sphere_src auto: C4-sized hierarchies keep their nodes and 16-bit leaf
  // records in LDS next to the hit rings (SPH_BVH_QLDS; before round 4 the
  // leaves came from global memory, SPH_BVH_MIX, r05b: C4 410 -> 386 ms)
  const int mode = c->opt_sphere_src == -1 ? levels_auto_mode(c->scene, sph_mode(c), (int)c->opt_lv_compact,
                                                              (int)c->opt_lv_split)
                                           : sph_mode(c);
  const hipError_t e = launch_levels(p, mode, maxs, std::max(1, c->cam.depth), batch_tiles, stream,
                                     c->opt_kernel_events ? &kev : nullptr, parts > 1 ? &aux : nullptr);
  if (c->opt_kernel_events) c->n_ev = kev.n;
  const hipError_t f = hipFreeAsync(buf, stream);
  HIPCHK(c, e);
  HIPCHK(c, f);
  return RTX_OK;
}

static rtx_status render_region(rtx_context* c, KParams& p, bool count, int maxs, hipStream_t stream) {
  const size_t npx = (size_t)p.nx * p.nrows;
  if (npx == 0) return RTX_OK;
  if (!count && levels_engine(c)) {
    const size_t padded = (size_t)((p.nx + 7) / 8) * ((p.nrows + 7) / 8) * 64;
    if (padded * (size_t)std::max(p.pre, p.max_samples) > (size_t)INT32_MAX)
      return fail(c, RTX_EINVAL, "%zu pixels x samples exceed the 2^31 work items of one launch", npx);
    return render_levels(c, p, maxs, stream);
  }
  const size_t ms = (size_t)std::max(p.pre, p.max_samples);
  // Work items are 32-bit on the device: (8x8-padded pixels) x samples must fit.
  const size_t padded = (size_t)((p.nx + 7) / 8) * ((p.nrows + 7) / 8) * 64;
  if (padded * ms > (size_t)INT32_MAX)
    return fail(c, RTX_EINVAL, "%zu pixels x %zu samples exceed the 2^31 work items of one launch", npx, ms);
  const size_t smp_bytes = npx * ms * 4 * sizeof(double);
  void* buf = nullptr;
  const size_t tiles = (size_t)((p.nx + 7) / 8) * ((p.nrows + 7) / 8);
  HIPCHK(c, hipMallocAsync(&buf, smp_bytes + (npx + 64 + 2 * tiles) * sizeof(int32_t), stream));
  p.samples = (double*)buf;
  p.extra_count = (int32_t*)((char*)buf + smp_bytes);
  p.extra_list = p.extra_count + 64;
  p.tile_cls = p.extra_list + npx;
  // Auto: the probe is an ordered linear walk, cheap for a few hundred spheres
  // (C2: 9.2 -> 8.9 ms); on C4 (4,096 spheres) it costs 2.2 ms and the order
  // gains nothing (the frame is 500 ms of evenly expensive tiles).
  const bool order = c->opt_tile_order > 0 || (c->opt_tile_order < 0 && c->scene.n_sphere <= RTX_TILE_ORDER_SPHERES);
  p.tile_order = order ? p.tile_cls + tiles : nullptr;
  KernelEvents kev{c->ev, 0, rtx_context::MAX_EV};
  if (c->opt_kernel_events && !count && !c->ev[0]) {
    for (int k = 0; k < 2 * rtx_context::MAX_EV; k++) HIPCHK(c, hipEventCreate(&c->ev[k]));
  }
  const hipError_t e = launch_render(p, sph_mode(c), count, maxs, stream,
                                     c->opt_kernel_events && !count ? &kev : nullptr);
  if (c->opt_kernel_events && !count) c->n_ev = kev.n;
  const hipError_t f = hipFreeAsync(buf, stream);
  HIPCHK(c, e);
  HIPCHK(c, f);
  return RTX_OK;
}

rtx_status rtx_render_device(rtx_context* c, int32_t x0, int32_t y0, int32_t x1, int32_t y1, uint64_t seed,
                             double* d_out, size_t row_stride, void* stream) {
  if (!c) return RTX_EINVAL;
  KParams p;
  rtx_status s = prep(c, p, seed);
  if (s) return s;
  if (x0 < 0 || y0 < 0 || x1 > c->cam.width || y1 > c->cam.height || x0 > x1 || y0 > y1)
    return fail(c, RTX_EINVAL, "region [%d,%d)x[%d,%d) outside the %dx%d image", x0, x1, y0, y1,
                c->cam.width, c->cam.height);
  if (row_stride < (size_t)(x1 - x0) * 3) return fail(c, RTX_EINVAL, "row_stride too small");
  const int maxs = required_stack(c);
  if (maxs < 0) return fail(c, RTX_EINVAL, "trace_depth x monte_carlo_diffusion_times too large");
  if ((s = ensure_stack(c, p, maxs))) return s;
  hipSetDevice(c->device);
  p.x0 = x0;
  p.nx = x1 - x0;
  p.y0 = y0;
  p.nrows = y1 - y0;
  p.out = d_out;
  p.stride = row_stride;
  if (x0 == 0 && y0 == 0 && x1 == c->cam.width && y1 == c->cam.height && levels_engine(c)) {
    // the whole frame: the reduction records rays per 8x8 tile (rtx_tile_rays)
    const size_t nt = (size_t)((x1 + 7) / 8) * ((y1 + 7) / 8);
    if (nt > c->tile_rays_n) {
      hipFree(c->d_tile_rays);
      c->d_tile_rays = nullptr;
      c->tile_rays_n = 0;
      HIPCHK(c, hipMalloc(&c->d_tile_rays, nt * sizeof(uint32_t)));
      HIPCHK(c, hipMemset(c->d_tile_rays, 0, nt * sizeof(uint32_t)));
      c->tile_rays_n = nt;
    }
    p.tile_rays = c->d_tile_rays;
  }
  return render_region(c, p, false, maxs, (hipStream_t)stream);
}

rtx_status rtx_tile_rays(rtx_context* c, int64_t* out, int32_t n) {
  if (!c || (!out && n > 0) || n < 0) return fail(c, RTX_EINVAL, "bad arguments");
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<uint32_t> v(c->tile_rays_n);
  if (c->d_tile_rays) {
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemcpy(v.data(), c->d_tile_rays, v.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
  }
  for (int k = 0; k < n; k++) out[k] = (size_t)k < v.size() ? (int64_t)v[k] : 0;
  return RTX_OK;
}

rtx_status rtx_render_tile_list_device(rtx_context* c, const int32_t* tiles, int32_t n, int32_t tile_rows,
                                       uint64_t seed, double* d_packed, void* stream) {
  if (!c) return RTX_EINVAL;
  if (n < 0 || (n > 0 && (!tiles || !d_packed)) || tile_rows <= 0) return fail(c, RTX_EINVAL, "bad tile list");
  KParams p;
  rtx_status s = prep(c, p, seed);
  if (s) return s;
  if (n == 0) return RTX_OK;
  const int ntiles = (c->cam.height + tile_rows - 1) / tile_rows;
  if ((int64_t)n * tile_rows > INT32_MAX) return fail(c, RTX_EINVAL, "%d tiles of %d rows exceed 2^31 rows", n, tile_rows);
  // an index past the bottom is padding: clamped to ntiles (rows y >= height render nothing), so no
  // tile * tile_rows product can overflow on the device (row_to_y)
  std::vector<int32_t> list(tiles, tiles + n);
  for (int k = 0; k < n; k++) {
    if (list[k] < 0) return fail(c, RTX_EINVAL, "tile %d: negative index %d", k, list[k]);
    if (list[k] > ntiles) list[k] = ntiles;
  }
  const int maxs = required_stack(c);
  if (maxs < 0) return fail(c, RTX_EINVAL, "trace_depth x monte_carlo_diffusion_times too large");
  if ((s = ensure_stack(c, p, maxs))) return s;
  hipSetDevice(c->device);
  if (c->rowtiles != list) {
    if ((size_t)n > c->rowtiles_cap) {
      hipFree(c->d_rowtiles);
      c->d_rowtiles = nullptr;
      c->rowtiles_cap = 0;
      HIPCHK(c, hipMalloc(&c->d_rowtiles, (size_t)n * sizeof(int32_t)));
      c->rowtiles_cap = (size_t)n;
    }
    c->rowtiles = list;
    // ordered before this call's launches on `stream` (a caller that changes
    // the list while another stream's render still reads it must sync first)
    HIPCHK(c, hipMemcpyAsync(c->d_rowtiles, c->rowtiles.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice,
                             (hipStream_t)stream));
  }
  p.x0 = 0;
  p.nx = c->cam.width;
  p.nrows = n * tile_rows;
  p.tile_rows = tile_rows;
  p.rank = 0;
  p.nranks = 1;
  p.row_tiles = c->d_rowtiles;
  p.out = d_packed;
  p.stride = (size_t)c->cam.width * 3;
  return render_region(c, p, false, maxs, (hipStream_t)stream);
}

int32_t rtx_tiles_rows_per_rank(int32_t height, int32_t tile_rows, int32_t nranks) {
  if (tile_rows <= 0 || nranks <= 0) return 0;
  const int32_t tiles = (height + tile_rows - 1) / tile_rows;
  return ((tiles + nranks - 1) / nranks) * tile_rows;
}

rtx_status rtx_render_tiles_device(rtx_context* c, int32_t tile_rows, int32_t rank, int32_t nranks,
                                   uint64_t seed, double* d_packed, void* stream) {
  if (!c) return RTX_EINVAL;
  KParams p;
  rtx_status s = prep(c, p, seed);
  if (s) return s;
  if (tile_rows <= 0 || nranks <= 0 || rank < 0 || rank >= nranks) return fail(c, RTX_EINVAL, "bad tiling");
  const int maxs = required_stack(c);
  if (maxs < 0) return fail(c, RTX_EINVAL, "trace_depth x monte_carlo_diffusion_times too large");
  if ((s = ensure_stack(c, p, maxs))) return s;
  hipSetDevice(c->device);
  p.x0 = 0;
  p.nx = c->cam.width;
  p.nrows = rtx_tiles_rows_per_rank(c->cam.height, tile_rows, nranks);
  p.tile_rows = tile_rows;
  p.rank = rank;
  p.nranks = nranks;
  p.out = d_packed;
  p.stride = (size_t)c->cam.width * 3;
  return render_region(c, p, false, maxs, (hipStream_t)stream);
}

rtx_status rtx_level_stats(rtx_context* c, int64_t* out, int32_t n) {
  if (!c || !out || n < 0) return fail(c, RTX_EINVAL, "bad arguments");
  HIPCHK(c, hipSetDevice(c->device));
  unsigned long long v[LV_MAXL + 3] = {0};
  if (c->d_lvstats) {
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemcpy(v, c->d_lvstats, sizeof v, hipMemcpyDeviceToHost));
  }
  for (int k = 0; k < n; k++) out[k] = k < LV_MAXL + 3 ? (int64_t)v[k] : 0;
  return RTX_OK;
}

rtx_status rtx_kernel_time(rtx_context* c, double* total_ms, int32_t* launches) {
  if (!c || !total_ms) return fail(c, RTX_EINVAL, "null argument");
  HIPCHK(c, hipSetDevice(c->device));
  // The union of the launches' intervals (the parts of a multi-stream
  // level render overlap), each placed relative to the first launch's start.
  std::vector<std::pair<double, double>> iv;
  for (int k = 0; k < c->n_ev; k++) {
    float a = 0.0f, b = 0.0f;
    HIPCHK(c, hipEventSynchronize(c->ev[2 * k + 1]));
    HIPCHK(c, hipEventElapsedTime(&a, c->ev[0], c->ev[2 * k]));
    HIPCHK(c, hipEventElapsedTime(&b, c->ev[0], c->ev[2 * k + 1]));
    iv.emplace_back(a, b);
  }
  std::sort(iv.begin(), iv.end());
  double sum = 0.0, lo = 0.0, hi = -1e300;
  for (const auto& v : iv) {
    if (v.first > hi) {
      if (hi > lo) sum += hi - lo;
      lo = v.first;
      hi = v.second;
    } else if (v.second > hi) {
      hi = v.second;
    }
  }
  if (hi > lo) sum += hi - lo;
  *total_ms = sum;
  if (launches) *launches = c->n_ev;
  return RTX_OK;
}

// Waits for `stream`, moves the device's raise record into `e` and resets it.
static rtx_status take_errors(rtx_context* c, void* stream, ErrState* e) {
  hipSetDevice(c->device);
  HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
  HIPCHK(c, hipMemcpy(e, c->d_err, sizeof *e, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemset(c->d_err, 0, 8));
  HIPCHK(c, hipMemset(((char*)c->d_err) + 8, 0xFF, sizeof(ErrState) - 8));
  HIPCHK(c, hipDeviceSynchronize());
  return RTX_OK;
}

// The first raise the reference would meet: the smallest key over the codes.
static rtx_status report_errors(rtx_context* c, const ErrState& e) {
  if (!e.flags) return RTX_OK;
  // device ERR_ code -> rtx_status (index = ERR_ code, rtx_vec3.h)
  static const rtx_status status_of[5] = {RTX_OK, RTX_EZERO_VEC, RTX_ECOLOR_GT1, RTX_EDOMAIN, RTX_ETYPE};
  rtx_status first = RTX_OK;
  unsigned long long key = ~0ull;
  for (int code = 1; code < 5; code++)
    if ((e.flags >> code & 1) && e.first[code] < key) {
      key = e.first[code];
      first = status_of[code];
    }
  const char* more = __builtin_popcount(e.flags) > 1 ? " (and other errors)" : "";
  if (c->err_keys_rays) return fail(c, first, "%s at ray %llu%s", rtx_status_string(first), key, more);
  // pixel keys are (x * height + y) * 2 + phase: render_sync's x-outer, y-inner
  // order (camera.rb:102-103), pre samples before extra samples (px_key)
  const unsigned long long H = c->have_cam ? (unsigned long long)c->cam.height : 1;
  const unsigned long long pix = key >> 1;
  return fail(c, first, "%s at pixel (%llu,%llu)%s", rtx_status_string(first), pix / H, pix % H, more);
}

rtx_status rtx_sync(rtx_context* c, void* stream) {
  if (!c) return RTX_EINVAL;
  ErrState e;
  const rtx_status s = take_errors(c, stream, &e);
  if (s) return s;
  return report_errors(c, e);
}

static rtx_status ensure_scratch(rtx_context* c, size_t bytes) {
  if (bytes <= c->scratch_bytes) return RTX_OK;
  hipFree(c->d_scratch);
  c->d_scratch = nullptr;
  c->scratch_bytes = 0;
  HIPCHK(c, hipMalloc(&c->d_scratch, bytes));
  c->scratch_bytes = bytes;
  return RTX_OK;
}

rtx_status rtx_render(rtx_context* c, int32_t x0, int32_t y0, int32_t x1, int32_t y1, uint64_t seed,
                      double* out, size_t row_stride) {
  if (!c || !out) return fail(c, RTX_EINVAL, "null argument");
  const int w = x1 - x0, h = y1 - y0;
  if (w < 0 || h < 0) return fail(c, RTX_EINVAL, "empty region");
  if (row_stride < (size_t)w * 3) return fail(c, RTX_EINVAL, "row_stride too small");
  if (w == 0 || h == 0) return RTX_OK;
  rtx_status s = rtx_sync(c, nullptr);               // clear stale device errors
  (void)s;
  hipSetDevice(c->device);
  if ((s = ensure_scratch(c, sizeof(double) * 3 * (size_t)w * h))) return s;
  if ((s = rtx_render_device(c, x0, y0, x1, y1, seed, c->d_scratch, (size_t)w * 3, nullptr))) return s;
  HIPCHK(c, hipMemcpy2D(out, row_stride * sizeof(double), c->d_scratch, (size_t)w * 3 * sizeof(double),
                        (size_t)w * 3 * sizeof(double), h, hipMemcpyDeviceToHost));
  return rtx_sync(c, nullptr);
}

rtx_status rtx_render_tiles(rtx_context* c, int32_t tile_rows, int32_t rank, int32_t nranks, uint64_t seed,
                            double* packed) {
  if (!c || !packed) return fail(c, RTX_EINVAL, "null argument");
  if (!c->have_cam) return fail(c, RTX_EINVAL, "no camera set");
  if (tile_rows <= 0 || nranks <= 0 || rank < 0 || rank >= nranks) return fail(c, RTX_EINVAL, "bad tiling");
  rtx_status s = rtx_sync(c, nullptr);               // clear stale device errors
  (void)s;
  hipSetDevice(c->device);
  const size_t rows = (size_t)rtx_tiles_rows_per_rank(c->cam.height, tile_rows, nranks);
  const size_t bytes = sizeof(double) * 3 * rows * (size_t)c->cam.width;
  if (bytes == 0) return RTX_OK;
  if ((s = ensure_scratch(c, bytes))) return s;
  HIPCHK(c, hipMemset(c->d_scratch, 0, bytes));
  if ((s = rtx_render_tiles_device(c, tile_rows, rank, nranks, seed, c->d_scratch, nullptr))) return s;
  HIPCHK(c, hipMemcpy(packed, c->d_scratch, bytes, hipMemcpyDeviceToHost));
  return rtx_sync(c, nullptr);
}

static rtx_status grow(rtx_context* c, double** buf, size_t* cap, size_t bytes) {
  if (bytes <= *cap) return RTX_OK;
  hipFree(*buf);
  *buf = nullptr;
  *cap = 0;
  HIPCHK(c, hipMalloc((void**)buf, bytes));
  *cap = bytes;
  return RTX_OK;
}

// rtx_render_multi / rtx_render_multi_plan: plan == nullptr deals the tiles
// round-robin, else rank k renders the list plan[k * per_rank .. + per_rank).
static rtx_status render_multi(rtx_context* const* ctxs, int32_t n, int32_t tile_rows, const int32_t* plan,
                               int32_t per_rank, uint64_t seed, double* out, size_t row_stride) {
  if (!ctxs || n < 1 || !ctxs[0]) return RTX_EINVAL;
  rtx_context* c0 = ctxs[0];
  if (!out || tile_rows <= 0) return fail(c0, RTX_EINVAL, "bad arguments");
  if (plan && (per_rank < 1 || (int64_t)per_rank * tile_rows > INT32_MAX / 2))
    return fail(c0, RTX_EINVAL, "bad plan: %d tiles per rank", per_rank);
  std::vector<int> devs(n);
  for (int k = 0; k < n; k++) {
    rtx_context* c = ctxs[k];
    if (!c || !c->have_scene || !c->have_cam) return fail(c0, RTX_EINVAL, "context %d has no scene or camera", k);
    if (c->cam.width != c0->cam.width || c->cam.height != c0->cam.height)
      return fail(c0, RTX_EINVAL, "context %d renders a different image size", k);
    devs[k] = c->device;
  }
  const int W = c0->cam.width, H = c0->cam.height;
  if (row_stride < (size_t)W * 3) return fail(c0, RTX_EINVAL, "row_stride too small");
  const int ntiles = (H + tile_rows - 1) / tile_rows;
  std::vector<int32_t> pl;                                     // the plan, padding clamped to ntiles
  if (plan) {
    pl.assign(plan, plan + (size_t)n * per_rank);
    std::vector<char> seen(ntiles, 0);
    for (int32_t& t : pl) {
      if (t < 0) return fail(c0, RTX_EINVAL, "plan: negative tile index %d", t);
      if (t >= ntiles) {
        t = ntiles;
        continue;
      }
      if (seen[t]++) return fail(c0, RTX_EINVAL, "plan: tile %d listed twice", t);
    }
    for (int t = 0; t < ntiles; t++)
      if (!seen[t]) return fail(c0, RTX_EINVAL, "plan: tile %d in no rank's list", t);
  }
  const int R = plan ? per_rank * tile_rows : rtx_tiles_rows_per_rank(H, tile_rows, n);
  const size_t count = (size_t)R * W * 3;                      // doubles per rank
  // clear stale device errors (as rtx_render: unsynced raises of earlier
  // asynchronous calls on these contexts are discarded, include/rtx.h)
  for (int k = 0; k < n; k++) (void)rtx_sync(ctxs[k], nullptr);
  // every rank renders its tiles on its own device; the devices run concurrently
  for (int k = 0; k < n; k++) {
    rtx_context* c = ctxs[k];
    HIPCHK(c0, hipSetDevice(c->device));
    rtx_status s = grow(c, &c->d_multi, &c->multi_bytes, count * sizeof(double));
    if (!s)
      s = plan ? rtx_render_tile_list_device(c, pl.data() + (size_t)k * per_rank, per_rank, tile_rows, seed,
                                             c->d_multi, nullptr)
               : rtx_render_tiles_device(c, tile_rows, k, n, seed, c->d_multi, nullptr);
    if (s) return fail(c0, s, "rank %d: %s", k, rtx_last_error(c));
  }
  HIPCHK(c0, hipSetDevice(c0->device));
  const size_t plan_dbl = plan ? ((size_t)n * per_rank * sizeof(int32_t) + 7) / 8 : 0;
  rtx_status s = grow(c0, &c0->d_gather, &c0->gather_bytes,
                      ((size_t)n * count + (size_t)W * H * 3 + plan_dbl) * sizeof(double));
  if (s) return s;
  double* gathered = c0->d_gather;
  double* frame = c0->d_gather + (size_t)n * count;
  int32_t* d_plan = plan ? reinterpret_cast<int32_t*>(frame + (size_t)W * H * 3) : nullptr;
  if (plan) HIPCHK(c0, hipMemcpy(d_plan, pl.data(), pl.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  bool distinct = true;
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++) distinct = distinct && devs[a] != devs[b];
  if (distinct) {
    // ONE gather to rank 0 over RCCL (xGMI): grouped ncclSend / ncclRecv on
    // every device's stream, ordered after that device's render.
    if (c0->comm_devs != devs) {
      for (size_t k = 0; k < c0->comms.size(); k++) {
        hipSetDevice(c0->comm_devs[k]);
        ncclCommDestroy(c0->comms[k]);
      }
      c0->comms.assign(n, nullptr);
      c0->comm_devs.clear();
      const ncclResult_t ri = ncclCommInitAll(c0->comms.data(), n, devs.data());
      if (ri != ncclSuccess) {
        c0->comms.clear();                       // nothing to destroy later
        return fail(c0, RTX_ERCCL, "ncclCommInitAll: %s", ncclGetErrorString(ri));
      }
      c0->comm_devs = devs;
    }
    // Every call between GroupStart and GroupEnd is made and GroupEnd always
    // runs, so a failure never leaves this thread inside an open RCCL group;
    // after one the cached communicators are torn down (the next call
    // re-initialises them).
    ncclResult_t r = ncclGroupStart();
    const char* what = r != ncclSuccess ? "ncclGroupStart" : nullptr;
    if (r == ncclSuccess) {
      for (int k = 0; k < n; k++) {
        hipSetDevice(devs[k]);
        const ncclResult_t rk = ncclSend(ctxs[k]->d_multi, count, ncclFloat64, 0, c0->comms[k], nullptr);
        if (rk != ncclSuccess && !what) r = rk, what = "ncclSend";
      }
      hipSetDevice(devs[0]);
      for (int k = 0; k < n; k++) {
        const ncclResult_t rk = ncclRecv(gathered + (size_t)k * count, count, ncclFloat64, k, c0->comms[0], nullptr);
        if (rk != ncclSuccess && !what) r = rk, what = "ncclRecv";
      }
      const ncclResult_t re = ncclGroupEnd();
      if (re != ncclSuccess && !what) r = re, what = "ncclGroupEnd";
    }
    if (what) {
      // sends / receives may already be enqueued: abort (ncclCommDestroy would
      // wait for them and can hang where abort does not)
      for (size_t k = 0; k < c0->comms.size(); k++) {
        hipSetDevice(c0->comm_devs[k]);
        ncclCommAbort(c0->comms[k]);
      }
      c0->comms.clear();
      c0->comm_devs.clear();
      hipSetDevice(devs[0]);
      return fail(c0, RTX_ERCCL, "%s: %s", what, ncclGetErrorString(r));
    }
  } else {
    // several ranks on one device (more workers than GPUs): device copies
    for (int k = 0; k < n; k++) {
      HIPCHK(c0, hipSetDevice(devs[k]));
      HIPCHK(c0, hipDeviceSynchronize());
      HIPCHK(c0, hipMemcpyPeer(gathered + (size_t)k * count, devs[0], ctxs[k]->d_multi, devs[k],
                               count * sizeof(double)));
    }
  }
  HIPCHK(c0, hipSetDevice(devs[0]));
  HIPCHK(c0, plan ? launch_unpack_plan(gathered, W, H, tile_rows, n, per_rank, d_plan, frame, (size_t)W * 3, nullptr)
                  : launch_unpack(gathered, W, H, tile_rows, n, R, frame, (size_t)W * 3, nullptr));
  HIPCHK(c0, hipMemcpy2D(out, row_stride * sizeof(double), frame, (size_t)W * 3 * sizeof(double),
                         (size_t)W * 3 * sizeof(double), H, hipMemcpyDeviceToHost));
  // the ranks' reference raises, merged: the first in render_sync order over
  // the whole frame (pixel keys do not depend on the rank that rendered them)
  ErrState all;
  all.flags = 0;
  for (int code = 0; code < 5; code++) all.first[code] = ~0ull;
  // Every rank's record is taken (and reset) even after one fails, so no
  // rank is left holding raises for a later call; the first failure wins.
  rtx_status take_fail = RTX_OK;
  int fail_rank = -1;
  for (int k = 0; k < n; k++) {
    ErrState e;
    const rtx_status st = take_errors(ctxs[k], nullptr, &e);
    if (st) {
      if (!take_fail) take_fail = st, fail_rank = k;
      continue;
    }
    all.flags |= e.flags;
    for (int code = 0; code < 5; code++)
      if (e.first[code] < all.first[code]) all.first[code] = e.first[code];
  }
  hipSetDevice(devs[0]);
  if (take_fail) return fail(c0, take_fail, "rank %d: %s", fail_rank, rtx_last_error(ctxs[fail_rank]));
  return report_errors(c0, all);
}

int32_t rtx_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

rtx_status rtx_render_multi(rtx_context* const* ctxs, int32_t n, int32_t tile_rows, uint64_t seed, double* out,
                            size_t row_stride) {
  return render_multi(ctxs, n, tile_rows, nullptr, 0, seed, out, row_stride);
}

rtx_status rtx_render_multi_plan(rtx_context* const* ctxs, int32_t n, int32_t tile_rows, const int32_t* plan,
                                 int32_t per_rank, uint64_t seed, double* out, size_t row_stride) {
  if (!plan) return ctxs && n > 0 && ctxs[0] ? fail(ctxs[0], RTX_EINVAL, "null plan") : RTX_EINVAL;
  return render_multi(ctxs, n, tile_rows, plan, per_rank, seed, out, row_stride);
}

rtx_status rtx_tile_probe(rtx_context* c, int64_t* out, int32_t n) {
  if (!c || n < 0 || (n > 0 && !out)) return fail(c, RTX_EINVAL, "bad arguments");
  KParams p;
  rtx_status s = prep(c, p, 1);
  if (s) return s;
  HIPCHK(c, hipSetDevice(c->device));
  p.x0 = 0;
  p.nx = c->cam.width;
  p.y0 = 0;
  p.nrows = c->cam.height;
  p.tile_rows = 0;
  const int tiles = ((p.nx + 7) / 8) * ((p.nrows + 7) / 8);
  int32_t* d = nullptr;
  HIPCHK(c, hipMalloc(&d, (size_t)std::max(1, tiles) * sizeof(int32_t)));
  std::vector<int32_t> v(tiles);
  hipError_t e = launch_tile_probe(p, d, nullptr);
  if (e == hipSuccess) e = hipMemcpy(v.data(), d, (size_t)tiles * sizeof(int32_t), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  HIPCHK(c, e);
  for (int k = 0; k < n; k++) out[k] = k < tiles ? (int64_t)v[k] : 0;
  return RTX_OK;
}

rtx_status rtx_lpt_plan(const int64_t* costs, int32_t n_tiles, int32_t nranks, int32_t* plan, int32_t cap,
                        int32_t* per_rank) {
  if (n_tiles < 0 || nranks < 1 || (n_tiles > 0 && !costs) || !per_rank) return RTX_EINVAL;
  std::vector<int32_t> order(n_tiles);
  for (int32_t t = 0; t < n_tiles; t++) order[t] = t;
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return costs[a] > costs[b]; });
  std::vector<int64_t> load(nranks, 0);
  std::vector<std::vector<int32_t>> lists(nranks);
  for (int32_t t : order) {                     // to the least-loaded rank (ties: fewer tiles, lower rank)
    int r = 0;
    for (int k = 1; k < nranks; k++)
      if (load[k] < load[r] || (load[k] == load[r] && lists[k].size() < lists[r].size())) r = k;
    lists[r].push_back(t);
    load[r] += costs[t];
  }
  size_t width = 0;
  for (auto& l : lists) {
    std::sort(l.begin(), l.end());
    width = std::max(width, l.size());
  }
  *per_rank = (int32_t)width;
  if (!plan) return RTX_OK;                     // (a query of the width)
  if (cap < 0 || (size_t)cap < width) return RTX_EINVAL;   // (a negative cap: refused, not a huge size_t)
  for (int k = 0; k < nranks; k++)
    for (size_t j = 0; j < width; j++) plan[(size_t)k * width + j] = j < lists[k].size() ? lists[k][j] : n_tiles;
  return RTX_OK;
}

rtx_status rtx_render_at(rtx_context* c, int32_t x, int32_t y, uint64_t seed, double rgb[3]) {
  return rtx_render(c, x, y, x + 1, y + 1, seed, rgb, 3);
}

rtx_status rtx_trace(rtx_context* c, int32_t n, const double* rays, const int32_t* keys, uint64_t seed,
                     double* out) {
  if (!c || n < 0 || (n && (!rays || !keys || !out))) return fail(c, RTX_EINVAL, "bad arguments");
  if (n == 0) return RTX_OK;
  KParams p;
  rtx_status s = prep(c, p, seed);
  if (s) return s;
  const int maxs = required_stack(c);
  if (maxs < 0) return fail(c, RTX_EINVAL, "trace_depth x monte_carlo_diffusion_times too large");
  if ((s = ensure_stack(c, p, maxs))) return s;
  rtx_sync(c, nullptr);
  hipSetDevice(c->device);
  const size_t rb = sizeof(double) * 6 * n, kb = sizeof(int32_t) * 3 * n, ob = sizeof(double) * 3 * n;
  if ((s = ensure_scratch(c, rb + kb + ob + 64))) return s;
  char* base = (char*)c->d_scratch;
  double* d_rays = (double*)base;
  double* d_out = (double*)(base + rb);
  int32_t* d_keys = (int32_t*)(base + rb + ob);
  HIPCHK(c, hipMemcpy(d_rays, rays, rb, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemcpy(d_keys, keys, kb, hipMemcpyHostToDevice));
  p.out = d_out;
  p.rays = d_rays;
  p.keys = d_keys;
  p.nrays = n;
  HIPCHK(c, launch_trace(p, sph_mode(c), maxs, nullptr));
  HIPCHK(c, hipMemcpy(out, d_out, ob, hipMemcpyDeviceToHost));
  c->err_keys_rays = true;
  const rtx_status st = rtx_sync(c, nullptr);
  c->err_keys_rays = false;
  return st;
}

rtx_status rtx_path_trace(rtx_context* c, int32_t n, const double* rays, double* out) {
  if (!c || n < 0 || (n && (!rays || !out))) return fail(c, RTX_EINVAL, "bad arguments");
  if (n == 0) return RTX_OK;
  KParams p;
  rtx_status s = prep(c, p, 1);
  if (s) return s;
  rtx_sync(c, nullptr);
  hipSetDevice(c->device);
  const size_t rb = sizeof(double) * 6 * n, ob = sizeof(double) * 3 * n;
  if ((s = ensure_scratch(c, rb + ob))) return s;
  double* d_rays = c->d_scratch;
  double* d_out = c->d_scratch + 6 * (size_t)n;
  HIPCHK(c, hipMemcpy(d_rays, rays, rb, hipMemcpyHostToDevice));
  p.out = d_out;
  p.rays = d_rays;
  p.nrays = n;
  HIPCHK(c, launch_path_trace(p, nullptr));
  HIPCHK(c, hipMemcpy(out, d_out, ob, hipMemcpyDeviceToHost));
  c->err_keys_rays = true;
  const rtx_status st = rtx_sync(c, nullptr);
  c->err_keys_rays = false;
  return st;
}

rtx_status rtx_count_work(rtx_context* c, uint64_t seed, uint64_t counts[RTX_NCOUNT]) {
  if (!c || !counts) return fail(c, RTX_EINVAL, "null argument");
  KParams p;
  rtx_status s = prep(c, p, seed);
  if (s) return s;
  const int maxs = required_stack(c);
  if (maxs < 0) return fail(c, RTX_EINVAL, "trace_depth x monte_carlo_diffusion_times too large");
  if ((s = ensure_stack(c, p, maxs))) return s;
  hipSetDevice(c->device);
  const int W = c->cam.width, H = c->cam.height;
  if ((s = ensure_scratch(c, sizeof(double) * 3 * (size_t)W * H))) return s;
  HIPCHK(c, hipMemset(c->d_counts, 0, sizeof(unsigned long long) * RTX_NCOUNT));
  p.x0 = 0;
  p.nx = W;
  p.nrows = H;
  p.out = c->d_scratch;
  p.stride = (size_t)W * 3;
  if ((s = render_region(c, p, true, maxs, nullptr))) return s;
  HIPCHK(c, hipDeviceSynchronize());
  unsigned long long tmp[RTX_NCOUNT];
  HIPCHK(c, hipMemcpy(tmp, c->d_counts, sizeof tmp, hipMemcpyDeviceToHost));
  for (int k = 0; k < RTX_NCOUNT; k++) counts[k] = tmp[k];
  return rtx_sync(c, nullptr);
}

rtx_status rtx_quantize_device(const double* d_rgb, int32_t w, int32_t h, size_t stride, int32_t blend,
                               uint8_t* d_out, void* stream) {
  if (w < 0 || h < 0 || stride < (size_t)w * 3 || (w * h && (!d_rgb || !d_out))) return RTX_EINVAL;
  return launch_quantize(d_rgb, w, h, stride, blend, d_out, (hipStream_t)stream) == hipSuccess ? RTX_OK
                                                                                                 : RTX_EHIP;
}

rtx_status rtx_quantize(const double* rgb, int32_t w, int32_t h, size_t stride, int32_t blend, uint8_t* out) {
  if (w < 0 || h < 0 || stride < (size_t)w * 3 || (w * h && (!rgb || !out))) return RTX_EINVAL;
  if (w * h == 0) return RTX_OK;
  double* d_in = nullptr;
  uint8_t* d_o = nullptr;
  const size_t ib = sizeof(double) * stride * h, ob = (size_t)w * h * 4;
  rtx_status s = RTX_OK;
  if (hipMalloc(&d_in, ib) != hipSuccess || hipMalloc(&d_o, ob) != hipSuccess ||
      hipMemcpy(d_in, rgb, ib, hipMemcpyHostToDevice) != hipSuccess ||
      launch_quantize(d_in, w, h, stride, blend, d_o, nullptr) != hipSuccess ||
      hipMemcpy(out, d_o, ob, hipMemcpyDeviceToHost) != hipSuccess)
    s = RTX_EHIP;
  hipFree(d_in);
  hipFree(d_o);
  return s;
}

// ------------------------------------------------------------------ Vec3 API
static rtx_vec3 mk(V3 a) {
  rtx_vec3 r;
  r.v[0] = a.x;
  r.v[1] = a.y;
  r.v[2] = a.z;
  r.r = sqrt(a.x * a.x + a.y * a.y + a.z * a.z);      // Vec3_c_create (fast_4d_matrix.c:62-73)
  return r;
}
static V3 un(rtx_vec3 a) { return v3(a.v[0], a.v[1], a.v[2]); }

rtx_vec3 rtx_vec3_from_a(double x, double y, double z) { return mk(v3(x, y, z)); }
double rtx_vec3_r(rtx_vec3 a) { return a.r; }
double rtx_vec3_r2(rtx_vec3 a) { return a.r * a.r; }
double rtx_vec3_dot(rtx_vec3 a, rtx_vec3 b) { return vdot(un(a), un(b)); }
rtx_status rtx_vec3_cos(rtx_vec3 a, rtx_vec3 b, double* out) {
  uint32_t err = 0;
  double v = vcos(un(a), un(b), err);
  if (out) *out = v;
  return err ? RTX_EZERO_VEC : RTX_OK;
}
rtx_vec3 rtx_vec3_cross(rtx_vec3 a, rtx_vec3 b) { return mk(vcross(un(a), un(b))); }
rtx_vec3 rtx_vec3_add(rtx_vec3 a, rtx_vec3 b) { return mk(vadd(un(a), un(b))); }
rtx_vec3 rtx_vec3_sub(rtx_vec3 a, rtx_vec3 b) { return mk(vsub(un(a), un(b))); }
rtx_vec3 rtx_vec3_mul(rtx_vec3 a, rtx_vec3 b) { return mk(vmul(un(a), un(b))); }
rtx_vec3 rtx_vec3_scale(rtx_vec3 a, double s) { return mk(vsc(un(a), s)); }
rtx_vec3 rtx_vec3_div(rtx_vec3 a, double s) { return mk(vdiv(un(a), s)); }
rtx_vec3 rtx_vec3_neg(rtx_vec3 a) { return mk(vneg(un(a))); }
rtx_vec3 rtx_vec3_pos(rtx_vec3 a) { return mk(un(a)); }
rtx_status rtx_vec3_normalize(rtx_vec3 a, rtx_vec3* out) {
  uint32_t err = 0;
  V3 v = vnorm(un(a), err);
  if (err) return RTX_EZERO_VEC;
  if (out) *out = mk(v);
  return RTX_OK;
}
// The bang forms mutate in place and recompute r (Vec3_c_recalc_r, :226-229);
// as values they equal the non-bang results.
rtx_vec3 rtx_vec3_add_bang(rtx_vec3 a, rtx_vec3 b) { return mk(vadd(un(a), un(b))); }
rtx_vec3 rtx_vec3_sub_bang(rtx_vec3 a, rtx_vec3 b) { return mk(vsub(un(a), un(b))); }
rtx_vec3 rtx_vec3_mul_bang(rtx_vec3 a, rtx_vec3 b) { return mk(vmul(un(a), un(b))); }
rtx_vec3 rtx_vec3_mul_bang_scalar(rtx_vec3 a, double s) { return mk(vsc(un(a), s)); }

double rtx_rand(uint64_t seed, int32_t x, int32_t y, int32_t sample, uint64_t path, int32_t draw) {
  return rand01(seed, x, y, sample, path, draw);
}

}  // extern "C"
