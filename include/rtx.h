/*
 * rtx.h — C-ABI of librtx, the MI355X-native replacement for the hot path of
 * a1exwang/raytracing_rb:  Camera#render_at -> RayTracer#trace_sync
 * (src/camera.rb:70-110, src/ray_tracer.rb:16-164) together with the native
 * Vec3 it runs on (ext/fast_4d_matrix/fast_4d_matrix.c) and the fork_jobs tile
 * scheduler that parallelises it (src/fork_jobs.rb:1-33, camera.rb:41-68).
 *
 * Plain C: no Ruby, HIP or torch types.  Pointers are caller-owned.  All
 * arithmetic is IEEE binary64 with the reference's operation order (no FMA).
 *
 * Reference interfaces replaced (file:line of the reference, read-only at
 * /root/reference):
 *   rtx_scene_upload      World.new(world.yml)         src/world.rb:15-34,
 *                          ConfigurableObject            src/configurable_object.rb:43-49,
 *                          Sphere/Plane/Box/Texture.new  src/objects/{sphere,plane,box,texture}.rb
 *   rtx_camera_set        Camera.new(world, camera.yml) src/camera.rb:26-34
 *   rtx_render            Camera#render_sync loops       src/camera.rb:101-110
 *   rtx_render_device     (same, device-resident output, async on a HIP stream)
 *   rtx_render_tiles_device  the per-child work of Camera#render_fork +
 *                          fork_jobs                      src/camera.rb:53-65, src/fork_jobs.rb:5-22
 *   rtx_render_multi      Camera#render_fork + fork_jobs over the node's GPUs with an RCCL gather
 *                                                         src/camera.rb:41-68, src/fork_jobs.rb:1-33
 *   rtx_render_at         Camera#render_at(x, y)         src/camera.rb:70-99
 *   rtx_trace             RayTracer#trace_sync(x, y, ray) src/ray_tracer.rb:16-46
 *   rtx_path_trace        RayTracer#path_trace_sync(x, y, ray) src/ray_tracer.rb:181-289 (dead code there)
 *   rtx_quantize          Camera#array_to_color + canvas.point  src/camera.rb:105,153-156
 *   rtx_vec3_*            Fast4DMatrix::Vec3 methods     ext/fast_4d_matrix/fast_4d_matrix.c:29-55
 *   rtx_status codes      the reference's raise sites    fast_4d_matrix.c:124,220,291;
 *                          ray_tracer.rb:294-296; world_object.rb:106; sphere.rb:45-46
 */
#ifndef RTX_H
#define RTX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTX_ABI_VERSION 1

typedef enum rtx_status {
  RTX_OK = 0,
  RTX_EZERO_VEC = 1,   /* "zero vector detected" fast_4d_matrix.c:124,291; world_object.rb:106 */
  RTX_ECOLOR_GT1 = 2,  /* "color greater than 1"  ray_tracer.rb:294-296 (also NaN channels)      */
  RTX_EDOMAIN = 3,     /* Math::DomainError / FloatDomainError: sphere.rb:45-46, texture.rb:24-25 */
  RTX_EHIP = 4,        /* HIP runtime failure                                                    */
  RTX_ERCCL = 5,       /* collective failure (reported by the host layer)                        */
  RTX_EINVAL = 6,      /* bad descriptor: the reference's NoMethodError/TypeError on missing keys */
  RTX_ENOMEM = 7,
  RTX_ETYPE = 8        /* TypeError "nil can't be coerced into Integer": path_trace's roulette_random
                          over unassigned probabilities, ray_tracer.rb:167 (world_object.rb:12)       */
} rtx_status;

enum rtx_object_type { RTX_SPHERE = 0, RTX_PLANE = 1, RTX_BOX = 2 };

/* One entry of world.yml `world_objects:` (YAML order is significant: the
 * first object wins distance ties, world.rb:48-50).  Field names are the YAML
 * property names of src/objects/{world_object,sphere,plane,box}.rb. */
typedef struct rtx_object_desc {
  int32_t type;                      /* rtx_object_type                                      */
  int32_t texture_id;                /* index into rtx_scene_desc.textures, -1 = none        */
  int32_t has_refractive_rate;       /* Ruby truthiness of `refractive_rate` (plane.rb:57)   */
  int32_t has_refractive_attenuation;
  double diffuse_rate[3];
  double ambient[3];
  double reflective_attenuation[3];
  double refractive_attenuation[3];
  double refractive_rate;
  /* Sphere (sphere.rb) */
  double center[3];
  double radius;
  double north_pole_vec[3];
  double greenwich_vec[3];
  double texture_u_offset;           /* Texture u_off/v_off: spheres only (sphere.rb:25)     */
  double texture_v_offset;
  /* Plane (plane.rb) / Box (box.rb) */
  double point[3];
  double front[3];
  double up[3];
  double u_unit, v_unit;             /* plane                                                */
  double width_front, width_up, width_left;   /* box                                       */
  double texture_horizontal_scale;
  double texture_vertical_scale;
} rtx_object_desc;

/* One entry of world.yml `lights:` (src/lights/light.rb:3-4, spot_light.rb:5). */
typedef struct rtx_light_desc {
  double position[3];
  double color[3];
  double radius;                     /* 0 = point light                                      */
  double high_light_rate;
  double high_light_angle;           /* degrees                                              */
} rtx_light_desc;

/* A decoded texture (texture.rb:12-20): RGB bytes, rows top-down, each byte the
 * high byte of the 16-bit quantum (`pixel.red >> 8`); the library applies /256.0. */
typedef struct rtx_texture_desc {
  int32_t width;
  int32_t height;
  const uint8_t* rgb;
} rtx_texture_desc;

typedef struct rtx_scene_desc {
  double max_distance;               /* world.yml max_distance         */
  double soft_shadow_exponent;       /* world.yml soft_shadow_exponent */
  int32_t n_objects;
  int32_t n_lights;
  int32_t n_textures;
  int32_t reserved;
  const rtx_object_desc* objects;
  const rtx_light_desc* lights;
  const rtx_texture_desc* textures;
} rtx_scene_desc;

/* camera.yml, 1:1 (src/camera.rb:17-24). */
typedef struct rtx_camera_desc {
  double position[3];
  double up[3];
  double front[3];
  double retina_width;
  double retina_height;
  double aperture_radius;
  double image_distance;
  double focal_distance;
  double variant_threshold;
  int32_t width;
  int32_t height;
  int32_t pre_sample_times;
  int32_t max_sample_times;
  int32_t trace_depth;
  int32_t monte_carlo_diffusion_times;
} rtx_camera_desc;

/* Vec3 value with its cached norm, as Vec3Type (fast_4d_matrix.c:57-60). */
typedef struct rtx_vec3 {
  double v[3];
  double r;
} rtx_vec3;

typedef struct rtx_context rtx_context;

/* ---- context ------------------------------------------------------------ */
rtx_status  rtx_context_create(int32_t device, rtx_context** out);
void        rtx_context_destroy(rtx_context* ctx);
const char* rtx_last_error(const rtx_context* ctx);
const char* rtx_status_string(rtx_status s);
int32_t     rtx_abi_version(void);
/* Identity of the build: the first 16 hex digits of the sha256 over the device
 * sources, headers and compiler flags it was built from (the host layer checks
 * it against the tree before use; the PMC profiles carry the same value). */
const char* rtx_build_id(void);

/* ---- scene / camera (World.new, Camera.new) ----------------------------- */
rtx_status rtx_scene_upload(rtx_context* ctx, const rtx_scene_desc* scene);
rtx_status rtx_camera_set(rtx_context* ctx, const rtx_camera_desc* camera);

/* ---- rendering ---------------------------------------------------------- */
/* Camera#render_sync: pixels [x0,x1) x [y0,y1) into the caller-owned host
 * buffer out_rgb (row-major; out_rgb[(y-y0)*row_stride + (x-x0)*3 + c]) in final
 * image orientation (row = y = top row first), before quantization.
 * Synchronous.  RNG key: seed (main.rb:10 uses Random.srand(1)).
 * The synchronous host-buffer calls (rtx_render, rtx_render_at,
 * rtx_render_tiles, rtx_render_multi) start by discarding raises that earlier
 * asynchronous *_device calls on the same context(s) recorded and nobody
 * collected: call rtx_sync first to read those. */
rtx_status rtx_render(rtx_context* ctx, int32_t x0, int32_t y0, int32_t x1, int32_t y1,
                      uint64_t seed, double* out_rgb, size_t row_stride);

/* As rtx_render, but d_out is DEVICE memory and the work is enqueued on
 * `hip_stream` (a hipStream_t, NULL = default) without host synchronization.
 * Reference raise sites are recorded on the device; read them with rtx_sync. */
rtx_status rtx_render_device(rtx_context* ctx, int32_t x0, int32_t y0, int32_t x1, int32_t y1,
                             uint64_t seed, double* d_out, size_t row_stride, void* hip_stream);

/* One rank's share of a frame split into `tile_rows`-row tiles dealt
 * round-robin: tile t belongs to rank t % nranks (the GPU replacement of
 * camera.rb:53-65's contiguous column bands).  Packed output in device memory:
 * local tile k of this rank = global tile k*nranks+rank is stored at rows
 * [k*tile_rows, (k+1)*tile_rows) of d_packed (width*3 doubles per row);
 * rows past the image bottom are left untouched.  Packed rows per rank:
 * rtx_tiles_rows_per_rank(). */
int32_t    rtx_tiles_rows_per_rank(int32_t height, int32_t tile_rows, int32_t nranks);
rtx_status rtx_render_tiles_device(rtx_context* ctx, int32_t tile_rows, int32_t rank, int32_t nranks,
                                   uint64_t seed, double* d_packed, void* hip_stream);

/* One rank's share given as an explicit list of `tile_rows`-row tiles (a
 * cost-balanced split of camera.rb:53-65's bands, e.g. longest-processing-time
 * over rtx_tile_rays): tiles[k] (host array, n entries; an index past the
 * image bottom is padding) is stored at rows [k*tile_rows, (k+1)*tile_rows)
 * of d_packed.  The list is copied to the device when it differs from the
 * previous call's.  Same bits as any other split. */
rtx_status rtx_render_tile_list_device(rtx_context* ctx, const int32_t* tiles, int32_t n, int32_t tile_rows,
                                       uint64_t seed, double* d_packed, void* hip_stream);

/* Rays traced per 8x8 tile (the tree records of its 64 x pre_sample_times
 * camera samples' trees; extra samples not counted) in the last whole-frame
 * render of this context with the bounce-level engine, row-major over the
 * frame's ceil(width/8) x ceil(height/8) tiles: a measured work map for
 * balancing tile splits.  Every whole-frame level render rewrites every
 * tile's count.  A sample re-rendered by the lanes engine (a capacity
 * overflow, rtx_level_stats' redo) has no tree records and counts 0 rays.
 * Synchronous; zeros before such a render. */
rtx_status rtx_tile_rays(rtx_context* ctx, int64_t* out, int32_t n);

/* Host-buffer variant of rtx_render_tiles_device (synchronous): packed holds
 * rtx_tiles_rows_per_rank() * width * 3 doubles.  One call per worker of
 * Camera#render_fork (camera.rb:41-68) in a single-process, multi-GPU host. */
rtx_status rtx_render_tiles(rtx_context* ctx, int32_t tile_rows, int32_t rank, int32_t nranks, uint64_t seed,
                            double* packed);

/* Camera#render_fork(path, n) + fork_jobs in one process (camera.rb:41-68,
 * fork_jobs.rb:5-22): ctxs[k] (each with the same scene and camera uploaded,
 * one per worker, normally one per GPU) renders rank k's share of the frame
 * cut into tile_rows-row tiles dealt round-robin; the packed tiles are
 * gathered to ctxs[0]'s device with ONE grouped RCCL ncclSend/ncclRecv over
 * xGMI (device copies instead when several contexts share a device),
 * unpacked there and copied into the caller's host buffer out_rgb (layout of
 * rtx_render).  Synchronous.  RTX_ERCCL when the collective fails (the group
 * is always closed and the cached communicators are re-created by the next
 * call).  The ranks' reference raises are merged: the one returned is the
 * first over the whole frame in render_sync order, as in rtx_render. */
rtx_status rtx_render_multi(rtx_context* const* ctxs, int32_t n, int32_t tile_rows, uint64_t seed,
                            double* out_rgb, size_t row_stride);

/* rtx_render_multi with an explicit split (camera.rb:53-65's bands replaced by
 * cost-balanced tile lists): rank k renders the tiles plan[k * per_rank ..
 * k * per_rank + per_rank) (rtx_render_tile_list_device; an index past the
 * image bottom is padding), the packed lists are gathered the same way and
 * unpacked by the plan.  Every tile must appear in exactly one list
 * (RTX_EINVAL otherwise).  Same bits as rtx_render. */
rtx_status rtx_render_multi_plan(rtx_context* const* ctxs, int32_t n, int32_t tile_rows, const int32_t* plan,
                                 int32_t per_rank, uint64_t seed, double* out_rgb, size_t row_stride);

/* A cheap work map without rendering: per 8x8 tile of the frame (row-major,
 * ceil(width/8) x ceil(height/8)) the weight of 4 probe rays (sample 0's lens
 * rays at the quadrant centres, one nearest-hit walk each: 1 per hit, +1
 * reflective, +3 refractive material; the expensive-tiles-first class of the
 * lanes engine).  Synchronous. */
rtx_status rtx_tile_probe(rtx_context* ctx, int64_t* out, int32_t n);

/* Longest-processing-time split of n_tiles tiles (costs[t]) over nranks:
 * tiles by decreasing cost (ties: lower index), each to the rank with the
 * least total so far (ties: fewer tiles, lower rank); every list ascending and
 * padded to one width with n_tiles.  *per_rank = that width; plan (nranks x
 * width, rank-major, cap >= width entries per rank) may be NULL to query it.
 * Host-only, deterministic (raytracing_rb_amd/tiles.py lpt_plan). */
rtx_status rtx_lpt_plan(const int64_t* costs, int32_t n_tiles, int32_t nranks, int32_t* plan, int32_t cap,
                        int32_t* per_rank);

/* Number of HIP devices visible to this process (the node's GPUs). */
int32_t    rtx_device_count(void);

/* Wait for `hip_stream` and report the first reference raise recorded by the
 * device since the last rtx_sync (RTX_OK if none); details in rtx_last_error.
 * "First" is the reference's order: pixels in render_sync order (x outer, y
 * inner, camera.rb:101-103), within a pixel its pre samples before its extra
 * samples and samples in order (camera.rb:72-97), within a sample trace_sync's
 * order; rays (rtx_trace) by index. */
rtx_status rtx_sync(rtx_context* ctx, void* hip_stream);

/* Camera#render_at(x, y): the averaged colour of one pixel. */
rtx_status rtx_render_at(rtx_context* ctx, int32_t x, int32_t y, uint64_t seed, double rgb[3]);

/* RayTracer#trace_sync(x, y, ray) for n rays at once (host buffers).
 * rays[i*6 + 0..2] = Ray#front, rays[i*6 + 3..5] = Ray#position;
 * keys[i*3 + 0..2] = (x, y, sample) — the RNG key of the ray tree. */
rtx_status rtx_trace(rtx_context* ctx, int32_t n, const double* rays, const int32_t* keys,
                     uint64_t seed, double* out_rgb);

/* RayTracer#path_trace_sync(x, y, ray) for n rays (host buffers, rays as in
 * rtx_trace).  Never called by the reference, reproduced with its behaviour:
 * black below trace_depth 1 or on a miss, the highlight sum when a light's
 * cone holds the ray, and RTX_ETYPE on any object hit (roulette_random over
 * nil probabilities raises before any Monte-Carlo child exists). */
rtx_status rtx_path_trace(rtx_context* ctx, int32_t n, const double* rays, double* out_rgb);

/* Camera#array_to_color (camera.rb:153-156) + PNG::Canvas#point: RGBA8,
 * byte = trunc(min(256*c, 255)); png_gem_blend != 0 additionally applies the
 * png gem's alpha blend over the black canvas ((v*255) >> 8).  Host buffers. */
rtx_status rtx_quantize(const double* rgb, int32_t width, int32_t height, size_t row_stride,
                        int32_t png_gem_blend, uint8_t* out_rgba);
/* Device variant (async on hip_stream). */
rtx_status rtx_quantize_device(const double* d_rgb, int32_t width, int32_t height, size_t row_stride,
                               int32_t png_gem_blend, uint8_t* d_out_rgba, void* hip_stream);

/* Algorithmic work counters of one frame (brute-force reference algorithm),
 * for the roofline: see DESIGN.md "Algorithmic FP64 ops".  counts[RTX_NCOUNT]. */
enum {
  RTX_CNT_RAYS = 0,          /* rt_map calls that passed the cutoff                     */
  RTX_CNT_SPHERE_TESTS,      /* Sphere#intersect calls from World#intersect            */
  RTX_CNT_SPHERE_HITS,
  RTX_CNT_PLANE_TESTS,
  RTX_CNT_BOX_TESTS,
  RTX_CNT_SHADE_HITS,        /* rays with a nearest hit                                 */
  RTX_CNT_COVER_SPHERE,      /* Sphere#cover_area calls                                 */
  RTX_CNT_COVER_PLANE,
  RTX_CNT_COVER_BOX,
  RTX_CNT_HIGHLIGHT_TESTS,   /* per ray x light                                         */
  RTX_CNT_PRIMARY,           /* lens_func samples                                       */
  RTX_NCOUNT
};
rtx_status rtx_count_work(rtx_context* ctx, uint64_t seed, uint64_t counts[RTX_NCOUNT]);

/* Device time of the ray-tree kernel launches of the last render call on this
 * context (HIP events recorded on the launch stream around each launch; needs
 * option "kernel_events" = 1 before the call).  Waits for those events.
 * Bounce-level engine: the level launches only (k_level / k_level_c, the split
 * kernels), not the per-batch reset, re-render or tree reduction. */
rtx_status rtx_kernel_time(rtx_context* ctx, double* total_ms, int32_t* launches);

/* Bounce-level engine statistics of the last render call (summed over its
 * batches): out[0] camera samples re-rendered by the lanes engine (buffer
 * overflow), out[1] child rays that found no room, out[2 + d] rays of tree
 * level d (d = 0 .. 64).  Synchronous.  Zeros for the lanes engine. */
rtx_status rtx_level_stats(rtx_context* ctx, int64_t* out, int32_t n);

/* Kernel-variant control for experiments; 0 = default. */
rtx_status rtx_set_option(rtx_context* ctx, const char* key, int64_t value);
rtx_status rtx_get_option(rtx_context* ctx, const char* key, int64_t* value);
/* read-only key: "engine_effective" (the engine the next render of the uploaded scene and camera runs:
         "engine", except that the bounce-level engine falls back to the lanes engine for trace_depth > 64,
         monte_carlo_diffusion_times > 14 or more than 255 lights), "lv_ray_bytes_effective" (80 or 96: the
         staged ray record of the next bounce-level render), "sph_mode_effective" (where the next bounce-level
         render's walks read the spheres: 0 linear walk, records in LDS; 1 linear, scalar loads; 2 hierarchy in
         LDS; 3 hierarchy by scalar loads; 4 nodes in LDS, leaf records global; 5 hierarchy and exact records in
         LDS; 6 nodes and 16-bit leaf records in LDS).
   keys: "bvh" (0 ordered linear walk, 1 hierarchy from "bvh_min" spheres,
         2 always; every choice renders the same bits), "bvh_min" [32], "bvh_sah" (1 [default] binned-SAH hierarchy
         unless it would not fit LDS where the median one does, 0 median; at the next upload), "sphere_src" (0 LDS
         staging, 1 scalar loads, 2 hierarchy nodes in LDS and leaf records from global memory, 3 the hierarchy and
         the binary64 records of the exact sphere test in LDS, 4 the nodes and 16-bit quantized leaf records in LDS
         with 16-bit traversal stacks (2, 3 and 4: bounce-level engine; the lanes engine stages as 0; 4 falls back
         to 2 when the scene's records cannot be quantized conservatively), -1 [default] auto: 3 when that and the
         hit ring fit LDS, 0 when the hierarchy and a hit ring do, else 4 when that and the compact hit ring fit,
         else 2 when the nodes and the compact ring fit, else 0;
         every choice renders the same bits), "lds_stack" (ray-stack entries per lane kept in LDS,
         -1 = as many as fit), "force_stack" (per-lane ray-stack bucket), "postpone" (hierarchy walks
         still running in fewer lanes of a wave than this are postponed; -1 [default] = 16 from 64 nodes, 0 never), "tile_order" (1 expensive
         8x8 tiles first by a primary-hit probe, 0 row-major, -1 [default] = 1 up to 512 spheres; the order
         changes no bit), "kernel_events" (1: time the ray-tree launches, rtx_kernel_time),
         "engine" (0 persistent lanes: one camera sample's ray tree per lane; 1 [default] bounce levels: one launch
         per tree level, one ray per lane; same bits), "lv_batch" (bounce levels: camera samples per batch,
         2^24), "lv_stage_pct" / "lv_rec_pct" (bounce-level buffer capacities in % of a batch's samples,
         300 / 1600, and at least "lv_floor" staging / 4 x "lv_floor" tree records, 2^20; samples that
         overflow them are re-rendered by the lanes engine, same bits), "lv_split" (bounce levels: 0 one fused
         launch per level, 1 three launches per level over dense queues: trace, shadow, shade; same bits; used up
         to 16 lights), "lv_static" (bounce levels: % of a level launch's 64-ray chunks scheduled statically, the
         rest claimed from sharded counters; -1 [default] = 100 up to 512 spheres, else 50; same bits),
         "lv_compact" (bounce levels: 1 park the rays that hit something in a per-wave LDS ring and run the
         shadow walks and shading on full waves, 0 off, -1 [default] = on whenever the rings fit the walk's
         LDS; a hierarchy too large for the full ring next to it gets the compact ring (hit point and ids only,
         the ray re-derived); 2 = the compact ring always; same bits), "lv_streams" (bounce levels: the region's 8x8 tiles in this many interleaved parts,
         1..4, rendered at once on as many HIP streams, parts 1.. on streams the context owns; one part's level
         tails and reductions overlap the others' work; 2 [default]; same bits), "lv_grid_div" (bounce levels:
         level grids = resident workgroups / this, 1 [default]), "lv_redo_blocks" (bounce levels: at most this
         many workgroups for the lanes-engine re-render of overflowed samples, launched after every batch and
         nearly always empty; 8 [default], 0 = every resident workgroup; same bits), "lv_fin_grid" (bounce levels:
         0 [default] one tree-reduction block per 8x8 tile, k > 0 k blocks per CU looping over the tiles; measured
         neutral on C2), "lv_ray_bytes" (bounce levels: staged ray record, 80 = origin, direction, attenuation,
         {path, root} with the RNG key decoded from the root, 96 = with a 64-bit path and the key stored; 0 [default]
         = 80 whenever (monte_carlo_diffusion_times + 3)^trace_depth <= 2^32, else 96; 80 for a camera whose paths
         do not fit fails the render with RTX_EINVAL; same bits), "exact_raises" (1 [default]: every shadow walk of
         local_lights also checks the Math.acos raise of the covers it skips, spheres whose binary cover factor is 0
         (sphere.rb:45-46), so the reference's raise is reported wherever it happens: the check
         is part of the shadow walk (a kernel variant); through the light buffer, its cell's leaves get a band
         test and a per-light raise buffer built at upload lists the rest of the raise region per direction and
         target distance (device memory: C2 18 KB, C4 77 MB at 160 cells per face side, at most 128 MB); without it (or for a target nearer the light than every object surface) the hierarchy
         walk visits the boxes the light's cone meets; 0: only the covers the walk evaluates; World#high_lights'
         lit_area is checked either way; same colours),
         "lv_hl_cap" (bounce levels: entries of the batch's list of highlight rays whose lit_area raise is checked
         after the levels (k_hl_raise); 0 [default] = 1/256 of the tree-record capacity, at least 4096; a ray that
         finds it full has its sample re-rendered by the lanes engine; same bits), "lv_sort" (bounce levels, fused
         level launches: 1 = before each level >= 1 one counting-sort pass lists its rays by bin, the direction's
         octant and the origin's cell in a grid over the spheres' box (lv_sort_bits), and the level takes its 64-ray
         chunks in that order, so a wave's rays start close together and point alike; records and children are
         placed as without it; 0 off, 1 / -1 [default] on; same bits), "lv_sort_from" (the first level binned;
         0 [default] = level 1 above 512 spheres, else the last level only and only in batches of at least 2^22
         camera samples; the levels before it keep the queue order; read-only "lv_sort_effective": whether the next
         whole-frame render bins a level, "lv_sort_last": the levels per batch the last bounce-level render binned), "lv_sort_bits" (2^bits origin cells per axis of a bin, 3 or 4; 0 [default] = 4 above 512
         spheres, else 3), "lv_sort_copy" (1: the binning pass also moves the level's ray records into bin
         order, so the level reads them in runs instead of gathering them; 0 [default]: the gathers cost less
         than the copy, C4 296 -> 342 ms per frame with it; same bits), "lbuf" (bounce levels: 1 [default] = the shadow walks visit only the leaves listed in a
         per-light cube map of the spheres as seen from the light, built at upload: staged in LDS next to the hit
         rings for scenes whose sphere records are staged (sphere mode 3, up to 512 spheres), read from global
         memory beside the 16-bit leaf records of larger scenes (sphere mode 6); 0 = the hierarchy walk; same
         bits). */

/* ---- Vec3 (fast_4d_matrix.c), pure host functions ------------------------ */
rtx_vec3   rtx_vec3_from_a(double x, double y, double z);                   /* :75-84   */
double     rtx_vec3_r(rtx_vec3 a);                                          /* :275-279 */
double     rtx_vec3_r2(rtx_vec3 a);                                         /* :280-284 */
double     rtx_vec3_dot(rtx_vec3 a, rtx_vec3 b);                            /* :98-107  */
rtx_status rtx_vec3_cos(rtx_vec3 a, rtx_vec3 b, double* out);               /* :109-129 */
rtx_vec3   rtx_vec3_cross(rtx_vec3 a, rtx_vec3 b);                          /* :131-141 */
rtx_vec3   rtx_vec3_add(rtx_vec3 a, rtx_vec3 b);                            /* :166-176 */
rtx_vec3   rtx_vec3_sub(rtx_vec3 a, rtx_vec3 b);                            /* :178-188 */
rtx_vec3   rtx_vec3_mul(rtx_vec3 a, rtx_vec3 b);                            /* :190-208 */
rtx_vec3   rtx_vec3_scale(rtx_vec3 a, double s);                            /* :190-208 */
rtx_vec3   rtx_vec3_div(rtx_vec3 a, double s);                              /* :209-224 */
rtx_vec3   rtx_vec3_neg(rtx_vec3 a);                                        /* :154-164 */
rtx_vec3   rtx_vec3_pos(rtx_vec3 a);                                        /* :143-152 */
rtx_status rtx_vec3_normalize(rtx_vec3 a, rtx_vec3* out);                   /* :286-293 */
rtx_vec3   rtx_vec3_add_bang(rtx_vec3 a, rtx_vec3 b);                       /* :230-240 */
rtx_vec3   rtx_vec3_sub_bang(rtx_vec3 a, rtx_vec3 b);                       /* :242-251 */
rtx_vec3   rtx_vec3_mul_bang(rtx_vec3 a, rtx_vec3 b);                       /* :253-273 */
rtx_vec3   rtx_vec3_mul_bang_scalar(rtx_vec3 a, double s);                  /* :253-273 */

/* The counter RNG contract (DESIGN.md "RNG"): u in [0,1). */
double rtx_rand(uint64_t seed, int32_t x, int32_t y, int32_t sample, uint64_t path, int32_t draw);

#ifdef __cplusplus
}
#endif
#endif /* RTX_H */
