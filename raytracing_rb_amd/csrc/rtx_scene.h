// rtx_scene.h — device-resident scene layout of librtx (host + device).
//
// The YAML scene of World.new (src/world.rb:15-34) flattened for the GPU:
//   * runs   : maximal runs of consecutive objects of one type, in YAML order.
//              Every object loop walks the runs in order, so the reference's
//              order semantics hold exactly (first object wins distance ties,
//              world.rb:48-50; cover areas subtracted in order, world.rb:64-67).
//   * spheres: a binary64 record for the exact Sphere#intersect and a float32
//              record {cx, cy, cz, R} for the conservative pre-test, staged in
//              LDS by every workgroup (16 B per sphere).
//   * planes / box faces: binary64 records.
//   * Material[n_obj], lights, textures — read once per shaded hit.
// Every derived constant (normalized axes, box faces, ...) is computed on the
// host with the reference's operation order (rtx_capi.cpp), so the device sees
// bit-identical values to what the Ruby code recomputes on every call.
#pragma once
#include <stdint.h>

namespace rtx {

enum : int32_t { OBJ_SPHERE = 0, OBJ_PLANE = 1, OBJ_BOX = 2 };

// Plane record (doubles): [0..2] P, [3..5] F, [6..8] left.normalize,
// [9..11] up.normalize, [12] u_unit, [13] v_unit.  A box = 6 plane records
// in the face order of box.rb:62-67.
constexpr int PLANE_GEO = 14;
constexpr int BOX_GEO = 6 * PLANE_GEO;

struct Run {
  int32_t type;
  int32_t obj0;     // global (YAML) index of the run's first object
  int32_t count;
  int32_t rec0;     // index of the first record in the type's array
};

struct Sphere64 {
  double c[3];
  double r;
};

// Four-wide bounding-box hierarchy over the spheres (built on the host,
// rtx_capi.cpp).  A node holds the float32 axis-aligned boxes of its (up to)
// four children; every child box contains every sphere below it exactly
// (bounds rounded outwards), so a float32 slab test of the box dilated by the
// margin of DESIGN.md §2.1 that misses proves the exact binary64 test of every
// sphere below it returns nil (or, for a shadow query, a zero cover).
//   child[k] >= 0        : internal node index
//   child[k] == BVH_NONE : empty slot
//   child[k] <  0        : leaf, ~child = leaf << 2 | (count - 1); its `count`
//                          (1..4) spheres sit in slots 4*leaf .. 4*leaf+count-1
//                          of the slot arrays (float32 pre-test record, binary64
//                          record, global object index); unused slots are padding.
// Nodes are in pre-order (root = 0).  Each lane traverses on its own, nearest
// child first; the traversal order never matters for the result: nearest hits
// compare (distance, object index) lexicographically and shadow covers are
// subtracted in object order (rtx_kernels.hip).
constexpr int BVH_LEAF = 4;
constexpr float CULL_M = 2e-5f;            // pre-test margin (exact culls)
constexpr int32_t BVH_NONE = 0x7fffffff;
constexpr int COVER_K = 4;        // per-lane ordered shadow-cover list (LDS); more -> ordered re-walk
constexpr size_t LBUF_MAX_WORDS = 8192;   // light buffer, all lights: at most 16 KB (staged in LDS next to the hit ring)
constexpr size_t LBUF_MAX_WORDS_GLOBAL = 1 << 18;   // scenes above 512 spheres: at most 512 KB, read from global memory
constexpr size_t RBUF_MAX_WORDS = 1 << 21;          // raise buffer, all lights: at most 8 MB (global memory, L2 / MALL)
constexpr size_t RBUF_MAX_WORDS_GLOBAL = 1 << 25;   // (scenes above 512 spheres, per-sphere lists: at most 128 MB)
constexpr uint32_t GATE_UNIT = 2;                    // raise-buffer gates: q units per 5-bit field (rtx_bvh_build.h gate_word)
// The raise buffer's per-light block: the floor, the entry count and 3 (6 n^2 + 1)
// list offsets, then the entries from this word on (a multiple of 4: every list
// starts 16-byte aligned, so a query reads four entries with one load).
constexpr size_t rbuf_head(int cells) { return (2 + 3 * ((size_t)cells + 1) + 3) & ~(size_t)3; }
struct Bvh4Node {
  float lh[3][4][2];      // [axis][child] = {lo, hi}: both slab planes of an axis in one 8-byte pair
                          // (one packed FP32 FMA, v_pk_fma_f32, gives both slab distances)
  int32_t child[4];
};
static_assert(sizeof(Bvh4Node) == 112, "Bvh4Node layout");

struct Material {
  double diffuse[3];
  double ambient[3];
  double refl_att[3];
  double refr_att[3];
  double rr;              // refractive_rate
  double hs, vs;          // texture scales
  double u_off, v_off;    // sphere texture offsets
  double gw_n[3], east_n[3], north_n[3];   // sphere texture axes (normalized)
  int32_t has_rr;         // Ruby truthiness of refractive_rate
  int32_t tex;            // -1 = none (boxes never shade with theirs, box.rb)
  int32_t type;
  int32_t rec;            // index into the type's record array
};

static_assert(sizeof(Material) % 16 == 0, "Material staged in LDS as float4");

struct LightDev {
  double pos[3];
  double color[3];
  double radius;
  double hl_rate;
  double hl_angle_rad;    // high_light_angle / 180.0 * PI (world.rb:91)
  double cos_lo2, cos_hi2;// squared |cos| decision band around cos(angle): exact acos only inside
  int32_t hl_mode;        // 0: band test valid, 1: always evaluate acos, 2: never fires
  float raise_f2;         // the raise buffer's floor^2 (rounded up) and log2 floor^2 (rtx_device.h raise_qa;
  float raise_lf2;        //  0 without a raise buffer)
  int32_t pad;
};

struct TexDev {
  int32_t w, h;
  int64_t off;            // byte offset of RGB8 texels in SceneDev::texels
};

struct SceneDev {
  const Run* runs;
  const Sphere64* sph64;
  const float* sph32;     // 4 floats per sphere: cx, cy, cz, R
  const double* planes;   // PLANE_GEO doubles per plane
  const double* boxes;    // BOX_GEO doubles per box
  const Material* mat;
  const Bvh4Node* bvh;    // n_nodes nodes, root = 0
  const float* bvh_sph32; // 16 floats per leaf (4 slots): {cx 0..3}, {cy 0..3}, {cz 0..3}, {R^2 0..3}
  const Sphere64* bvh_sph64; // binary64 record per slot
  const uint32_t* bvh_q;  // 8 words per leaf: 16-bit quantized pre-test records {x 0..3}, {y}, {z}, {r} (SPH_BVH_QLDS)
  const int32_t* bvh_obj; // slot -> global (YAML) object index (-1 = padding)
  const int32_t* sph_obj; // sphere record -> global (YAML) object index
  const LightDev* light;
  const TexDev* tex;
  const uint8_t* texels;
  int32_t n_obj, n_light, n_sphere, n_plane, n_box, n_runs;
  int32_t n_nodes, n_slots;
  int32_t bvh_root;       // root reference (BVH_NONE: no spheres)
  int32_t bvh_stack;      // per-lane traversal stack entries the hierarchy can need
  double max_distance;
  double sse;             // soft_shadow_exponent
  float sph_scale;        // max over spheres of |C|_1 + R (pre-test margin scale)
  int32_t sse_is_two;     // pow(area, 2.0) == area*area (glibc, checked)
  // bvh_q decoding: center axis a = fmaf(q, q_step[a], q_org[a]), radius = q * q_rstep
  // (>= R + the center's decoding error); q_ok: the records are conservative
  // for the pre-test and every reference fits a 16-bit traversal stack
  float q_org[3], q_step[3], q_rstep;
  int32_t q_ok;
  float q_err;            // bound on |decoded - true| of a 16-bit record's center and radius (exact_raises' band)
  // box of every sphere (float32, rounded outwards): center and half extents (exact_raises' cone bound)
  float root_c[3], root_h[3];
  // light buffer (null when not built): per light lbuf_stride
  // uint16 words, 6 lbuf_n^2 + 1 cell offsets, then the cells' leaf references
  const uint16_t* lbuf;
  int32_t lbuf_n, lbuf_stride;
  // raise buffer (rtx_bvh_build.h build_raise_buffer; null when
  // not built): per light rbuf_stride words (floor, count, 3 (6 rbuf_n^2 + 1)
  // offsets, entries); per light rgate_stride 16-bit gate words: the floor
  // (float bits), 6 words of padding, one word per raise-buffer cell
  // (raise_gates); lbuf_n is a multiple of rbuf_n
  const uint32_t* rbuf;
  const uint16_t* rgate;
  int32_t rbuf_n, rbuf_stride, rgate_stride;
  int32_t rbuf_sphere;    // 1: the lists' entries name sphere slots (larger scenes), 0: leaves
  float rbuf_inv_m;       // rbuf_n / lbuf_n: a light-buffer cell index i has its parent at (int)((i + 0.5) * this)
};

struct CameraDev {
  double pos[3];
  double left[3];          // up.cross(front).normalize          (camera.rb:130)
  double left_n[3];        // left.normalize                      (camera.rb:136)
  double up_n[3];          // up.normalize                        (camera.rb:134,136)
  double front[3];
  double retina_center[3]; // position - front.normalize * image_distance (camera.rb:131)
  double pofp[3];          // position + front.normalize * object_distance (camera.rb:142)
  double retina_width, retina_height, aperture_radius;
  double variant_threshold;
  int32_t width, height, pre, max_samples, depth, pt;
};

}  // namespace rtx
