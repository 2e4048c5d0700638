// rtx_scene.h — device-resident scene layout of librtx (host + device).
//
// The YAML scene of World.new (src/world.rb:15-34) flattened into two tiers:
//   * hot  : ObjInfo[n] + a flat double array of per-object geometry, read by
//            every lane in the same order (uniform index => scalar loads /
//            LDS broadcast), YAML order preserved (first object wins ties,
//            world.rb:48-50; cover areas are subtracted in that order,
//            world.rb:64-67);
//   * cold : Material[n], lights, textures — touched once per shaded hit.
// Every derived constant (normalized axes, box faces, ...) is computed on the
// host with the reference's operation order (rtx_capi.cpp), so the device sees
// bit-identical values to what the Ruby code recomputes on every call.
#pragma once
#include <stdint.h>

namespace rtx {

enum : int32_t { OBJ_SPHERE = 0, OBJ_PLANE = 1, OBJ_BOX = 2 };

// Geometry records (offsets in doubles into SceneDev::geo).
//   sphere : [0..2] C, [3] R, [4] R*R (cull only), [5] |C|_1 + R (cull scale)
//   plane  : [0..2] P, [3..5] F, [6..8] left.normalize, [9..11] up.normalize, [12] u_unit, [13] v_unit
//   box    : 6 faces x 14 doubles (plane layout), face order of box.rb:62-67
constexpr int SPHERE_GEO = 6;
constexpr int PLANE_GEO = 14;
constexpr int BOX_GEO = 6 * PLANE_GEO;

struct ObjInfo {
  int32_t type;
  int32_t geo;      // offset into geo[]
  int32_t pad0, pad1;
};

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
  int32_t tex;            // -1 = none (ignored for boxes, box.rb never shades with it)
  int32_t face_rr_pad0, face_rr_pad1;
};

struct LightDev {
  double pos[3];
  double color[3];
  double radius;
  double hl_rate;
  double hl_angle_rad;    // high_light_angle / 180.0 * PI (world.rb:91)
  double cos_lo2, cos_hi2;// squared |cos| decision band around cos(angle): exact acos only inside
  int32_t hl_mode;        // 0: band test valid, 1: always evaluate acos, 2: never fires
  int32_t pad;
};

struct TexDev {
  int32_t w, h;
  int64_t off;            // byte offset of RGB8 texels in SceneDev::texels
};

struct SceneDev {
  const ObjInfo* info;
  const double* geo;
  const Material* mat;
  const LightDev* light;
  const TexDev* tex;
  const uint8_t* texels;
  int32_t n_obj, n_light, n_sphere, n_plane, n_box, n_geo;
  double max_distance;
  double sse;             // soft_shadow_exponent
  int32_t sse_is_two;     // pow(area, 2.0) == area*area fast path
  int32_t pad;
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
