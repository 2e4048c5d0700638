// scene_load.hpp — World.new / Camera.new (src/world.rb:15-34,
// src/camera.rb:26-34, src/configurable_object.rb:11-49) for the CLI: YAML
// files -> the flat rtx_scene_desc / rtx_camera_desc of include/rtx.h.
// Field for field the same descriptors as raytracing_rb_amd/config.py builds
// (tests/test_cli.py compares the two), including its checks of the reference's
// raise sites (a missing property is a NoMethodError there).
#pragma once

#include <cmath>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rtx.h"
#include "png_io.hpp"
#include "yaml_lite.hpp"

namespace rtxcli {

struct ConfigError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline YNode load_yaml_file(const std::string& path) {
  const std::vector<uint8_t> d = read_file(path);
  YNode n = parse_yaml(std::string(d.begin(), d.end()));
  if (n.kind != YNode::MAP) throw ConfigError(path + ": top level must be a mapping");
  return n;
}

// hash_value_parse_vector's Vec3: a 3-element array of numbers (configurable_object.rb:16-18)
inline bool is_vec(const YNode* n) {
  if (!n || n->kind != YNode::SEQ || n->seq.size() != 3) return false;
  for (const YNode& e : n->seq)
    if (!is_num(&e)) return false;
  return true;
}

inline const YNode* need(const YNode& props, const std::string& key, const std::string& where) {
  const YNode* v = props.get(key);
  if (!v || classify(*v) == SType::Null) throw ConfigError(where + ": missing property '" + key + "'");
  return v;
}
inline void need_vec(const YNode& props, const std::string& key, const std::string& where, double out[3]) {
  const YNode* v = need(props, key, where);
  if (!is_vec(v)) throw ConfigError(where + ": '" + key + "' must be a 3-vector");
  for (int i = 0; i < 3; i++) out[i] = to_double(v->seq[i]);
}
inline double need_num(const YNode& props, const std::string& key, const std::string& where) {
  const YNode* v = need(props, key, where);
  if (!is_num(v)) throw ConfigError(where + ": '" + key + "' must be a number");
  return to_double(*v);
}
// `float(props.get(key) or dflt)`
inline double num_or(const YNode& props, const std::string& key, double dflt, const std::string& where) {
  const YNode* v = props.get(key);
  if (!truthy(v)) return dflt;
  if (!is_num(v)) throw ConfigError(where + ": '" + key + "' must be a number");
  return to_double(*v);
}

inline std::string dirname_of(const std::string& p) {
  const size_t k = p.find_last_of('/');
  return k == std::string::npos ? std::string(".") : p.substr(0, k);
}
inline bool file_exists(const std::string& p) {
  FILE* f = fopen(p.c_str(), "rb");
  if (f) fclose(f);
  return f != nullptr;
}
inline std::string norm_path(const std::string& p) {   // os.path.normpath for the forms used here
  std::vector<std::string> parts;
  const bool abs = !p.empty() && p[0] == '/';
  size_t i = 0;
  while (i <= p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    const std::string s = p.substr(i, j - i);
    if (s == "..") {
      if (!parts.empty() && parts.back() != "..") parts.pop_back();
      else if (!abs) parts.push_back(s);
    } else if (!s.empty() && s != ".") {
      parts.push_back(s);
    }
    i = j + 1;
  }
  std::string o = abs ? "/" : "";
  for (size_t k = 0; k < parts.size(); k++) o += (k ? "/" : "") + parts[k];
  return o.empty() ? "." : o;
}

// Decoded textures, deduplicated by resolved path (texture.rb:8-21).
struct TextureStore {
  std::string base_dir;
  std::map<std::string, std::string> remap;
  std::vector<std::string> paths;
  std::vector<std::vector<uint8_t>> images;
  std::vector<int> ws, hs;

  std::string resolve(std::string p) const {
    auto it = remap.find(p);
    if (it != remap.end()) p = it->second;
    if (!p.empty() && p[0] == '/') return p;
    const std::string cand = norm_path(base_dir + "/" + p);
    return file_exists(cand) ? cand : p;
  }
  int add(const std::string& p) {
    const std::string rp = resolve(p);
    for (size_t k = 0; k < paths.size(); k++)
      if (paths[k] == rp) return (int)k;
    if (!file_exists(rp)) throw ConfigError("texture file not found: " + p);
    int w, h;
    images.push_back(png_decode_rgb8(rp, w, h));
    paths.push_back(rp);
    ws.push_back(w);
    hs.push_back(h);
    return (int)paths.size() - 1;
  }
};

struct Scene {
  std::vector<rtx_object_desc> objects;
  std::vector<rtx_light_desc> lights;
  std::vector<rtx_texture_desc> tex;
  TextureStore store;
  rtx_scene_desc desc{};

  void finish() {
    tex.resize(store.images.size());
    for (size_t k = 0; k < tex.size(); k++) {
      tex[k].width = store.ws[k];
      tex[k].height = store.hs[k];
      tex[k].rgb = store.images[k].data();
    }
    desc.n_objects = (int32_t)objects.size();
    desc.n_lights = (int32_t)lights.size();
    desc.n_textures = (int32_t)tex.size();
    desc.objects = objects.data();
    desc.lights = lights.data();
    desc.textures = tex.data();
  }
};

inline std::string scalar_text(const YNode* n) { return n && n->kind == YNode::SCALAR ? n->s : std::string(); }

inline rtx_object_desc build_object(const YNode& item, int idx, TextureStore& textures) {
  const std::string kind = scalar_text(item.get("type"));
  static const YNode empty_map = [] {
    YNode m;
    m.kind = YNode::MAP;
    return m;
  }();
  const YNode* pp = item.get("properties");
  const YNode& props = pp && pp->kind == YNode::MAP ? *pp : empty_map;
  const std::string where = "world_objects[" + std::to_string(idx) + "] (" + kind + " " +
                            scalar_text(props.get("name")) + ")";
  rtx_object_desc d{};
  d.texture_id = -1;
  need_vec(props, "diffuse_rate", where, d.diffuse_rate);               // world_object.rb:71-73
  need_vec(props, "ambient", where, d.ambient);
  need_vec(props, "reflective_attenuation", where, d.reflective_attenuation);   // ray_tracer.rb:99
  const YNode* rr = props.get("refractive_rate");
  const bool rr_false = rr && classify(*rr) == SType::Bool && !truthy(rr);
  d.has_refractive_rate = rr && classify(*rr) != SType::Null && !rr_false;       // Ruby truthiness
  if (d.has_refractive_rate) d.refractive_rate = need_num(props, "refractive_rate", where);
  const YNode* ra = props.get("refractive_attenuation");
  if (ra && classify(*ra) != SType::Null) {
    need_vec(props, "refractive_attenuation", where, d.refractive_attenuation);
    d.has_refractive_attenuation = 1;
  }
  const bool tex = truthy(props.get("texture_file_path"));
  const std::string texp = scalar_text(props.get("texture_file_path"));
  if (kind == "Sphere") {
    d.type = RTX_SPHERE;
    need_vec(props, "center", where, d.center);
    d.radius = need_num(props, "radius", where);
    if (!d.has_refractive_rate) throw ConfigError(where + ": missing property 'refractive_rate'");   // sphere.rb:93
    if (!d.has_refractive_attenuation)                                                             // ray_tracer.rb:117
      throw ConfigError(where + ": missing property 'refractive_attenuation'");
    if (tex) {
      d.texture_id = textures.add(texp);
      need_vec(props, "north_pole_vec", where, d.north_pole_vec);
      need_vec(props, "greenwich_vec", where, d.greenwich_vec);
      d.texture_horizontal_scale = need_num(props, "texture_horizontal_scale", where);
      d.texture_vertical_scale = need_num(props, "texture_vertical_scale", where);
      d.texture_u_offset = num_or(props, "texture_u_offset", 0.0, where);                     // texture.rb:15-16
      d.texture_v_offset = num_or(props, "texture_v_offset", 0.0, where);
    }
  } else if (kind == "Plane") {
    d.type = RTX_PLANE;
    need_vec(props, "point", where, d.point);
    need_vec(props, "front", where, d.front);
    need_vec(props, "up", where, d.up);
    if (d.has_refractive_rate && !d.has_refractive_attenuation)
      throw ConfigError(where + ": missing property 'refractive_attenuation'");
    if (tex) {
      d.texture_id = textures.add(texp);
      d.u_unit = need_num(props, "u_unit", where);
      d.v_unit = need_num(props, "v_unit", where);
      d.texture_horizontal_scale = need_num(props, "texture_horizontal_scale", where);
      d.texture_vertical_scale = need_num(props, "texture_vertical_scale", where);
    } else {
      d.u_unit = num_or(props, "u_unit", 1.0, where);
      d.v_unit = num_or(props, "v_unit", 1.0, where);
    }
  } else if (kind == "Box") {
    d.type = RTX_BOX;
    need_vec(props, "point", where, d.point);
    need_vec(props, "front", where, d.front);
    need_vec(props, "up", where, d.up);
    d.width_front = need_num(props, "width_front", where);
    d.width_up = need_num(props, "width_up", where);
    d.width_left = need_num(props, "width_left", where);
    if (d.has_refractive_rate && !d.has_refractive_attenuation)
      throw ConfigError(where + ": missing property 'refractive_attenuation'");
    if (tex) d.texture_id = textures.add(texp);          // loaded (box.rb:17-19), never used for shading
  } else {
    throw ConfigError(where + ": unknown object type '" + kind + "' (eval of Alex::Objects::" + kind + ")");
  }
  return d;
}

inline rtx_light_desc build_light(const YNode& item, int idx, bool need_radius) {
  const std::string kind = scalar_text(item.get("type"));
  YNode empty;
  empty.kind = YNode::MAP;
  const YNode* pp = item.get("properties");
  const YNode& props = pp && pp->kind == YNode::MAP ? *pp : empty;
  const std::string where = "lights[" + std::to_string(idx) + "] (" + kind + " " + scalar_text(props.get("name")) + ")";
  if (kind != "Spot")
    throw ConfigError(where + ": unknown light type '" + kind + "' (eval of Alex::Lights::" + kind + "Light)");
  rtx_light_desc d{};
  need_vec(props, "position", where, d.position);
  need_vec(props, "color", where, d.color);
  const YNode* r = props.get("radius");
  if (!r || classify(*r) == SType::Null) {
    if (need_radius) throw ConfigError(where + ": missing property 'radius'");   // sphere.rb:34 multiplies it
    d.radius = 0.0;
  } else {
    d.radius = need_num(props, "radius", where);
  }
  d.high_light_rate = need_num(props, "high_light_rate", where);
  d.high_light_angle = need_num(props, "high_light_angle", where);
  return d;
}

inline void load_world(const std::string& path, Scene& sc, const std::map<std::string, std::string>& remap = {}) {
  const YNode cfg = load_yaml_file(path);
  char buf[4096];
  const std::string abs = realpath(path.c_str(), buf) ? std::string(buf) : path;
  sc.store.base_dir = dirname_of(abs);
  sc.store.remap = remap;
  const YNode* objs = cfg.get("world_objects");
  const YNode* lights = cfg.get("lights");
  bool has_sphere = false;
  if (objs && objs->kind == YNode::SEQ) {
    for (size_t i = 0; i < objs->seq.size(); i++) {
      const YNode& it = objs->seq[i];
      if (it.kind != YNode::MAP) continue;              // array_parse_vector drops scalars
      sc.objects.push_back(build_object(it, (int)sc.objects.size(), sc.store));
      has_sphere |= scalar_text(it.get("type")) == "Sphere";
    }
  }
  if (lights && lights->kind == YNode::SEQ)
    for (size_t i = 0; i < lights->seq.size(); i++)
      if (lights->seq[i].kind == YNode::MAP)
        sc.lights.push_back(build_light(lights->seq[i], (int)sc.lights.size(), has_sphere));
  sc.desc.max_distance = need_num(cfg, "max_distance", "world");
  sc.desc.soft_shadow_exponent = need_num(cfg, "soft_shadow_exponent", "world");
  sc.finish();
}

// camera.yml -> rtx_camera_desc (camera.rb:17-24); overrides "key=value" as the Python loader's.
inline rtx_camera_desc load_camera(const std::string& path, const std::map<std::string, double>& overrides = {}) {
  const YNode cfg = load_yaml_file(path);
  rtx_camera_desc d{};
  auto vecf = [&](const char* k, double out[3]) { need_vec(cfg, k, "camera", out); };
  auto numf = [&](const char* k) {
    auto it = overrides.find(k);
    return it != overrides.end() ? it->second : need_num(cfg, k, "camera");
  };
  auto intf = [&](const char* k) {
    const double v = numf(k);
    if (std::floor(v) != v) throw ConfigError(std::string("camera: '") + k + "' must be an integer");
    return (int32_t)v;
  };
  vecf("position", d.position);
  vecf("up", d.up);
  vecf("front", d.front);
  d.retina_width = numf("retina_width");
  d.retina_height = numf("retina_height");
  d.aperture_radius = numf("aperture_radius");
  d.image_distance = numf("image_distance");
  d.focal_distance = numf("focal_distance");
  d.variant_threshold = numf("variant_threshold");
  d.width = intf("width");
  d.height = intf("height");
  d.pre_sample_times = intf("pre_sample_times");
  d.max_sample_times = intf("max_sample_times");
  d.trace_depth = intf("trace_depth");
  d.monte_carlo_diffusion_times = intf("monte_carlo_diffusion_times");
  if (d.pre_sample_times < 1) throw ConfigError("camera: pre_sample_times must be >= 1 (camera.rb:81 divides by it)");
  if (d.width < 1 || d.height < 1) throw ConfigError("camera: width/height must be >= 1");
  return d;
}

}  // namespace rtxcli
