// rtx_main.cpp — native counterpart of the reference's CLI, src/main.rb:
//
//   rtx s  out.png world.yml camera.yml      Camera#render_sync  (main.rb:17-18)
//   rtx N  out.png world.yml camera.yml      Camera#render_fork with N workers
//                                             (main.rb:19-21): the frame's 8-row
//                                             tiles split over N workers on the
//                                             node's GPUs (one librtx context per
//                                             worker): round-robin, or from 8
//                                             workers cost-balanced lists (LPT over
//                                             rtx_tile_probe's work map)
// options:
//   --seed S             RNG seed (main.rb:10 seeds Random with 1; default 1)
//   --device D           first GPU (default 0)
//   --set key=value      camera.yml override (e.g. --set width=64)
//   --remap old=new      texture path substitution (a missing reference texture)
//   --float-out F        also write the float64 framebuffer (H*W*3 doubles, rows top-down)
//   --no-blend           plain array_to_color bytes (no png-gem Color#blend over black)
//   --balance B          rtx N's split: rr (round-robin tiles), lpt (tile lists by the
//                        probe's costs), auto (lpt from 8 workers, the default)
//   --dump-scene         print the scene/camera descriptors as JSON and exit (no GPU)
//   --decode-png P       print W, H and an FNV-1a hash of P's RGB8 decode and exit (no GPU)
//
// YAML and PNG are parsed here in C++ (yaml_lite.hpp, png_io.hpp, zlib); every
// pixel is computed by librtx's HIP kernels through the C-ABI (include/rtx.h).
#include <chrono>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rtx.h"
#include "png_io.hpp"
#include "scene_load.hpp"

using namespace rtxcli;

namespace {

constexpr int TILE_ROWS = 8;

struct Opts {
  std::string mode, out, world, camera, float_out, decode_png;
  uint64_t seed = 1;
  int device = 0;
  bool blend = true, dump = false;
  std::string balance = "auto";
  std::map<std::string, double> set;
  std::map<std::string, std::string> remap;
  std::map<std::string, long long> opt;          // --option key=value: rtx_set_option
};

// The reference's raise sites surface as this process's error message + exit 1.
[[noreturn]] void die(const std::string& m) {
  fprintf(stderr, "rtx: %s\n", m.c_str());
  exit(1);
}

void check(rtx_context* c, rtx_status s, const char* what) {
  if (s != RTX_OK) die(std::string(what) + ": " + rtx_status_string(s) + " (" + (c ? rtx_last_error(c) : "") + ")");
}

void json_arr(FILE* f, const double* v, int n) {
  fputc('[', f);
  for (int i = 0; i < n; i++) fprintf(f, "%s%.17g", i ? ", " : "", v[i]);
  fputc(']', f);
}

void dump_scene(const Scene& sc, const rtx_camera_desc* cam) {
  FILE* f = stdout;
  fprintf(f, "{\"max_distance\": %.17g, \"soft_shadow_exponent\": %.17g, \"objects\": [", sc.desc.max_distance,
          sc.desc.soft_shadow_exponent);
  for (size_t i = 0; i < sc.objects.size(); i++) {
    const rtx_object_desc& o = sc.objects[i];
    fprintf(f, "%s{\"type\": %d, \"texture_id\": %d, \"has_refractive_rate\": %d, \"has_refractive_attenuation\": %d",
            i ? ", " : "", o.type, o.texture_id, o.has_refractive_rate, o.has_refractive_attenuation);
#define F3(name)                      \
  fprintf(f, ", \"" #name "\": ");    \
  json_arr(f, o.name, 3);
#define F1(name) fprintf(f, ", \"" #name "\": %.17g", o.name);
    F3(diffuse_rate) F3(ambient) F3(reflective_attenuation) F3(refractive_attenuation) F1(refractive_rate)
    F3(center) F1(radius) F3(north_pole_vec) F3(greenwich_vec) F1(texture_u_offset) F1(texture_v_offset)
    F3(point) F3(front) F3(up) F1(u_unit) F1(v_unit) F1(width_front) F1(width_up) F1(width_left)
    F1(texture_horizontal_scale) F1(texture_vertical_scale)
#undef F3
#undef F1
    fputc('}', f);
  }
  fprintf(f, "], \"lights\": [");
  for (size_t i = 0; i < sc.lights.size(); i++) {
    const rtx_light_desc& l = sc.lights[i];
    fprintf(f, "%s{\"position\": ", i ? ", " : "");
    json_arr(f, l.position, 3);
    fprintf(f, ", \"color\": ");
    json_arr(f, l.color, 3);
    fprintf(f, ", \"radius\": %.17g, \"high_light_rate\": %.17g, \"high_light_angle\": %.17g}", l.radius,
            l.high_light_rate, l.high_light_angle);
  }
  fprintf(f, "], \"textures\": [");
  for (size_t i = 0; i < sc.tex.size(); i++) {
    uint64_t h = 1469598103934665603ull;                 // FNV-1a of the RGB8 bytes
    const size_t n = (size_t)sc.tex[i].width * sc.tex[i].height * 3;
    for (size_t k = 0; k < n; k++) h = (h ^ sc.tex[i].rgb[k]) * 1099511628211ull;
    fprintf(f, "%s{\"width\": %d, \"height\": %d, \"fnv1a\": \"%016" PRIx64 "\"}", i ? ", " : "", sc.tex[i].width,
            sc.tex[i].height, h);
  }
  fprintf(f, "]");
  if (cam) {
    fprintf(f, ", \"camera\": {\"position\": ");
    json_arr(f, cam->position, 3);
    fprintf(f, ", \"up\": ");
    json_arr(f, cam->up, 3);
    fprintf(f, ", \"front\": ");
    json_arr(f, cam->front, 3);
    fprintf(f,
            ", \"retina_width\": %.17g, \"retina_height\": %.17g, \"aperture_radius\": %.17g, \"image_distance\": "
            "%.17g, \"focal_distance\": %.17g, \"variant_threshold\": %.17g, \"width\": %d, \"height\": %d, "
            "\"pre_sample_times\": %d, \"max_sample_times\": %d, \"trace_depth\": %d, "
            "\"monte_carlo_diffusion_times\": %d}",
            cam->retina_width, cam->retina_height, cam->aperture_radius, cam->image_distance, cam->focal_distance,
            cam->variant_threshold, cam->width, cam->height, cam->pre_sample_times, cam->max_sample_times,
            cam->trace_depth, cam->monte_carlo_diffusion_times);
  }
  fprintf(f, "}\n");
}

rtx_context* make_context(int device, const Scene& sc, const rtx_camera_desc& cam) {
  rtx_context* c = nullptr;
  if (rtx_context_create(device, &c) != RTX_OK) die("cannot create a context on GPU " + std::to_string(device));
  check(c, rtx_scene_upload(c, &sc.desc), "World.new");
  check(c, rtx_camera_set(c, &cam), "Camera.new");
  return c;
}

// Camera#render_fork (camera.rb:41-68): worker k of n renders its tiles on GPU
// (device + k) % ngpu (round-robin t % n == k, or an LPT list); the packed
// tiles are gathered to the first worker's GPU with one RCCL send/recv group
// (device copies when workers share a GPU) and the frame returned.
std::vector<double> render_fork(const Opts& o, const Scene& sc, const rtx_camera_desc& cam, int n) {
  const int W = cam.width, H = cam.height;
  const int ngpu = rtx_device_count();
  if (ngpu < 1) die("no GPU visible");
  std::vector<rtx_context*> ctx(n, nullptr);
  for (int k = 0; k < n; k++) ctx[k] = make_context((o.device + k) % ngpu, sc, cam);
  for (int k = 0; k < n; k++)
    for (const auto& kv : o.opt) check(ctx[k], rtx_set_option(ctx[k], kv.first.c_str(), kv.second), "option");
  std::vector<double> fb((size_t)W * H * 3);
  rtx_status s;
  if (o.balance == "lpt" || (o.balance == "auto" && n >= 8)) {
    // cost-balanced tile lists: the probe's work map (no render), summed per
    // 8-row tile (= one row of 8x8 tiles), longest processing time first
    const int tx = (W + 7) / 8, ty = (H + 7) / 8;
    std::vector<int64_t> probe((size_t)tx * ty), cost(ty, 0);
    check(ctx[0], rtx_tile_probe(ctx[0], probe.data(), (int32_t)probe.size()), "tile probe");
    for (int y = 0; y < ty; y++)
      for (int x = 0; x < tx; x++) cost[y] += probe[(size_t)y * tx + x];
    int32_t per = 0;
    check(ctx[0], rtx_lpt_plan(cost.data(), ty, n, nullptr, 0, &per), "lpt plan");
    std::vector<int32_t> plan((size_t)n * per);
    check(ctx[0], rtx_lpt_plan(cost.data(), ty, n, plan.data(), per, &per), "lpt plan");
    s = rtx_render_multi_plan(ctx.data(), n, TILE_ROWS, plan.data(), per, o.seed, fb.data(), (size_t)W * 3);
  } else {
    s = rtx_render_multi(ctx.data(), n, TILE_ROWS, o.seed, fb.data(), (size_t)W * 3);
  }
  if (s) die(std::string("render_fork: ") + rtx_status_string(s) + " (" + rtx_last_error(ctx[0]) + ")");
  for (rtx_context* c : ctx) rtx_context_destroy(c);
  return fb;
}

Opts parse_args(int argc, char** argv) {
  Opts o;
  std::vector<std::string> pos;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) die("missing value for " + a);
      return argv[++i];
    };
    auto kv = [&](const std::string& s, std::string& k, std::string& v) {
      const size_t e = s.find('=');
      if (e == std::string::npos) die("expected key=value after " + a);
      k = s.substr(0, e);
      v = s.substr(e + 1);
    };
    if (a == "--seed") o.seed = strtoull(val().c_str(), nullptr, 10);
    else if (a == "--device") o.device = atoi(val().c_str());
    else if (a == "--float-out") o.float_out = val();
    else if (a == "--no-blend") o.blend = false;
    else if (a == "--balance") {
      o.balance = val();
      if (o.balance != "rr" && o.balance != "lpt" && o.balance != "auto") die("--balance must be rr, lpt or auto");
    }
    else if (a == "--dump-scene") o.dump = true;
    else if (a == "--decode-png") o.decode_png = val();
    else if (a == "--set") {
      std::string k, v;
      kv(val(), k, v);
      o.set[k] = strtod(v.c_str(), nullptr);
    } else if (a == "--remap") {
      std::string k, v;
      kv(val(), k, v);
      o.remap[k] = v;
    } else if (a == "--option") {
      std::string k, v;
      kv(val(), k, v);
      o.opt[k] = strtoll(v.c_str(), nullptr, 10);
    } else pos.push_back(a);
  }
  if (!o.decode_png.empty()) return o;
  if (o.dump && (pos.size() == 1 || pos.size() == 2)) {          // --dump-scene world.yml [camera.yml]
    o.world = pos[0];
    if (pos.size() == 2) o.camera = pos[1];
    return o;
  }
  if (pos.size() != 4) {
    puts("parameter error");                                       // main.rb:5-8
    exit(1);
  }
  o.mode = pos[0];
  o.out = pos[1];
  o.world = pos[2];
  o.camera = pos[3];
  return o;
}

}  // namespace

int main(int argc, char** argv) {
  const Opts o = parse_args(argc, argv);
  try {
    if (!o.decode_png.empty()) {
      int w, h;
      const std::vector<uint8_t> img = png_decode_rgb8(o.decode_png, w, h);
      uint64_t hh = 1469598103934665603ull;
      for (uint8_t b : img) hh = (hh ^ b) * 1099511628211ull;
      printf("%d %d %016" PRIx64 "\n", w, h, hh);
      return 0;
    }
    Scene sc;
    load_world(o.world, sc, o.remap);                              // World.new (main.rb:15)
    rtx_camera_desc cam{};
    if (!o.camera.empty()) cam = load_camera(o.camera, o.set);     // Camera.new (main.rb:16)
    if (o.dump) {
      dump_scene(sc, o.camera.empty() ? nullptr : &cam);
      return 0;
    }
    const int W = cam.width, H = cam.height;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<double> fb;
    int workers = 1;
    if (o.mode == "s") {                                           // Camera#render_sync
      rtx_context* c = make_context(o.device, sc, cam);
      for (const auto& kv : o.opt) check(c, rtx_set_option(c, kv.first.c_str(), kv.second), "option");
      fb.resize((size_t)W * H * 3);
      check(c, rtx_render(c, 0, 0, W, H, o.seed, fb.data(), (size_t)W * 3), "render_sync");
      rtx_context_destroy(c);
    } else {                                                        // mode N
      workers = atoi(o.mode.c_str());                              // String#to_i (main.rb:20)
      if (workers < 1) die("worker count must be >= 1");
      fb = render_fork(o, sc, cam, workers);
    }
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<uint8_t> rgba((size_t)W * H * 4);                 // array_to_color + canvas.point
    if (rtx_quantize(fb.data(), W, H, (size_t)W * 3, o.blend ? 1 : 0, rgba.data()) != RTX_OK) die("quantize failed");
    png_write_rgba8(o.out, rgba.data(), W, H);                     // Camera#save_image
    if (!o.float_out.empty()) {
      FILE* f = fopen(o.float_out.c_str(), "wb");
      if (!f || fwrite(fb.data(), sizeof(double), fb.size(), f) != fb.size()) die("cannot write " + o.float_out);
      fclose(f);
    }
    fprintf(stderr, "rtx: %dx%d, %d sample(s)/px, depth %d, %d worker(s): %.3f s (%.2f Mpixels/s)\n", W, H,
            cam.pre_sample_times, cam.trace_depth, workers, secs, W * (double)H / secs / 1e6);
  } catch (const std::exception& e) {
    die(e.what());
  }
  return 0;
}
