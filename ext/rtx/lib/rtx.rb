# frozen_string_literal: true
#
# rtx.rb -- the Ruby side of the drop-in boundary: a Fiddle (libffi) binding of
# librtx's C-ABI (include/rtx.h), the MI355X replacement of the reference's hot
# path Camera#render_at -> RayTracer#trace_sync (src/camera.rb:70-110,
# src/ray_tracer.rb:16-164), its native Vec3 (ext/fast_4d_matrix/
# fast_4d_matrix.c:29-55) and its fork_jobs tile scheduler (src/fork_jobs.rb,
# camera.rb:41-68).  Fiddle ships with Ruby's standard library: no compiler is
# needed on the Ruby side.
#
# Kept in sync with include/rtx.h by tests/test_ruby_glue.py (struct field
# lists and every extern signature are parsed from both files and compared).
#
#   require_relative 'ext/rtx/lib/rtx'            # the binding
#   require_relative 'ext/rtx/lib/rtx/reference'  # World / Camera / RayTracer glue
require 'fiddle'
require 'fiddle/import'

module RTX
  extend Fiddle::Importer
  dlload ENV.fetch('RTX_LIB', File.expand_path('../../../raytracing_rb_amd/librtx.so', __dir__))

  ABI_VERSION = 1

  # ---- include/rtx.h structs (field order, types and array sizes = the header)
  ObjectDesc = struct [
    'int type', 'int texture_id', 'int has_refractive_rate', 'int has_refractive_attenuation',
    'double diffuse_rate[3]', 'double ambient[3]', 'double reflective_attenuation[3]',
    'double refractive_attenuation[3]', 'double refractive_rate',
    'double center[3]', 'double radius', 'double north_pole_vec[3]', 'double greenwich_vec[3]',
    'double texture_u_offset', 'double texture_v_offset',
    'double point[3]', 'double front[3]', 'double up[3]', 'double u_unit', 'double v_unit',
    'double width_front', 'double width_up', 'double width_left',
    'double texture_horizontal_scale', 'double texture_vertical_scale'
  ]
  LightDesc = struct [
    'double position[3]', 'double color[3]', 'double radius',
    'double high_light_rate', 'double high_light_angle'
  ]
  TextureDesc = struct ['int width', 'int height', 'void* rgb']
  SceneDesc = struct [
    'double max_distance', 'double soft_shadow_exponent',
    'int n_objects', 'int n_lights', 'int n_textures', 'int reserved',
    'void* objects', 'void* lights', 'void* textures'
  ]
  CameraDesc = struct [
    'double position[3]', 'double up[3]', 'double front[3]',
    'double retina_width', 'double retina_height', 'double aperture_radius',
    'double image_distance', 'double focal_distance', 'double variant_threshold',
    'int width', 'int height', 'int pre_sample_times', 'int max_sample_times',
    'int trace_depth', 'int monte_carlo_diffusion_times'
  ]

  SPHERE, PLANE, BOX = 0, 1, 2

  # ---- context
  extern 'int rtx_context_create(int, void*)'
  extern 'void rtx_context_destroy(void*)'
  extern 'char* rtx_last_error(void*)'
  extern 'char* rtx_status_string(int)'
  extern 'int rtx_abi_version()'
  extern 'char* rtx_build_id()'
  # ---- World.new / Camera.new
  extern 'int rtx_scene_upload(void*, void*)'
  extern 'int rtx_camera_set(void*, void*)'
  # ---- rendering
  extern 'int rtx_render(void*, int, int, int, int, unsigned long long, void*, size_t)'
  extern 'int rtx_render_device(void*, int, int, int, int, unsigned long long, void*, size_t, void*)'
  extern 'int rtx_tiles_rows_per_rank(int, int, int)'
  extern 'int rtx_render_tiles_device(void*, int, int, int, unsigned long long, void*, void*)'
  extern 'int rtx_render_tiles(void*, int, int, int, unsigned long long, void*)'
  extern 'int rtx_render_tile_list_device(void*, void*, int, int, unsigned long long, void*, void*)'
  extern 'int rtx_tile_rays(void*, void*, int)'
  extern 'int rtx_render_multi(void*, int, int, unsigned long long, void*, size_t)'
  extern 'int rtx_render_multi_plan(void*, int, int, void*, int, unsigned long long, void*, size_t)'
  extern 'int rtx_tile_probe(void*, void*, int)'
  extern 'int rtx_lpt_plan(void*, int, int, void*, int, void*)'
  extern 'int rtx_device_count()'
  extern 'int rtx_sync(void*, void*)'
  extern 'int rtx_render_at(void*, int, int, unsigned long long, void*)'
  extern 'int rtx_trace(void*, int, void*, void*, unsigned long long, void*)'
  extern 'int rtx_path_trace(void*, int, void*, void*)'
  extern 'int rtx_quantize(void*, int, int, size_t, int, void*)'
  extern 'int rtx_quantize_device(void*, int, int, size_t, int, void*, void*)'
  extern 'int rtx_count_work(void*, unsigned long long, void*)'
  extern 'int rtx_kernel_time(void*, void*, void*)'
  extern 'int rtx_level_stats(void*, void*, int)'
  extern 'int rtx_set_option(void*, char*, long long)'
  extern 'int rtx_get_option(void*, char*, void*)'
  extern 'double rtx_rand(unsigned long long, int, int, int, unsigned long long, int)'
  # The rtx_vec3_* functions (Fast4DMatrix::Vec3, fast_4d_matrix.c:29-55) take
  # and return rtx_vec3 BY VALUE, which Fiddle::Importer cannot pass; they are
  # not bound here.  The glue needs none of them: after it, the hot path makes
  # no Vec3 call (the whole ray tree runs on the GPU), and the configuration
  # code keeps the reference's own Fast4DMatrix extension.

  # include/rtx.h rtx_status -> the reference's raise (INTEGRATION.md §5)
  ERRORS = {
    1 => [RuntimeError, 'zero vector detected'],                     # fast_4d_matrix.c:124,291
    2 => [RuntimeError, 'color greater than 1'],                     # ray_tracer.rb:294-296
    3 => [Math::DomainError, 'Numerical argument is out of domain'], # sphere.rb:45-46, texture.rb:24-25
    4 => [RuntimeError, 'HIP runtime failure'],
    5 => [RuntimeError, 'RCCL collective failure'],
    6 => [ArgumentError, 'bad scene or camera description'],
    7 => [NoMemoryError, 'out of device memory'],
    8 => [TypeError, "nil can't be coerced into Integer"]            # ray_tracer.rb:167
  }.freeze

  class Error < StandardError
    attr_reader :status

    def initialize(status, message)
      @status = status
      super(message)
    end
  end

  def self.check(ctx, status)
    return if status.zero?

    klass, text = ERRORS.fetch(status, [RuntimeError, 'rtx error'])
    detail = ctx ? rtx_last_error(ctx).to_s : ''
    # the reference raises these classes itself; keep them rescuable as such
    raise klass, "#{text} (#{detail})" unless klass == RuntimeError

    raise Error.new(status, "#{text} (#{detail})")
  end

  # One librtx context on device `device` (World.new + Camera.new uploaded).
  class Context
    attr_reader :ptr

    def initialize(device = 0)
      holder = Fiddle::Pointer.malloc(Fiddle::SIZEOF_VOIDP)
      RTX.check(nil, RTX.rtx_context_create(device, holder))
      @ptr = holder.ptr
      @keep = []
    end

    def upload_scene(scene_desc, keep)
      @keep = keep                          # descriptor memory stays alive with the context
      RTX.check(@ptr, RTX.rtx_scene_upload(@ptr, scene_desc))
    end

    def set_camera(camera_desc)
      RTX.check(@ptr, RTX.rtx_camera_set(@ptr, camera_desc))
    end

    def set_option(key, value)
      RTX.check(@ptr, RTX.rtx_set_option(@ptr, key.to_s, value))
    end

    def destroy
      RTX.rtx_context_destroy(@ptr) if @ptr
      @ptr = nil
    end
  end

  # Host buffer of n doubles.
  def self.doubles(n)
    Fiddle::Pointer.malloc(8 * n)
  end
end
