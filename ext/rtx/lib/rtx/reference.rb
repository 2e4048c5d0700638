# frozen_string_literal: true
#
# rtx/reference.rb -- the glue a maintainer of a1exwang/raytracing_rb adds so
# that the reference's own World / Camera / RayTracer run their hot path on
# librtx (the MI355X HIP path) instead of in Ruby.  It is prepended to the
# reference classes; their constructors, YAML loading (ConfigurableObject,
# src/configurable_object.rb:43-49) and signatures stay as they are.
#
#   require_relative 'src/camera'; require_relative 'src/world'
#   require_relative 'ext/rtx/lib/rtx/reference'
#   world  = Alex::World.new('config/world.yml')
#   camera = Alex::Camera.new(world, 'config/camera.yml')
#   camera.render_sync('out.png')        # one rtx_render call, no per-pixel Ruby
#   camera.render_fork('out.png', 8)     # rtx_render_multi over the node's GPUs
#
# Replaced, file:line of the reference:
#   Camera#render_sync   src/camera.rb:101-110   -> rtx_render + rtx_quantize
#   Camera#render_fork   src/camera.rb:41-68,    -> rtx_render_multi (8-row tiles
#                        src/fork_jobs.rb:1-33       round-robin, one RCCL gather)
#   Camera#render_at     src/camera.rb:70-99     -> rtx_render_at
#   RayTracer#trace_sync src/ray_tracer.rb:16-46 -> rtx_trace
#   RayTracer#path_trace_sync src/ray_tracer.rb:181-195 -> rtx_path_trace
# Random.rand becomes the counter RNG keyed by (seed, x, y, sample, path, draw)
# (DESIGN.md §2.3); main.rb:10's Random.srand(1) becomes seed 1.
require_relative '../rtx'

module RTX
  # World#upload (src/world.rb:15-34): one ObjectDesc per @world_objects entry
  # and one LightDesc per @lights entry, in YAML order (the first object wins
  # distance ties, world.rb:48-50); textures decoded once by the reference's
  # own Texture (texture.rb:17-20, bytes = pixel >> 8).
  module WorldGlue
    def rtx_scene_desc
      objs = instance_variable_get(:@world_objects)
      lights = instance_variable_get(:@lights)
      tex_index = {}
      tex_bufs = []
      obj_buf = Fiddle::Pointer.malloc([1, objs.size].max * ObjectDesc.size)
      objs.each_with_index do |o, i|
        d = ObjectDesc.malloc
        RTX.fill_object(d, o, tex_index, tex_bufs)
        obj_buf[i * ObjectDesc.size, ObjectDesc.size] = d.to_ptr[0, ObjectDesc.size]
      end
      light_buf = Fiddle::Pointer.malloc([1, lights.size].max * LightDesc.size)
      lights.each_with_index do |l, i|
        d = LightDesc.malloc
        d.position = l.position.to_a
        d.color = l.color.to_a
        d.radius = (l.radius || 0.0).to_f      # sphere.rb:36 needs it only with spheres
        d.high_light_rate = l.high_light_rate.to_f
        d.high_light_angle = l.high_light_angle.to_f
        light_buf[i * LightDesc.size, LightDesc.size] = d.to_ptr[0, LightDesc.size]
      end
      tex_buf = Fiddle::Pointer.malloc([1, tex_bufs.size].max * TextureDesc.size)
      tex_bufs.each_with_index do |(w, h, rgb), i|
        d = TextureDesc.malloc
        d.width = w
        d.height = h
        d.rgb = rgb
        tex_buf[i * TextureDesc.size, TextureDesc.size] = d.to_ptr[0, TextureDesc.size]
      end
      s = SceneDesc.malloc
      s.max_distance = max_distance.to_f
      s.soft_shadow_exponent = soft_shadow_exponent.to_f
      s.n_objects = objs.size
      s.n_lights = lights.size
      s.n_textures = tex_bufs.size
      s.reserved = 0
      s.objects = obj_buf
      s.lights = light_buf
      s.textures = tex_buf
      [s, [obj_buf, light_buf, tex_buf, tex_bufs]]
    end
  end

  def self.iv(o, name)
    o.instance_variable_get("@#{name}")
  end

  def self.vec(o, name)
    v = iv(o, name)
    v ? v.to_a.map(&:to_f) : [0.0, 0.0, 0.0]
  end

  # One world object -> rtx_object_desc (the properties the reference reads:
  # world_object.rb, sphere.rb, plane.rb, box.rb).
  def self.fill_object(d, o, tex_index, tex_bufs)
    d.type = case o
             when Alex::Objects::Sphere then SPHERE
             when Alex::Objects::Box then BOX
             when Alex::Objects::Plane then PLANE
             else raise ArgumentError, "unknown world object #{o.class}"
             end
    d.diffuse_rate = vec(o, :diffuse_rate)
    d.ambient = vec(o, :ambient)
    d.reflective_attenuation = vec(o, :reflective_attenuation)
    rr = iv(o, :refractive_rate)
    d.has_refractive_rate = rr ? 1 : 0          # Ruby truthiness (plane.rb:57)
    d.refractive_rate = rr ? rr.to_f : 0.0
    ra = iv(o, :refractive_attenuation)
    d.has_refractive_attenuation = ra ? 1 : 0
    d.refractive_attenuation = ra ? ra.to_a : [0.0, 0.0, 0.0]
    d.texture_id = -1
    path = iv(o, :texture_file_path)
    if path
      d.texture_id = tex_index[path] ||= begin
        t = o.texture                             # Alex::Texture, already decoded
        rgb = t.to_a.flat_map { |row| row.flat_map { |c| c.to_a.map { |v| (v * 256.0).round } } }
        tex_bufs << [t.width, t.height, Fiddle::Pointer[rgb.pack('C*')]]
        tex_bufs.size - 1
      end
      d.texture_horizontal_scale = iv(o, :texture_horizontal_scale).to_f
      d.texture_vertical_scale = iv(o, :texture_vertical_scale).to_f
    end
    case d.type
    when SPHERE
      d.center = vec(o, :center)
      d.radius = iv(o, :radius).to_f
      if path
        d.north_pole_vec = vec(o, :north_pole_vec)
        d.greenwich_vec = vec(o, :greenwich_vec)
        d.texture_u_offset = (iv(o, :texture_u_offset) || 0.0).to_f   # texture.rb:15-16
        d.texture_v_offset = (iv(o, :texture_v_offset) || 0.0).to_f
      end
    when PLANE
      d.point = vec(o, :point)
      d.front = vec(o, :front)
      d.up = vec(o, :up)
      d.u_unit = (iv(o, :u_unit) || 1.0).to_f
      d.v_unit = (iv(o, :v_unit) || 1.0).to_f
    when BOX
      d.point = vec(o, :point)
      d.front = vec(o, :front)
      d.up = vec(o, :up)
      d.width_front = iv(o, :width_front).to_f
      d.width_up = iv(o, :width_up).to_f
      d.width_left = iv(o, :width_left).to_f
    end
  end

  # camera.yml -> rtx_camera_desc (camera.rb:17-24)
  def self.camera_desc(cam)
    d = CameraDesc.malloc
    d.position = cam.position.to_a
    d.up = cam.up.to_a
    d.front = cam.front.to_a
    d.retina_width = cam.retina_width.to_f
    d.retina_height = cam.retina_height.to_f
    d.aperture_radius = cam.aperture_radius.to_f
    d.image_distance = cam.image_distance.to_f
    d.focal_distance = cam.focal_distance.to_f
    d.variant_threshold = cam.variant_threshold.to_f
    d.width = cam.width
    d.height = cam.height
    d.pre_sample_times = cam.pre_sample_times
    d.max_sample_times = cam.max_sample_times
    d.trace_depth = cam.trace_depth
    d.monte_carlo_diffusion_times = cam.monte_carlo_diffusion_times
    d
  end

  module CameraGlue
    TILE_ROWS = 8

    def initialize(world, config_file)
      super
      @rtx_seed = 1                                 # main.rb:10 Random.srand(1)
      @rtx_ctx = rtx_context(0)
      @ray_tracer.rtx_bind(@rtx_ctx, @rtx_seed)
    end

    def rtx_context(device)
      ctx = Context.new(device)
      desc, keep = @world.rtx_scene_desc
      ctx.upload_scene(desc, keep)
      ctx.set_camera(RTX.camera_desc(self))
      ctx
    end

    # Camera#render_at (camera.rb:70-99): pre samples, the variance test, the
    # extra samples, on the GPU; same return value.
    def render_at(x, y)
      rgb = RTX.doubles(3)
      RTX.check(@rtx_ctx.ptr, RTX.rtx_render_at(@rtx_ctx.ptr, x, y, @rtx_seed, rgb))
      { position: [x, @height - 1 - y], color: rgb[0, 24].unpack('d3') }
    end

    # Camera#render_sync (camera.rb:101-110): the whole frame in one call.
    def render_sync(file_path)
      buf = RTX.doubles(@width * @height * 3)
      RTX.check(@rtx_ctx.ptr, RTX.rtx_render(@rtx_ctx.ptr, 0, 0, @width, @height, @rtx_seed, buf, @width * 3))
      rtx_paint(buf)
      save_image(file_path)
    end

    # Camera#render_fork (camera.rb:41-68 + fork_jobs.rb): `threads` workers,
    # one librtx context each, on device k % rtx_device_count(); the frame in
    # 8-row tiles dealt round-robin, ONE RCCL gather to the first device.
    def render_fork(file_path, threads)
      ndev = [RTX.rtx_device_count, 1].max
      ctxs = Array.new(threads) { |k| rtx_context(k % ndev) }
      list = Fiddle::Pointer[ctxs.map { |c| c.ptr.to_i }.pack('Q*')]
      buf = RTX.doubles(@width * @height * 3)
      begin
        RTX.check(ctxs[0].ptr, RTX.rtx_render_multi(list, threads, TILE_ROWS, @rtx_seed, buf, @width * 3))
      ensure
        ctxs.each(&:destroy)
      end
      rtx_paint(buf)
      save_image(file_path)
    end

    private

    # array_to_color (camera.rb:153-156) on the GPU's quantizer, then the
    # reference's own canvas.point (the png gem blends over its black canvas)
    def rtx_paint(buf)
      rgba = Fiddle::Pointer.malloc(@width * @height * 4)
      RTX.check(nil, RTX.rtx_quantize(buf, @width, @height, @width * 3, 0, rgba))
      bytes = rgba[0, @width * @height * 4].unpack('C*')
      @width.times do |x|
        @height.times do |y|
          o = 4 * (y * @width + x)
          @canvas.point(x, @height - 1 - y, PNG::Color.new(bytes[o], bytes[o + 1], bytes[o + 2]))
        end
      end
    end
  end

  module RayTracerGlue
    def rtx_bind(ctx, seed)
      @rtx_ctx = ctx
      @rtx_seed = seed
    end

    # RayTracer#trace_sync (ray_tracer.rb:16-46); the RNG key is (x, y, sample 0)
    def trace_sync(x, y, ray)
      rays = [*ray.front.to_a, *ray.position.to_a].pack('d6')
      keys = [x, y, 0].pack('l3')
      out = RTX.doubles(3)
      RTX.check(@rtx_ctx.ptr, RTX.rtx_trace(@rtx_ctx.ptr, 1, rays, keys, @rtx_seed, out))
      Vec3.from_a(*out[0, 24].unpack('d3'))
    end

    # RayTracer#path_trace_sync (ray_tracer.rb:181-195), dead code in the
    # reference: raises TypeError on any hit, as roulette_random does
    def path_trace_sync(_x, _y, ray)
      out = RTX.doubles(3)
      rays = [*ray.front.to_a, *ray.position.to_a].pack('d6')
      RTX.check(@rtx_ctx.ptr, RTX.rtx_path_trace(@rtx_ctx.ptr, 1, rays, out))
      Vec3.from_a(*out[0, 24].unpack('d3'))
    end
  end
end

Alex::World.prepend(RTX::WorldGlue)
Alex::Camera.prepend(RTX::CameraGlue)
Alex::RayTracer.prepend(RTX::RayTracerGlue)
