"""The reference's Ruby API surface for this path, over librtx.

    world  = World("scenes/c2_world.yml")               # World.new        (src/world.rb:15)
    camera = Camera(world, "scenes/c2_camera.yml")      # Camera.new       (src/camera.rb:26)
    camera.render_sync("out.png")                        # Camera#render_sync (camera.rb:101)
    camera.render_fork("out.png", 8)                     # Camera#render_fork (camera.rb:41)
    camera.render_at(x, y)  -> {"position": [x, H-1-y], "color": [r, g, b]}   (camera.rb:70-99)
    camera.ray_tracer.trace_sync(x, y, Ray(front, position))  -> Vec3         (ray_tracer.rb:16)

Every pixel is computed by the HIP kernels through the C-ABI; there is no CPU
path.  Reference raise sites surface as ``RtxError`` (e.g. "color greater than
1", ray_tracer.rb:295).  The RNG is the counter hash of DESIGN.md §2.2, seeded
with ``seed`` (the reference seeds with ``Random.srand(1)``, main.rb:10).
"""

import os

import numpy as np

from . import config, png
from .runtime import Renderer, RtxError, quantize
from .vec3 import Vec3

EPSILON = 1e-5                      # Alex::EPSILON (src/libs/algebra.rb:2)


class Ray:
    """Alex::Ray (src/libs/algebra.rb:3-17): ``front`` is not normalized."""

    def __init__(self, front, position):
        self.front = front if isinstance(front, Vec3) else Vec3(*front)
        self.position = position if isinstance(position, Vec3) else Vec3(*position)

    def distance(self, pos):
        return (self.position - pos).r

    def __repr__(self):
        return "->%s, pos: %s" % (self.front.to_s(), self.position.to_s())


class World:
    """World.new(config_file) (src/world.rb:15-34): YAML scene -> device scene."""

    def __init__(self, config_file, texture_remap=None):
        self.config_file = config_file
        self.cfg = config.load_yaml(config_file)
        self.scene = config.SceneDescriptor(self.cfg, os.path.dirname(os.path.abspath(config_file)), texture_remap)
        self.max_distance = self.cfg.get("max_distance")
        self.soft_shadow_exponent = self.cfg.get("soft_shadow_exponent")
        self.world_objects = self.cfg.get("world_objects") or []
        self.lights = self.cfg.get("lights") or []


class RayTracer:
    """RayTracer (src/ray_tracer.rb): ``trace_sync`` of explicit rays on the GPU."""

    def __init__(self, renderer, seed=1):
        self._r = renderer
        self.seed = seed

    def trace_sync(self, x, y, ray, sample=0):
        """Sum of the ray tree's leaf colours for ``ray`` (ray_tracer.rb:16-46).
        (x, y, sample) key the path-tracing draws of the tree."""
        rays = np.array([ray.front.to_a() + ray.position.to_a()], np.float64)
        out = self._r.trace(rays, np.array([[x, y, sample]], np.int32), seed=self.seed)
        return Vec3(*out[0])

    def path_trace_sync(self, x, y, ray):
        """RayTracer#path_trace_sync (ray_tracer.rb:181-289), dead code in the
        reference: black, a highlight sum, or RtxError(kind "type") on a hit."""
        rays = np.array([ray.front.to_a() + ray.position.to_a()], np.float64)
        return Vec3(*self._r.path_trace(rays)[0])

    def trace_many(self, fronts, positions, keys):
        """Batched trace_sync: fronts/positions [n, 3], keys [n, 3] = (x, y, sample)."""
        rays = np.concatenate([np.asarray(fronts, np.float64), np.asarray(positions, np.float64)], axis=1)
        return self._r.trace(rays, keys, seed=self.seed)


class Camera:
    """Camera (src/camera.rb:15-157)."""

    def __init__(self, world, config_file=None, device=0, seed=1, **overrides):
        ccfg = config.load_yaml(config_file) if config_file else {}
        ccfg.update(overrides)
        self.cfg = ccfg
        self.world = world
        self.desc = config.build_camera(ccfg)
        self.width, self.height = self.desc.width, self.desc.height
        self.seed = seed
        self.device = device
        self._r = Renderer(world.scene, self.desc, device=device)
        self.ray_tracer = RayTracer(self._r, seed)
        self.canvas = None                                   # RGBA8 [H, W, 4] once rendered

    # -- camera.rb:70-99
    def render_at(self, x, y):
        c = self._r.render_at(x, y, seed=self.seed)
        return {"position": [x, self.height - 1 - y], "color": [float(v) for v in c]}

    def render(self, x0=0, y0=0, x1=None, y1=None):
        """Float64 framebuffer [H, W, 3], row = y (final image orientation)."""
        return self._r.render(x0, y0, x1, y1, seed=self.seed)

    # -- camera.rb:101-110 + save_image (:36-39)
    def render_sync(self, file_path=None, png_gem_blend=True):
        fb = self.render()
        self.canvas = quantize(fb, png_gem_blend=png_gem_blend)
        if file_path:
            self.save_image(file_path)
        return fb

    # -- camera.rb:41-68: N workers -> N GPUs of this node (tiles + gather)
    def render_fork(self, file_path=None, threads=None, tile_rows=8, png_gem_blend=True):
        import torch
        from . import tiles
        n = threads or max(1, torch.cuda.device_count())
        ndev = max(1, torch.cuda.device_count())
        rs = [self._r] + [Renderer(self.world.scene, self.desc, device=(k % ndev)) for k in range(1, n)]
        R = tiles.rows_per_rank(self.height, tile_rows, n)
        packed = []
        for k, r in enumerate(rs):
            dev = torch.device("cuda", r.device)
            buf = torch.zeros((R, self.width, 3), dtype=torch.float64, device=dev)
            with torch.cuda.device(dev):
                r.render_tiles_device(buf.data_ptr(), tile_rows, k, n, seed=self.seed,
                                      stream=torch.cuda.current_stream(dev).cuda_stream)
            packed.append(buf)
        for r in rs:
            r.sync()
        dev0 = torch.device("cuda", self.device)
        gathered = torch.cat([b.to(dev0) for b in packed], 0)
        fb = tiles.unpack(gathered, self.height, tile_rows, n).cpu().numpy()
        self.canvas = quantize(fb, png_gem_blend=png_gem_blend)
        if file_path:
            self.save_image(file_path)
        return fb

    def save_image(self, file_path):
        if self.canvas is None:
            raise RuntimeError("nothing rendered yet")
        png.write(file_path, self.canvas)

    @staticmethod
    def array_to_color(arr):
        """camera.rb:153-156 (without the canvas blend)."""
        return [int(min(v * 256.0, 255)) for v in arr]


__all__ = ["World", "Camera", "RayTracer", "Ray", "Vec3", "RtxError", "EPSILON"]
