"""Thin Python handle over librtx (``include/rtx.h``).

``Renderer`` owns one ``rtx_context`` (one HIP device) with an uploaded scene
and camera.  Host-buffer calls are synchronous; ``*_device`` calls take raw
device pointers (e.g. ``torch.Tensor.data_ptr()``) and a HIP stream handle and
return immediately.  Errors raise ``RtxError`` carrying the reference's raise
site (``rtx_status``).  There is no CPU fallback: without librtx.so nothing here
works.
"""

import ctypes as C

import numpy as np

from . import _abi
from ._abi import RTX_NCOUNT, COUNTER_NAMES, load_library


class RtxError(RuntimeError):
    KINDS = {1: "zero_vec", 2: "color_gt1", 3: "domain", 4: "hip", 5: "rccl", 6: "invalid", 7: "nomem",
             8: "type"}

    def __init__(self, status, msg):
        super().__init__("%s (rtx_status %d)" % (msg, status))
        self.status = status
        self.kind = self.KINDS.get(status, "unknown")


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class Renderer:
    def __init__(self, scene, camera, device=0):
        """scene: config.SceneDescriptor; camera: _abi.CameraDesc."""
        self.lib = load_library()
        self.h = C.c_void_p()
        st = self.lib.rtx_context_create(device, C.byref(self.h))
        if st:
            raise RtxError(st, "rtx_context_create failed")
        self.device = device
        self._scene = scene
        self.camera = camera
        self._check(self.lib.rtx_scene_upload(self.h, C.byref(scene.desc)))
        self._check(self.lib.rtx_camera_set(self.h, C.byref(camera)))

    # ------------------------------------------------------------ plumbing
    def _check(self, st):
        if st:
            raise RtxError(st, self.lib.rtx_last_error(self.h).decode())

    def close(self):
        if self.h:
            self.lib.rtx_context_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def width(self):
        return self.camera.width

    @property
    def height(self):
        return self.camera.height

    def set_camera(self, camera):
        self.camera = camera
        self._check(self.lib.rtx_camera_set(self.h, C.byref(camera)))

    def set_option(self, key, value):
        self._check(self.lib.rtx_set_option(self.h, key.encode(), int(value)))

    # ------------------------------------------------------------ host API
    def render(self, x0=0, y0=0, x1=None, y1=None, seed=1):
        """Float64 framebuffer [y1-y0, x1-x0, 3] (row = y, top first)."""
        x1 = self.width if x1 is None else x1
        y1 = self.height if y1 is None else y1
        out = np.empty((y1 - y0, x1 - x0, 3), np.float64)
        self._check(self.lib.rtx_render(self.h, x0, y0, x1, y1, seed, _dp(out), (x1 - x0) * 3))
        return out

    def render_at(self, x, y, seed=1):
        out = np.empty(3, np.float64)
        self._check(self.lib.rtx_render_at(self.h, x, y, seed, _dp(out)))
        return out

    def trace(self, rays, keys, seed=1):
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
        keys = np.ascontiguousarray(keys, np.int32).reshape(-1, 3)
        out = np.empty((len(rays), 3), np.float64)
        self._check(self.lib.rtx_trace(self.h, len(rays), _dp(rays),
                                       keys.ctypes.data_as(C.POINTER(C.c_int32)), seed, _dp(out)))
        return out

    def path_trace(self, rays):
        """RayTracer#path_trace_sync for rays [n, 6] = (front, position) -> [n, 3]."""
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
        out = np.empty((len(rays), 3), np.float64)
        self._check(self.lib.rtx_path_trace(self.h, len(rays), _dp(rays), _dp(out)))
        return out

    def count_work(self, seed=1):
        cnt = (C.c_uint64 * RTX_NCOUNT)()
        self._check(self.lib.rtx_count_work(self.h, seed, cnt))
        return dict(zip(COUNTER_NAMES, [int(v) for v in cnt]))

    # ------------------------------------------------------------ device API
    def render_device(self, d_out, seed=1, x0=0, y0=0, x1=None, y1=None, row_stride=None, stream=None):
        x1 = self.width if x1 is None else x1
        y1 = self.height if y1 is None else y1
        row_stride = (x1 - x0) * 3 if row_stride is None else row_stride
        self._check(self.lib.rtx_render_device(self.h, x0, y0, x1, y1, seed, C.c_void_p(d_out), row_stride,
                                               C.c_void_p(stream or 0)))

    def rows_per_rank(self, tile_rows, nranks):
        return self.lib.rtx_tiles_rows_per_rank(self.height, tile_rows, nranks)

    def render_tiles_device(self, d_packed, tile_rows, rank, nranks, seed=1, stream=None):
        self._check(self.lib.rtx_render_tiles_device(self.h, tile_rows, rank, nranks, seed, C.c_void_p(d_packed),
                                                     C.c_void_p(stream or 0)))

    def render_tile_list_device(self, d_packed, tiles, tile_rows, seed=1, stream=None):
        """The tile_rows-row tiles `tiles` (image tile indices; past the bottom: padding)
        into packed rows k * tile_rows (rtx_render_tile_list_device)."""
        t = np.ascontiguousarray(tiles, np.int32)
        self._check(self.lib.rtx_render_tile_list_device(self.h, t.ctypes.data_as(C.POINTER(C.c_int32)), len(t),
                                                         tile_rows, seed, C.c_void_p(d_packed),
                                                         C.c_void_p(stream or 0)))

    def tile_probe(self):
        """Probe weights per 8x8 tile [ceil(H/8), ceil(W/8)] without rendering (rtx_tile_probe)."""
        tx, ty = (self.width + 7) // 8, (self.height + 7) // 8
        out = np.zeros(tx * ty, np.int64)
        self._check(self.lib.rtx_tile_probe(self.h, out.ctypes.data_as(C.POINTER(C.c_int64)), len(out)))
        return out.reshape(ty, tx)

    def tile_rays(self):
        """Rays per 8x8 tile [ceil(H/8), ceil(W/8)] of the last whole-frame level render (rtx_tile_rays)."""
        ty, tx = (self.height + 7) // 8, (self.width + 7) // 8
        out = np.zeros(ty * tx, np.int64)
        self._check(self.lib.rtx_tile_rays(self.h, out.ctypes.data_as(C.POINTER(C.c_int64)), len(out)))
        return out.reshape(ty, tx)

    def get_option(self, key):
        v = C.c_int64()
        self._check(self.lib.rtx_get_option(self.h, key.encode(), C.byref(v)))
        return v.value

    ENGINES = {0: "lanes", 1: "levels"}

    def engine(self):
        """Name of the ray-tree engine the next render of this scene and camera
        runs (read-only option "engine_effective": "engine", except that the
        bounce-level engine hands cameras it cannot take to the lanes engine)."""
        return self.ENGINES[self.get_option("engine_effective")]

    def level_stats(self):
        """Bounce-level engine statistics of the last render call: {"redo", "dropped", "rays": [per level]}."""
        n = 2 + 65
        out = (C.c_int64 * n)()
        self._check(self.lib.rtx_level_stats(self.h, out, n))
        rays = list(out[2:])
        while rays and rays[-1] == 0:
            rays.pop()
        return {"redo": out[0], "dropped": out[1], "rays": rays}

    def kernel_time(self):
        """(total ms, launches) of the ray-tree kernel launches of the last render
        call (HIP events on the launch stream; needs set_option("kernel_events", 1))."""
        ms = C.c_double()
        n = C.c_int32()
        self._check(self.lib.rtx_kernel_time(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def sync(self, stream=None):
        self._check(self.lib.rtx_sync(self.h, C.c_void_p(stream or 0)))

    def quantize_device(self, d_rgb, d_rgba, png_gem_blend=True, stream=None, width=None, height=None):
        w = self.width if width is None else width
        h = self.height if height is None else height
        st = self.lib.rtx_quantize_device(C.c_void_p(d_rgb), w, h, w * 3, int(png_gem_blend), C.c_void_p(d_rgba),
                                          C.c_void_p(stream or 0))
        if st:
            raise RtxError(st, "rtx_quantize_device failed")


def render_multi(renderers, tile_rows=8, seed=1):
    """Camera#render_fork over several contexts in one process (rtx_render_multi):
    renderer k renders rank k's tiles on its device, ONE RCCL gather to the first
    renderer's device.  Returns the float64 frame [H, W, 3]."""
    if not renderers:
        raise ValueError("no renderers")
    lib = load_library()
    r0 = renderers[0]
    hs = (C.c_void_p * len(renderers))(*[r.h.value for r in renderers])
    out = np.empty((r0.height, r0.width, 3), np.float64)
    st = lib.rtx_render_multi(hs, len(renderers), tile_rows, seed, _dp(out), r0.width * 3)
    if st:
        raise RtxError(st, lib.rtx_last_error(r0.h).decode())
    return out


def render_multi_plan(renderers, plan, tile_rows=8, seed=1):
    """render_multi with explicit tile lists (rtx_render_multi_plan): plan[k] is
    renderer k's list of tile_rows-row tiles (equal lengths, padded past the
    bottom, e.g. tiles.lpt_plan).  Returns the float64 frame [H, W, 3]."""
    if not renderers or len(plan) != len(renderers):
        raise ValueError("one tile list per renderer")
    lib = load_library()
    r0 = renderers[0]
    per = len(plan[0])
    flat = np.ascontiguousarray(np.asarray(plan, np.int32).reshape(-1))
    hs = (C.c_void_p * len(renderers))(*[r.h.value for r in renderers])
    out = np.empty((r0.height, r0.width, 3), np.float64)
    st = lib.rtx_render_multi_plan(hs, len(renderers), tile_rows, flat.ctypes.data_as(C.POINTER(C.c_int32)), per,
                                   seed, _dp(out), r0.width * 3)
    if st:
        raise RtxError(st, lib.rtx_last_error(r0.h).decode())
    return out


def lpt_plan_native(costs, nranks):
    """rtx_lpt_plan (host C++): the same plan as tiles.lpt_plan."""
    lib = load_library()
    c = np.ascontiguousarray(np.asarray(costs, np.int64))
    per = C.c_int32(0)
    st = lib.rtx_lpt_plan(c.ctypes.data_as(C.POINTER(C.c_int64)), len(c), nranks, None, 0, C.byref(per))
    if st:
        raise RtxError(st, "rtx_lpt_plan failed")
    out = np.zeros(nranks * per.value, np.int32)
    st = lib.rtx_lpt_plan(c.ctypes.data_as(C.POINTER(C.c_int64)), len(c), nranks,
                          out.ctypes.data_as(C.POINTER(C.c_int32)), per.value, C.byref(per))
    if st:
        raise RtxError(st, "rtx_lpt_plan failed")
    return [list(map(int, out[k * per.value:(k + 1) * per.value])) for k in range(nranks)]


def device_count():
    return load_library().rtx_device_count()


def quantize(rgb, png_gem_blend=True):
    """array_to_color + canvas point (camera.rb:105,153-156) on the GPU -> RGBA8 [H, W, 4]."""
    lib = load_library()
    rgb = np.ascontiguousarray(rgb, np.float64)
    h, w, _ = rgb.shape
    out = np.empty((h, w, 4), np.uint8)
    st = lib.rtx_quantize(_dp(rgb), w, h, w * 3, int(png_gem_blend), out.ctypes.data_as(C.POINTER(C.c_uint8)))
    if st:
        raise RtxError(st, "rtx_quantize failed")
    return out


def vec3_lib():
    return load_library()


__all__ = ["Renderer", "RtxError", "quantize", "render_multi", "render_multi_plan", "lpt_plan_native", "device_count",
           "_abi"]
