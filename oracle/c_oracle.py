"""ctypes front-end of the C oracle (``rt_oracle.c``) — TEST INFRASTRUCTURE ONLY.

Takes the same flat descriptors the product consumes (``include/rtx.h``),
built by ``raytracing_rb_amd.config`` (the tests then independently check that
loader against ``rt_ref.load_scene``).
"""

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "librt_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        from raytracing_rb_amd._abi import CameraDesc, SceneDesc
        L = C.CDLL(LIB)
        L.rto_create.restype = C.c_void_p
        L.rto_create.argtypes = [C.POINTER(SceneDesc), C.POINTER(CameraDesc), C.c_char_p, C.c_size_t]
        L.rto_destroy.argtypes = [C.c_void_p]
        L.rto_last_error.restype = C.c_char_p
        L.rto_last_error.argtypes = [C.c_void_p]
        L.rto_render.restype = C.c_int
        L.rto_render.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64,
                                 C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
        L.rto_render_pixels.restype = C.c_int
        L.rto_render_pixels.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_uint64, C.c_void_p,
                                        C.c_void_p, C.c_void_p]
        L.rto_trace.restype = C.c_int
        L.rto_trace.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                C.c_void_p]
        L.rto_lens.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_void_p]
        L.rto_render_fork.restype = C.c_int
        L.rto_render_fork.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_uint64, C.c_void_p]
        L.rto_rand.restype = C.c_double
        L.rto_rand.argtypes = [C.c_uint64, C.c_int32, C.c_int32, C.c_int32, C.c_uint64, C.c_int32]
        _lib = L
    return _lib


class Oracle:
    def __init__(self, scene, camera):
        """scene: raytracing_rb_amd.config.SceneDescriptor; camera: CameraDesc."""
        self._scene = scene           # keep the descriptor arrays alive
        self.camera = camera
        err = C.create_string_buffer(256)
        self.h = lib().rto_create(C.byref(scene.desc), C.byref(camera), err, 256)
        if not self.h:
            raise ValueError(err.value.decode())

    def __del__(self):
        if getattr(self, "h", None):
            lib().rto_destroy(self.h)
            self.h = None

    def render(self, x0=0, y0=0, x1=None, y1=None, seed=1, counts=False):
        x1 = self.camera.width if x1 is None else x1
        y1 = self.camera.height if y1 is None else y1
        out = np.zeros((y1 - y0, x1 - x0, 3), np.float64)
        st = np.zeros((y1 - y0, x1 - x0), np.int32)
        cnt = np.zeros(16, np.uint64)
        rc = lib().rto_render(self.h, x0, y0, x1, y1, seed, out.ctypes.data, (x1 - x0) * 3,
                              st.ctypes.data, cnt.ctypes.data)
        if counts:
            return out, st, rc, cnt
        return out, st, rc

    def render_pixels(self, xy, seed=1, counts=False):
        xy = np.ascontiguousarray(xy, np.int32).reshape(-1, 2)
        out = np.zeros((len(xy), 3), np.float64)
        st = np.zeros(len(xy), np.int32)
        cnt = np.zeros(16, np.uint64)
        rc = lib().rto_render_pixels(self.h, len(xy), xy.ctypes.data, seed, out.ctypes.data,
                                     st.ctypes.data, cnt.ctypes.data)
        if counts:
            return out, st, rc, cnt
        return out, st, rc

    def trace(self, rays, keys, seed=1):
        rays = np.ascontiguousarray(rays, np.float64).reshape(-1, 6)
        keys = np.ascontiguousarray(keys, np.int32).reshape(-1, 3)
        out = np.zeros((len(rays), 3), np.float64)
        st = np.zeros(len(rays), np.int32)
        rc = lib().rto_trace(self.h, len(rays), rays.ctypes.data, keys.ctypes.data, seed,
                             out.ctypes.data, st.ctypes.data)
        return out, st, rc

    def lens(self, x, y, j, seed=1):
        r = np.zeros(6, np.float64)
        lib().rto_lens(self.h, x, y, j, seed, r.ctypes.data)
        return r

    def render_fork(self, nprocs, col_stride=1, seed=1):
        out = np.zeros((self.camera.height, self.camera.width, 3), np.float64)
        rc = lib().rto_render_fork(self.h, nprocs, col_stride, seed, out.ctypes.data)
        if rc:
            raise RuntimeError("rto_render_fork failed: %d" % rc)
        return out

    def last_error(self):
        return lib().rto_last_error(self.h).decode()
