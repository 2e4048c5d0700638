"""rtx — the Camera#render_at -> RayTracer#trace_sync hot path of
a1exwang/raytracing_rb, rebuilt for AMD Instinct MI355X (gfx950).

The compute runs in hand-written HIP kernels (``csrc/``) behind the C-ABI
``include/rtx.h`` (``librtx.so``).  This package is the host side: YAML scene
loading (``config``), the Ruby API surface (``api``: World / Camera /
RayTracer / Ray, ``vec3``: Fast4DMatrix::Vec3), the ctypes handle
(``runtime``), frame sharding over GPUs (``tiles``) and PNG I/O (``png``).
There is no CPU fallback: without librtx.so the package cannot render.
"""

__version__ = "0.1.0"


def __getattr__(name):          # lazy: importing the package must not need a GPU
    if name in ("World", "Camera", "RayTracer", "Ray", "EPSILON"):
        from . import api
        return getattr(api, name)
    if name == "Vec3":
        from .vec3 import Vec3
        return Vec3
    raise AttributeError(name)
