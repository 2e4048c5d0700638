"""ctypes mirror of ``include/rtx.h`` and the loader of ``librtx.so``.

The library is the product: if it is missing or fails to load this module
raises — there is no CPU fallback anywhere in ``raytracing_rb_amd``.
"""

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RTX_LIB", os.path.join(_HERE, "librtx.so"))

RTX_OK, RTX_EZERO_VEC, RTX_ECOLOR_GT1, RTX_EDOMAIN, RTX_EHIP, RTX_ERCCL, RTX_EINVAL, RTX_ENOMEM = range(8)
RTX_SPHERE, RTX_PLANE, RTX_BOX = 0, 1, 2
COUNTER_NAMES = ["rays", "sphere_tests", "sphere_hits", "plane_tests", "box_tests", "shade_hits",
                 "cover_sphere", "cover_plane", "cover_box", "highlight_tests", "primary"]
RTX_NCOUNT = len(COUNTER_NAMES)

D3 = C.c_double * 3


class ObjectDesc(C.Structure):
    _fields_ = [
        ("type", C.c_int32), ("texture_id", C.c_int32),
        ("has_refractive_rate", C.c_int32), ("has_refractive_attenuation", C.c_int32),
        ("diffuse_rate", D3), ("ambient", D3), ("reflective_attenuation", D3),
        ("refractive_attenuation", D3), ("refractive_rate", C.c_double),
        ("center", D3), ("radius", C.c_double), ("north_pole_vec", D3), ("greenwich_vec", D3),
        ("texture_u_offset", C.c_double), ("texture_v_offset", C.c_double),
        ("point", D3), ("front", D3), ("up", D3), ("u_unit", C.c_double), ("v_unit", C.c_double),
        ("width_front", C.c_double), ("width_up", C.c_double), ("width_left", C.c_double),
        ("texture_horizontal_scale", C.c_double), ("texture_vertical_scale", C.c_double),
    ]


class LightDesc(C.Structure):
    _fields_ = [("position", D3), ("color", D3), ("radius", C.c_double),
                ("high_light_rate", C.c_double), ("high_light_angle", C.c_double)]


class TextureDesc(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("rgb", C.POINTER(C.c_uint8))]


class SceneDesc(C.Structure):
    _fields_ = [("max_distance", C.c_double), ("soft_shadow_exponent", C.c_double),
                ("n_objects", C.c_int32), ("n_lights", C.c_int32), ("n_textures", C.c_int32),
                ("reserved", C.c_int32),
                ("objects", C.POINTER(ObjectDesc)), ("lights", C.POINTER(LightDesc)),
                ("textures", C.POINTER(TextureDesc))]


class CameraDesc(C.Structure):
    _fields_ = [("position", D3), ("up", D3), ("front", D3),
                ("retina_width", C.c_double), ("retina_height", C.c_double),
                ("aperture_radius", C.c_double), ("image_distance", C.c_double),
                ("focal_distance", C.c_double), ("variant_threshold", C.c_double),
                ("width", C.c_int32), ("height", C.c_int32),
                ("pre_sample_times", C.c_int32), ("max_sample_times", C.c_int32),
                ("trace_depth", C.c_int32), ("monte_carlo_diffusion_times", C.c_int32)]


class Vec3T(C.Structure):
    _fields_ = [("v", D3), ("r", C.c_double)]


# (name, restype, argtypes) of every symbol include/rtx.h declares.
_P = C.c_void_p
_I = C.c_int32
_D = C.c_double
_U64 = C.c_uint64
_SZ = C.c_size_t
_DP = C.POINTER(C.c_double)
SIGNATURES = [
    ("rtx_context_create", _I, [_I, C.POINTER(_P)]),
    ("rtx_context_destroy", None, [_P]),
    ("rtx_last_error", C.c_char_p, [_P]),
    ("rtx_status_string", C.c_char_p, [_I]),
    ("rtx_abi_version", _I, []),
    ("rtx_build_id", C.c_char_p, []),
    ("rtx_scene_upload", _I, [_P, C.POINTER(SceneDesc)]),
    ("rtx_camera_set", _I, [_P, C.POINTER(CameraDesc)]),
    ("rtx_render", _I, [_P, _I, _I, _I, _I, _U64, _DP, _SZ]),
    ("rtx_render_device", _I, [_P, _I, _I, _I, _I, _U64, _P, _SZ, _P]),
    ("rtx_tiles_rows_per_rank", _I, [_I, _I, _I]),
    ("rtx_render_tiles_device", _I, [_P, _I, _I, _I, _U64, _P, _P]),
    ("rtx_render_tiles", _I, [_P, _I, _I, _I, _U64, _DP]),
    ("rtx_render_tile_list_device", _I, [_P, C.POINTER(C.c_int32), _I, _I, _U64, _P, _P]),
    ("rtx_tile_rays", _I, [_P, C.POINTER(C.c_int64), _I]),
    ("rtx_render_multi", _I, [C.POINTER(_P), _I, _I, _U64, _DP, _SZ]),
    ("rtx_render_multi_plan", _I, [C.POINTER(_P), _I, _I, C.POINTER(C.c_int32), _I, _U64, _DP, _SZ]),
    ("rtx_tile_probe", _I, [_P, C.POINTER(C.c_int64), _I]),
    ("rtx_lpt_plan", _I, [C.POINTER(C.c_int64), _I, _I, C.POINTER(C.c_int32), _I, C.POINTER(C.c_int32)]),
    ("rtx_device_count", _I, []),
    ("rtx_sync", _I, [_P, _P]),
    ("rtx_render_at", _I, [_P, _I, _I, _U64, _DP]),
    ("rtx_trace", _I, [_P, _I, _DP, C.POINTER(C.c_int32), _U64, _DP]),
    ("rtx_path_trace", _I, [_P, _I, _DP, _DP]),
    ("rtx_quantize", _I, [_DP, _I, _I, _SZ, _I, C.POINTER(C.c_uint8)]),
    ("rtx_quantize_device", _I, [_P, _I, _I, _SZ, _I, _P, _P]),
    ("rtx_count_work", _I, [_P, _U64, C.POINTER(C.c_uint64)]),
    ("rtx_set_option", _I, [_P, C.c_char_p, C.c_int64]),
    ("rtx_get_option", _I, [_P, C.c_char_p, C.POINTER(C.c_int64)]),
    ("rtx_level_stats", _I, [_P, C.POINTER(C.c_int64), _I]),
    ("rtx_kernel_time", _I, [_P, _DP, C.POINTER(C.c_int32)]),
    ("rtx_vec3_from_a", Vec3T, [_D, _D, _D]),
    ("rtx_vec3_r", _D, [Vec3T]),
    ("rtx_vec3_r2", _D, [Vec3T]),
    ("rtx_vec3_dot", _D, [Vec3T, Vec3T]),
    ("rtx_vec3_cos", _I, [Vec3T, Vec3T, _DP]),
    ("rtx_vec3_cross", Vec3T, [Vec3T, Vec3T]),
    ("rtx_vec3_add", Vec3T, [Vec3T, Vec3T]),
    ("rtx_vec3_sub", Vec3T, [Vec3T, Vec3T]),
    ("rtx_vec3_mul", Vec3T, [Vec3T, Vec3T]),
    ("rtx_vec3_scale", Vec3T, [Vec3T, _D]),
    ("rtx_vec3_div", Vec3T, [Vec3T, _D]),
    ("rtx_vec3_neg", Vec3T, [Vec3T]),
    ("rtx_vec3_pos", Vec3T, [Vec3T]),
    ("rtx_vec3_normalize", _I, [Vec3T, C.POINTER(Vec3T)]),
    ("rtx_vec3_add_bang", Vec3T, [Vec3T, Vec3T]),
    ("rtx_vec3_sub_bang", Vec3T, [Vec3T, Vec3T]),
    ("rtx_vec3_mul_bang", Vec3T, [Vec3T, Vec3T]),
    ("rtx_vec3_mul_bang_scalar", Vec3T, [Vec3T, _D]),
    ("rtx_rand", _D, [_U64, _I, _I, _I, _U64, _I]),
]

_lib = None


class RtxLibraryMissing(RuntimeError):
    pass


def load_library(path=None):
    """Load librtx.so (built by ``__graft_entry__.build()``) or raise."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RtxLibraryMissing(
            "librtx.so not found at %s — build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback)" % p)
    lib = C.CDLL(p)
    in_tree = p == os.path.join(_HERE, "librtx.so")
    for name, res, args in SIGNATURES:
        if not in_tree and not hasattr(lib, name):
            continue                  # an older diagnostic build (tools/variants.py): what it exports
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rtx_abi_version() != 1:
        raise RtxLibraryMissing("librtx ABI version mismatch")
    if p == os.path.join(_HERE, "librtx.so"):
        # the in-tree library must be the build of the sources beside it: a
        # stale binary would be tested and benchmarked in place of the code
        from . import _build
        built, tree = lib.rtx_build_id().decode(), _build.source_sha()
        if built != tree:
            raise RtxLibraryMissing(
                "stale librtx.so: built from sources %s, the tree holds %s — rebuild with "
                "`python -c 'import __graft_entry__ as g; g.build()'`" % (built, tree))
    if path is None:
        _lib = lib
    return lib
