"""YAML scene/camera configuration -> flat C-ABI descriptors.

Mirrors ``Alex::ConfigurableObject`` (``src/configurable_object.rb:11-49``):
YAML is loaded, every 3-number array becomes a float Vec3, other scalars are
kept, top-level keys become attributes.  ``World#parse_objects`` /
``#parse_lights`` (``src/world.rb:21-34``) turn the ``type:`` strings into
Sphere / Plane / Box objects and SpotLights, in YAML order (the order matters:
the first object wins distance ties).

Required properties are validated here and raise ``ConfigError`` where the
reference would crash later with NoMethodError/TypeError on a ``nil``
(e.g. a sphere without ``refractive_rate``: ``sphere.rb:93-94``).
"""

import ctypes as C
import os
import re

import numpy as np
import yaml

from . import png
from ._abi import (RTX_BOX, RTX_PLANE, RTX_SPHERE, CameraDesc, LightDesc, ObjectDesc, SceneDesc,
                   TextureDesc)


class ConfigError(ValueError):
    pass


class _Loader(getattr(yaml, "CSafeLoader", yaml.SafeLoader)):
    """YAML 1.1 as Psych reads it: ``1e-5`` is a Float (PyYAML needs a '.').
    libyaml's parser when present (same documents, ~6x faster on C4's 2 MB)."""


_Loader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(r"^[-+]?(?:[0-9][0-9_]*)(?:\.[0-9_]*)?[eE][-+]?[0-9]+$"),
    list("-+0123456789"))


def _is_num(v):
    return isinstance(v, (int, float)) and not isinstance(v, bool)


def _vec_or(v):
    if isinstance(v, list) and len(v) == 3 and all(_is_num(e) for e in v):
        return tuple(float(e) for e in v)
    return None


def parse_vectors(node):
    """hash_value_parse_vector / array_parse_vector (configurable_object.rb:11-41)."""
    if isinstance(node, dict):
        out = {}
        for k, v in node.items():
            vec = _vec_or(v)
            if isinstance(v, dict):
                out[str(k)] = parse_vectors(v)
            elif vec is not None:
                out[str(k)] = vec
            elif isinstance(v, list):
                out[str(k)] = parse_vectors(v)
            else:
                out[str(k)] = v
        return out
    if isinstance(node, list):
        out = []
        for v in node:
            vec = _vec_or(v)
            if isinstance(v, dict):
                out.append(parse_vectors(v))
            elif vec is not None:
                out.append(vec)
            elif isinstance(v, list):
                out.append(parse_vectors(v))
            # scalars inside arrays are dropped, as array_parse_vector does
        return out
    return node


def load_yaml(path):
    with open(path) as f:
        cfg = yaml.load(f, Loader=_Loader)
    if not isinstance(cfg, dict):
        raise ConfigError("%s: top level must be a mapping" % path)
    return parse_vectors(cfg)


# ------------------------------------------------------------------ textures
class TextureStore:
    """Decoded textures, deduplicated by resolved path (texture.rb:8-21)."""

    def __init__(self, base_dir, remap=None):
        self.base_dir = base_dir
        self.remap = dict(remap or {})
        self.paths = []
        self.images = []

    def resolve(self, p):
        p = self.remap.get(p, p)
        if os.path.isabs(p):
            return p
        cand = os.path.normpath(os.path.join(self.base_dir, p))
        return cand if os.path.exists(cand) else p

    def add(self, p):
        rp = self.resolve(p)
        if rp in self.paths:
            return self.paths.index(rp)
        if not os.path.exists(rp):
            raise ConfigError("texture file not found: %s" % p)
        self.paths.append(rp)
        self.images.append(np.ascontiguousarray(png.decode_rgb8(rp)))
        return len(self.paths) - 1


# ------------------------------------------------------------------ scene
def _need(props, key, where, vec=False):
    if key not in props or props[key] is None:
        raise ConfigError("%s: missing property '%s'" % (where, key))
    v = props[key]
    if vec:
        if not (isinstance(v, tuple) and len(v) == 3):
            raise ConfigError("%s: '%s' must be a 3-vector" % (where, key))
    elif not _is_num(v):
        raise ConfigError("%s: '%s' must be a number" % (where, key))
    return v


def _set3(dst, v):
    for i in range(3):
        dst[i] = float(v[i])


def build_object(item, idx, textures):
    kind = item.get("type")
    props = item.get("properties") or {}
    where = "world_objects[%d] (%s %s)" % (idx, kind, props.get("name", ""))
    d = ObjectDesc()
    d.texture_id = -1
    _set3(d.diffuse_rate, _need(props, "diffuse_rate", where, True))          # world_object.rb:71-73
    _set3(d.ambient, _need(props, "ambient", where, True))
    _set3(d.reflective_attenuation, _need(props, "reflective_attenuation", where, True))  # ray_tracer.rb:99
    rr = props.get("refractive_rate")
    d.has_refractive_rate = int(rr is not None and rr is not False)           # Ruby truthiness
    if d.has_refractive_rate:
        d.refractive_rate = float(_need(props, "refractive_rate", where))
    ra = props.get("refractive_attenuation")
    if ra is not None:
        _set3(d.refractive_attenuation, _need(props, "refractive_attenuation", where, True))
        d.has_refractive_attenuation = 1
    tex = props.get("texture_file_path")
    if kind == "Sphere":
        d.type = RTX_SPHERE
        _set3(d.center, _need(props, "center", where, True))
        d.radius = float(_need(props, "radius", where))
        if not d.has_refractive_rate:          # sphere.rb:93-94 always divides by it
            raise ConfigError("%s: missing property 'refractive_rate'" % where)
        if not d.has_refractive_attenuation:  # ray_tracer.rb:117
            raise ConfigError("%s: missing property 'refractive_attenuation'" % where)
        if tex:
            d.texture_id = textures.add(tex)
            _set3(d.north_pole_vec, _need(props, "north_pole_vec", where, True))
            _set3(d.greenwich_vec, _need(props, "greenwich_vec", where, True))
            d.texture_horizontal_scale = float(_need(props, "texture_horizontal_scale", where))
            d.texture_vertical_scale = float(_need(props, "texture_vertical_scale", where))
            d.texture_u_offset = float(props.get("texture_u_offset") or 0.0)   # texture.rb:15-16
            d.texture_v_offset = float(props.get("texture_v_offset") or 0.0)
    elif kind == "Plane":
        d.type = RTX_PLANE
        _set3(d.point, _need(props, "point", where, True))
        _set3(d.front, _need(props, "front", where, True))
        _set3(d.up, _need(props, "up", where, True))
        if d.has_refractive_rate and not d.has_refractive_attenuation:
            raise ConfigError("%s: missing property 'refractive_attenuation'" % where)
        if tex:
            d.texture_id = textures.add(tex)
            d.u_unit = float(_need(props, "u_unit", where))
            d.v_unit = float(_need(props, "v_unit", where))
            d.texture_horizontal_scale = float(_need(props, "texture_horizontal_scale", where))
            d.texture_vertical_scale = float(_need(props, "texture_vertical_scale", where))
        else:
            d.u_unit = float(props.get("u_unit") or 1.0)
            d.v_unit = float(props.get("v_unit") or 1.0)
    elif kind == "Box":
        d.type = RTX_BOX
        _set3(d.point, _need(props, "point", where, True))
        _set3(d.front, _need(props, "front", where, True))
        _set3(d.up, _need(props, "up", where, True))
        d.width_front = float(_need(props, "width_front", where))
        d.width_up = float(_need(props, "width_up", where))
        d.width_left = float(_need(props, "width_left", where))
        if d.has_refractive_rate and not d.has_refractive_attenuation:
            raise ConfigError("%s: missing property 'refractive_attenuation'" % where)
        if tex:   # loaded (box.rb:17-19) but never used for shading
            d.texture_id = textures.add(tex)
    else:
        raise ConfigError("%s: unknown object type %r (eval of Alex::Objects::%s)" % (where, kind, kind))
    return d


def build_light(item, idx, need_radius):
    kind = item.get("type")
    props = item.get("properties") or {}
    where = "lights[%d] (%s %s)" % (idx, kind, props.get("name", ""))
    if kind != "Spot":
        raise ConfigError("%s: unknown light type %r (eval of Alex::Lights::%sLight)" % (where, kind, kind))
    d = LightDesc()
    _set3(d.position, _need(props, "position", where, True))
    _set3(d.color, _need(props, "color", where, True))
    if props.get("radius") is None:
        if need_radius:     # sphere.rb:36 multiplies light_radius
            raise ConfigError("%s: missing property 'radius'" % where)
        d.radius = 0.0
    else:
        d.radius = float(_need(props, "radius", where))
    d.high_light_rate = float(_need(props, "high_light_rate", where))
    d.high_light_angle = float(_need(props, "high_light_angle", where))
    return d


class SceneDescriptor:
    """Owns the ctypes arrays behind an ``rtx_scene_desc``."""

    def __init__(self, world_cfg, base_dir, remap=None):
        self.cfg = world_cfg
        self.textures = TextureStore(base_dir, remap)
        objs = world_cfg.get("world_objects") or []
        lights = world_cfg.get("lights") or []
        self.objects = (ObjectDesc * max(1, len(objs)))()
        for i, it in enumerate(objs):
            self.objects[i] = build_object(it, i, self.textures)
        has_sphere = any((it.get("type") == "Sphere") for it in objs)
        self.lights = (LightDesc * max(1, len(lights)))()
        for i, it in enumerate(lights):
            self.lights[i] = build_light(it, i, has_sphere)
        self.tex_arrays = [np.ascontiguousarray(im, dtype=np.uint8) for im in self.textures.images]
        self.tex_descs = (TextureDesc * max(1, len(self.tex_arrays)))()
        for i, a in enumerate(self.tex_arrays):
            self.tex_descs[i].height, self.tex_descs[i].width = a.shape[0], a.shape[1]
            self.tex_descs[i].rgb = a.ctypes.data_as(C.POINTER(C.c_uint8))
        self.desc = SceneDesc()
        self.desc.max_distance = float(_need(world_cfg, "max_distance", "world"))
        self.desc.soft_shadow_exponent = float(_need(world_cfg, "soft_shadow_exponent", "world"))
        self.desc.n_objects = len(objs)
        self.desc.n_lights = len(lights)
        self.desc.n_textures = len(self.tex_arrays)
        self.desc.objects = C.cast(self.objects, C.POINTER(ObjectDesc))
        self.desc.lights = C.cast(self.lights, C.POINTER(LightDesc))
        self.desc.textures = C.cast(self.tex_descs, C.POINTER(TextureDesc))
        self.n_objects = len(objs)


CAMERA_KEYS_VEC = ("position", "up", "front")
CAMERA_KEYS_F = ("retina_width", "retina_height", "aperture_radius", "image_distance", "focal_distance",
                 "variant_threshold")
CAMERA_KEYS_I = ("width", "height", "pre_sample_times", "max_sample_times", "trace_depth",
                 "monte_carlo_diffusion_times")


def build_camera(cfg):
    """camera.yml -> rtx_camera_desc (camera.rb:17-24)."""
    d = CameraDesc()
    for k in CAMERA_KEYS_VEC:
        _set3(getattr(d, k), _need(cfg, k, "camera", True))
    for k in CAMERA_KEYS_F:
        setattr(d, k, float(_need(cfg, k, "camera")))
    for k in CAMERA_KEYS_I:
        v = _need(cfg, k, "camera")
        if int(v) != v:
            raise ConfigError("camera: '%s' must be an integer" % k)
        setattr(d, k, int(v))
    if d.pre_sample_times < 1:
        raise ConfigError("camera: pre_sample_times must be >= 1 (camera.rb:81 divides by it)")
    if d.width < 1 or d.height < 1:
        raise ConfigError("camera: width/height must be >= 1")
    return d


def load_scene(world_yml, camera_yml=None, camera_overrides=None, remap=None):
    """World.new(world_yml) + Camera.new(world, camera_yml) as descriptors."""
    wcfg = load_yaml(world_yml)
    scene = SceneDescriptor(wcfg, os.path.dirname(os.path.abspath(world_yml)), remap)
    cam = None
    if camera_yml is not None or camera_overrides:
        ccfg = load_yaml(camera_yml) if camera_yml is not None else {}
        ccfg.update(camera_overrides or {})
        cam = build_camera(ccfg)
    return scene, cam
