"""The native CLI (raytracing_rb_amd/rtx, the src/main.rb counterpart): its C++
YAML loader and PNG decoder against the Python host layer's, on every committed
scene and on YAML edge cases; its GPU render against the Python API (gpu)."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REFERENCE, ROOT, SCENES

CLI = os.path.join(ROOT, "raytracing_rb_amd", "rtx")


@pytest.fixture(scope="module")
def cli():
    """The binary __graft_entry__.build() makes (relinked here only if stale: g++, seconds)."""
    from raytracing_rb_amd import _build
    assert os.path.exists(_build.OUT), "librtx.so missing: run __graft_entry__.build()"
    return _build.build_cli()


def _fnv1a(b):
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return "%016x" % h


def _py_dump(world, camera=None, remap=None):
    from raytracing_rb_amd import config
    sd, cd = config.load_scene(world, camera, remap=remap)
    objs = []
    for i in range(sd.n_objects):
        o = sd.objects[i]
        d = {k: getattr(o, k) for k, _ in o._fields_}
        objs.append({k: (list(v) if not isinstance(v, (int, float)) else v) for k, v in d.items()})
    lights = []
    for i in range(sd.desc.n_lights):
        l = sd.lights[i]
        lights.append({k: (list(getattr(l, k)) if k in ("position", "color") else getattr(l, k)) for k, _ in l._fields_})
    tex = [{"width": a.shape[1], "height": a.shape[0], "fnv1a": _fnv1a(a.tobytes())} for a in sd.tex_arrays]
    out = {"max_distance": sd.desc.max_distance, "soft_shadow_exponent": sd.desc.soft_shadow_exponent,
           "objects": objs, "lights": lights, "textures": tex}
    if cd is not None:
        out["camera"] = {k: (list(getattr(cd, k)) if k in ("position", "up", "front") else getattr(cd, k))
                         for k, _ in cd._fields_}
    return out


def _cli_dump(cli, world, camera=None, remap=()):
    args = [cli, "--dump-scene", world] + ([camera] if camera else [])
    for k, v in remap:
        args += ["--remap", "%s=%s" % (k, v)]
    r = subprocess.run(args, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout)


@pytest.mark.parametrize("world,camera", [("c0_world.yml", "camera.yml"), ("c1_world.yml", "c1_camera.yml"),
                                          ("c2_world.yml", "c2_camera.yml"), ("mix_world.yml", "mix_camera.yml"),
                                          ("c4_world.yml", "c4_camera.yml")])
def test_cli_loader_matches_python_loader(cli, world, camera):
    if world == "c4_world.yml":
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import make_scenes
        make_scenes.ensure_c4()
    w, c = os.path.join(SCENES, world), os.path.join(SCENES, camera)
    assert _cli_dump(cli, w, c) == _py_dump(w, c)


@pytest.mark.skipif(not os.path.exists(os.path.join(REFERENCE, "config", "world.yml")),
                    reason="reference checkout not present (GPU box)")
def test_cli_loads_reference_config(cli):
    """The reference's own config/world.yml + camera.yml (duplicate keys, '-' on its
    own line); its missing floor.jpg remapped to our checker, RubyOnRails.png to its
    copy in scenes/textures."""
    remap = {"./textures/floor.jpg": os.path.join(SCENES, "textures", "checker.png"),
             "./textures/RubyOnRails.png": os.path.join(SCENES, "textures", "RubyOnRails.png")}
    w, c = os.path.join(REFERENCE, "config", "world.yml"), os.path.join(REFERENCE, "config", "camera.yml")
    assert _cli_dump(cli, w, c, remap.items()) == _py_dump(w, c, remap)


EDGE = """# comment line
max_distance: 1e4          # a float without a dot (Psych reads it as Float)
soft_shadow_exponent: 2
lights:
- type: Spot               # sequence at the key's own column
  properties:
    name: 'quoted # not a comment'
    position: [5, -4, 0.9]
    color: [1, 1, 1]
    radius: .5
    high_light_rate: 1
    high_light_angle: 3
world_objects:
  -
    type: Sphere
    properties:
      name:    "dup"
      center:  [1.0, 2, 3e0]
      radius:  0.7
      radius:  0.75        # duplicate key: the last value wins
      refractive_rate: 1.6
      reflective_attenuation: [0.1, 0.1, 0.1]
      refractive_attenuation: [0.8, 0.8, 0.8]
      diffuse_rate: [0.09, 0.09, 0.09]
      ambient: [0.01, 0.01, 0.01]
      unused_list: [1, 2]
  - type: Plane
    properties:
      point: [0, 0, -1]
      front: [0, 0, 1]
      up: [1, 0, 0]
      u_unit: 0            # `or 1.0`: 0 is falsy in Python -> 1.0
      refractive_rate: false
      diffuse_rate: [0.6, 0.6, 0.6]
      reflective_attenuation: [0.3, 0.3, 0.3]
      ambient: [0.05, 0.05, 0.05]
"""


def test_cli_yaml_edge_cases(cli, tmp_path):
    p = tmp_path / "edge.yml"
    p.write_text(EDGE)
    got = _cli_dump(cli, str(p))
    assert got == _py_dump(str(p))
    assert got["objects"][0]["radius"] == 0.75 and got["objects"][1]["u_unit"] == 1.0
    assert got["objects"][1]["has_refractive_rate"] == 0 and got["lights"][0]["radius"] == 0.5


def test_cli_missing_property_and_usage(cli, tmp_path):
    p = tmp_path / "bad.yml"
    p.write_text(EDGE.replace("      refractive_attenuation: [0.8, 0.8, 0.8]\n", ""))
    r = subprocess.run([cli, "--dump-scene", str(p)], capture_output=True, text=True)
    assert r.returncode == 1 and "refractive_attenuation" in r.stderr
    r = subprocess.run([cli, "s", "out.png"], capture_output=True, text=True)
    assert r.stdout.strip() == "parameter error"                      # main.rb:5-8


@pytest.mark.parametrize("name", ["rails_synth.png", "checker.png"])
def test_cli_png_decoder_matches_python(cli, name):
    from raytracing_rb_amd import png
    p = os.path.join(SCENES, "textures", name)
    a = png.decode_rgb8(p)
    r = subprocess.run([cli, "--decode-png", p], capture_output=True, text=True, check=True)
    assert r.stdout.split() == [str(a.shape[1]), str(a.shape[0]), _fnv1a(a.tobytes())]


@pytest.mark.parametrize("mode,bits", [("RGB", 8), ("P", 8), ("LA", 8), ("RGBA", 16), ("L", 8)])
def test_cli_png_decoder_formats(cli, tmp_path, mode, bits):
    from PIL import Image
    from raytracing_rb_amd import png
    rs = np.random.RandomState(4)
    p = str(tmp_path / "t.png")
    if bits == 16:
        png.write(p, rs.randint(0, 65536, (9, 11, 4)).astype(np.uint16))
    else:
        Image.fromarray(rs.randint(0, 256, (9, 11, 4)).astype(np.uint8), "RGBA").convert(mode).save(p, optimize=True)
    a = png.decode_rgb8(p)
    r = subprocess.run([cli, "--decode-png", p], capture_output=True, text=True, check=True)
    assert r.stdout.split() == [str(a.shape[1]), str(a.shape[0]), _fnv1a(a.tobytes())]


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_cli_render_matches_python_api(gpu, cli, tmp_path):
    """`rtx s`, `rtx 3` (three workers, round-robin tiles or LPT lists) and `rtx 8`
    (LPT lists by the probe's costs) render the frame the Python API renders,
    bit for bit, and write the same PNG bytes."""
    from raytracing_rb_amd.api import Camera, World
    w, c = os.path.join(SCENES, "mix_world.yml"), os.path.join(SCENES, "mix_camera.yml")
    cam = Camera(World(w), c, width=40, height=23)
    fb = cam.render_sync(str(tmp_path / "py.png"))
    for mode, extra in (("s", []), ("3", []), ("3", ["--balance", "lpt"]), ("8", [])):   # 8 workers: LPT lists
        out, raw = str(tmp_path / ("cli_%s.png" % mode)), str(tmp_path / ("cli_%s.f64" % mode))
        r = subprocess.run([cli, mode, out, w, c, "--set", "width=40", "--set", "height=23", "--float-out", raw] + extra,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        got = np.fromfile(raw, np.float64).reshape(fb.shape)
        assert np.array_equal(got.view(np.uint64), fb.view(np.uint64)), mode
        assert open(out, "rb").read() == open(tmp_path / "py.png", "rb").read(), mode


@pytest.mark.gpu
def test_cli_reports_reference_raise(gpu, cli, tmp_path):
    src = open(os.path.join(SCENES, "c1_world.yml")).read()
    src = src.replace("diffuse_rate:           [0.5, 0.5, 0.5]", "diffuse_rate:           [0.99, 0.99, 0.99]")
    src = src.replace("ambient:                [0.05, 0.05, 0.05]", "ambient:                [0.3, 0.3, 0.3]", 1)
    p = tmp_path / "bright.yml"
    p.write_text(src)
    r = subprocess.run([cli, "s", str(tmp_path / "o.png"), str(p), os.path.join(SCENES, "c1_camera.yml"),
                        "--set", "width=24", "--set", "height=14"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "color greater than 1" in r.stderr
