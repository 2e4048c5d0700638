"""The light buffer: every sphere that can cover a shadow
ray's target is in a leaf listed in the cell the device looks up.  The raise
buffer: every sphere at a tangency where Sphere#cover_area's
Math.acos can raise (sphere.rb:42-46) is in a leaf of the lists the device
reads, unless the device walks the hierarchy for that target.

tools/lbuf_check.cpp builds the hierarchy and the light buffer with librtx's
host builder (rtx_bvh_build.h) and restates query_lbuf's float32 cell lookup;
for random targets it finds, in binary64, every sphere within R of the segment
from the target to the light (a superset of World#lit_area's covers) and counts
those whose leaf is missing from the cell.  The GPU tests compare frames with
and without the buffer (test_gpu_levels.py)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT, SCENES


@pytest.fixture(scope="module")
def tool(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("lbuf") / "lbuf_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-w", "-o", exe, os.path.join(ROOT, "tools", "lbuf_check.cpp")],
                   check=True, timeout=300)
    return exe


def _run(tool, lights, spheres, n, per_light=20000, raise_nc=None):
    text = "".join("light %s\n" % " ".join(repr(float(x)) for x in L) for L in lights)
    text += "".join("%r %r %r %r\n" % tuple(map(float, s)) for s in spheres)
    args = [tool, str(n), str(per_light)] + (["raise", str(raise_nc)] if raise_nc else [])
    out = subprocess.run(args, input=text, capture_output=True, text=True, timeout=300)
    assert out.returncode in (0, 3), out.stderr
    f = out.stdout.split()
    return dict(zip(f[0::2], map(int, f[1::2]))), out.stderr


def _scene_spheres(world, camera):
    from raytracing_rb_amd import config
    sd, _ = config.load_scene(os.path.join(SCENES, world), os.path.join(SCENES, camera))
    lights = [tuple(L.position) for L in sd.lights]
    spheres = [(o.center[0], o.center[1], o.center[2], o.radius) for o in sd.objects[:sd.n_objects] if o.type == 0]
    return lights, spheres, [float(L.radius) for L in sd.lights]


@pytest.mark.parametrize("world,camera", [("c2_world.yml", "c2_camera.yml"), ("mix_world.yml", "mix_camera.yml")])
@pytest.mark.parametrize("n", [8, 16, 24])
def test_scene_light_buffers_hold_every_cover(tool, world, camera, n):
    lights, spheres, _ = _scene_spheres(world, camera)
    r, err = _run(tool, lights, spheres, n)
    assert r["covers"] > 1000 and r["misses"] == 0, (r, err)


def test_random_scenes_and_lights_inside_on_and_near_spheres(tool):
    rng = np.random.default_rng(7)
    for trial in range(6):
        k = [5, 40, 300][trial % 3]
        c = rng.uniform(-5, 5, (k, 3))
        rad = rng.uniform(0.05, 1.2, k)
        spheres = np.concatenate([c, rad[:, None]], axis=1)
        s0 = spheres[0]
        u = rng.normal(size=3)
        u /= np.linalg.norm(u)
        lights = [rng.uniform(-8, 8, 3),                 # anywhere
                  s0[:3] + 0.3 * s0[3] * u,              # inside a sphere: its leaf in every cell
                  s0[:3] + s0[3] * u,                    # on its surface
                  s0[:3] + (s0[3] + 1e-7) * u]           # just outside
        r, err = _run(tool, lights, spheres, 16, per_light=8000)
        assert r["misses"] == 0, (trial, r, err)


# ------------------------------------------------------------------ the raise buffer
@pytest.mark.parametrize("world,camera,n,nc", [("c2_world.yml", "c2_camera.yml", 24, 12),
                                               ("c2_world.yml", "c2_camera.yml", 24, 8),
                                               ("c2_world.yml", "c2_camera.yml", 16, 8),
                                               ("mix_world.yml", "mix_camera.yml", 24, 12),
                                               ("c4_world.yml", "c4_camera.yml", 160, 160),
                                               ("c4_world.yml", "c4_camera.yml", 160, 40)])
def test_scene_raise_buffers_hold_every_tangency(tool, world, camera, n, nc):
    """The scenes' own buffers (rtx_scene_upload's resolutions: C2 and mix 24 /
    12, C4 160 / 160 with per-sphere lists; and coarser ones): no tangent sphere
    outside the lists (fallback targets walk the hierarchy)."""
    lights, spheres, radii = _scene_spheres(world, camera)
    r, err = _run(tool, [tuple(L) + (rad,) for L, rad in zip(lights, radii)], spheres, n,
                  per_light=20000, raise_nc=nc)
    assert r["tangencies"] - r["fallbacks"] > 2000 and r["misses"] == 0, (r, err)


def test_raise_buffers_random_scenes_and_lights(tool):
    """Random scenes, lights of random radius anywhere, inside, on and just
    outside a sphere; both nested resolutions."""
    rng = np.random.default_rng(11)
    for trial in range(6):
        k = [5, 40, 300][trial % 3]
        c = rng.uniform(-5, 5, (k, 3))
        rad = rng.uniform(0.05, 1.2, k)
        spheres = np.concatenate([c, rad[:, None]], axis=1)
        s0 = spheres[0]
        u = rng.normal(size=3)
        u /= np.linalg.norm(u)
        lights = [tuple(rng.uniform(-8, 8, 3)) + (rng.uniform(0.1, 2.0),),
                  tuple(s0[:3] + 0.3 * s0[3] * u) + (0.5,),
                  tuple(s0[:3] + s0[3] * u) + (0.8,),
                  tuple(s0[:3] + (s0[3] + 1e-7) * u) + (1.5,),
                  tuple(rng.uniform(-8, 8, 3)) + (0.0,)]      # a point light: no raises, no lists
        for n, nc in ((16, 8), (24, 12)):
            r, err = _run(tool, lights, spheres, n, per_light=6000, raise_nc=nc)
            assert r["misses"] == 0 and r["tangencies"] > r["fallbacks"], (trial, n, r, err)


def test_raise_buffer_check_has_teeth(tool, tmp_path):
    """The same check with one of the device's lists left out finds misses
    (so a zero above means every list was needed and held the spheres)."""
    src = open(os.path.join(ROOT, "tools", "lbuf_lookup.h")).read()
    lights, spheres, radii = _scene_spheres("c2_world.yml", "c2_camera.yml")
    L = [tuple(l) + (rad,) for l, rad in zip(lights, radii)]
    for drop in ("t == 1", "t == 2"):              # B1, M
        d = tmp_path / drop.replace(" ", "").replace("=", "")
        (d / "tools").mkdir(parents=True)
        (d / "tools" / "lbuf_lookup.h").write_text(
            src.replace("if (!open[t]) continue;", "if (!open[t] || %s) continue;" % drop).replace(
                '"../raytracing_rb_amd/csrc/rtx_bvh_build.h"', '"%s/raytracing_rb_amd/csrc/rtx_bvh_build.h"' % ROOT))
        chk = open(os.path.join(ROOT, "tools", "lbuf_check.cpp")).read().replace(
            '"../raytracing_rb_amd/csrc/rtx_bvh_build.h"', '"%s/raytracing_rb_amd/csrc/rtx_bvh_build.h"' % ROOT)
        (d / "tools" / "lbuf_check.cpp").write_text(chk)
        exe = str(d / "chk")
        subprocess.run(["g++", "-O2", "-std=c++17", "-w", "-o", exe, str(d / "tools" / "lbuf_check.cpp")],
                       check=True, timeout=300)
        r, err = _run(exe, L, spheres, 24, per_light=20000, raise_nc=8)
        assert r["misses"] > 0, (drop, r)
