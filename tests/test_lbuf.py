"""The light buffer: every sphere that can cover a shadow
ray's target is in a leaf listed in the cell the device looks up.

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


def _run(tool, lights, spheres, n, per_light=20000):
    text = "".join("light %r %r %r\n" % tuple(map(float, L)) for L in lights)
    text += "".join("%r %r %r %r\n" % tuple(map(float, s)) for s in spheres)
    out = subprocess.run([tool, str(n), str(per_light)], input=text, capture_output=True, text=True, timeout=300)
    assert out.returncode in (0, 3), out.stderr
    f = out.stdout.split()
    return dict(zip(f[0::2], map(int, f[1::2]))), out.stderr


def _scene_spheres(world, camera):
    from raytracing_rb_amd import config
    sd, _ = config.load_scene(os.path.join(SCENES, world), os.path.join(SCENES, camera))
    lights = [tuple(L.position) for L in sd.lights]
    spheres = [(o.center[0], o.center[1], o.center[2], o.radius) for o in sd.objects[:sd.n_objects] if o.type == 0]
    return lights, spheres


@pytest.mark.parametrize("world,camera", [("c2_world.yml", "c2_camera.yml"), ("mix_world.yml", "mix_camera.yml")])
@pytest.mark.parametrize("n", [8, 16, 24])
def test_scene_light_buffers_hold_every_cover(tool, world, camera, n):
    lights, spheres = _scene_spheres(world, camera)
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
