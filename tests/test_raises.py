"""Sphere#cover_area's Math.acos raise (sphere.rb:42-46) on the two lit_area
calls of the reference:

* World#high_lights' `&& lit_area(ray.position, light.position, light.radius,
  object)` (world.rb:92-93): always truthy, but it runs for every light whose
  cone the ray is in, and its raise aborts the render.  Reproduced by both
  oracles and both engines.
* World#local_lights' lit_area (world.rb:76) over spheres whose binary cover
  factor is 0 (behind the target, inside the cone off the line, beyond the
  light): option exact_raises = 1, the default, checks them (the light buffer's
  cell and the raise buffer's lists, or the widened hierarchy walk, DESIGN.md
  §2.4); exact_raises = 0 reports only the covers the walks evaluate.

The raising spheres are found by tools/raise_search.py (committed in
tests/golden/raise_scenes.json): a sphere placed within a few ulps of the
tangency d = |R - r1|, where cos_theta rounds below -1.
"""

import json
import os
import re
import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import raise_cases  # noqa: E402
import raise_search  # noqa: E402

with open(os.path.join(GOLDEN, "raise_scenes.json")) as _f:
    CASES = json.load(_f)


def _v(a):
    return "[%s]" % ", ".join(repr(float(x)) for x in a)


def _light(L, radius, angle):
    return """lights:
  - type: Spot
    properties:
      name: L
      position: %s
      radius: %r
      color: [0.5, 0.5, 0.5]
      high_light_rate: 1.0
      high_light_angle: %r
""" % (_v(L), float(radius), float(angle))


def _sphere(name, C, R):
    return """  - type: Sphere
    properties:
      name: %s
      center: %s
      radius: %r
      refractive_rate: 1.5
      diffuse_rate: [0.5, 0.5, 0.5]
      ambient: [0.05, 0.05, 0.05]
      reflective_attenuation: [0.3, 0.3, 0.3]
      refractive_attenuation: [0.0, 0.0, 0.0]
""" % (name, _v(C), float(R))


def _fillers(n):
    """n small spheres far from every axis and cone of these scenes (so that a
    hierarchy is built, bvh_min = 32): they neither raise nor occlude."""
    rng = np.random.default_rng(5)
    out = ""
    for i in range(n):
        c = (rng.uniform(-20, 20), 60.0 + rng.uniform(0, 20), rng.uniform(-20, 20))
        out += _sphere("f%d" % i, c, 0.3 + 0.2 * rng.uniform())
    return out


def _world(tmp_path, case, angle, extra="", fillers=0, plane=False, sphere=True, name="w.yml"):
    c = CASES[case]
    src = "max_distance: 10000\nsoft_shadow_exponent: 2\n" + _light(c["L"], c["light_radius"], angle)
    src += "world_objects:\n"
    if plane:
        src += """  - type: Plane
    properties:
      name: ground
      point: [0.0, 0.0, 0.0]
      front: [0.0, 0.0, 1.0]
      up: [1.0, 0.0, 0.0]
      diffuse_rate: [0.6, 0.6, 0.6]
      reflective_attenuation: [0.3, 0.3, 0.3]
      ambient: [0.05, 0.05, 0.05]
"""
    if sphere:
        src += _sphere("raiser", c["center"], c["radius"])
    src += extra + _fillers(fillers)
    p = tmp_path / name
    p.write_text(src)
    return str(p)


def _camera(tmp_path, T, front, w=24, h=16, depth=2):
    p = tmp_path / "c.yml"
    p.write_text("""position: %s
up: [0.0, 0.0, 1.0]
front: %s
retina_width: 0.016
retina_height: 0.012
aperture_radius: 0.0
image_distance: 0.0171
focal_distance: 0.017
width: %d
height: %d
pre_sample_times: 1
max_sample_times: 1
variant_threshold: 0.001
trace_depth: %d
monte_carlo_diffusion_times: 1
""" % (_v(T), _v(front), w, h, depth))
    return str(p)


def _load(w, c):
    from raytracing_rb_amd import config
    return config.load_scene(w, c)


def _first_pixel(status, code):
    """The first raise in render_sync order (x outer, y inner, camera.rb:102-103)."""
    ys, xs = np.nonzero(status)
    assert len(xs), "no raise"
    k = np.argmin(xs * status.shape[0] + ys)
    assert status[ys[k], xs[k]] == code
    return int(xs[k]), int(ys[k])


# ------------------------------------------------------------------ CPU: the search and the oracles
def test_search_reproduces_committed_configurations():
    got = raise_search.search_all(raise_cases.pixel_T())
    assert got == CASES


@pytest.mark.parametrize("case", sorted(CASES))
def test_found_sphere_raises_in_the_reference_arithmetic(case):
    c = CASES[case]
    cos = raise_search.cover_raises(c["center"], c["radius"], c["T"], c["L"], c["light_radius"])
    assert cos is not None and min(cos) < -1.0
    # one ulp of the radius either way leaves the tangency: at least one side does not raise
    up = np.nextafter(c["radius"], 2 * c["radius"])
    dn = np.nextafter(c["radius"], 0.0)
    r_up = raise_search.cover_raises(c["center"], up, c["T"], c["L"], c["light_radius"])
    r_dn = raise_search.cover_raises(c["center"], dn, c["T"], c["L"], c["light_radius"])
    assert not (r_up and min(r_up) < -1 and r_dn and min(r_dn) < -1)


def _highlight_scene(tmp_path, fillers=0, sphere=True):
    c = CASES["highlight"]
    w = _world(tmp_path, "highlight", 12.0, fillers=fillers, sphere=sphere)
    cam = _camera(tmp_path, c["T"], c["L"])      # looking at the light: the central pixels fire
    return _load(w, cam)


def test_oracles_raise_on_highlight_lit_area(oracle_lib, tmp_path):
    """C oracle and rt_ref: every camera ray in the light's cone raises (its
    origin is the camera position exactly, aperture 0); without the sphere none."""
    from oracle import rt_ref
    from oracle.c_oracle import Oracle
    sd, cd = _highlight_scene(tmp_path)
    out, status, rc = Oracle(sd, cd).render()
    assert rc == 3 and (status == 3).sum() > 10, (rc, (status == 3).sum())
    x, y = _first_pixel(status, 3)
    # the Python restatement raises at the same first pixel
    c = CASES["highlight"]
    _, cam = rt_ref.load_scene(str(tmp_path / "w.yml"), str(tmp_path / "c.yml"))
    with pytest.raises(Exception) as e:
        for xx in range(cd.width):                # render_sync: x outer, y inner
            for yy in range(cd.height):
                cam.render_at(xx, yy)
    assert "DomainError" in str(e.value)
    assert (xx, yy) == (x, y)
    # control: the same scene without the raising sphere renders, highlights and all
    sd2, cd2 = _highlight_scene(tmp_path, sphere=False)
    out2, status2, rc2 = Oracle(sd2, cd2).render()
    assert rc2 == 0 and not status2.any() and out2.max() > 0
    assert c["center"][0] < 0                     # the sphere is behind the camera: no ray ever meets it


def _shadow_trace(tmp_path, case, fillers=0, name="w.yml"):
    """rtx_trace of the ray (0,0,1) -> (0,0,-1): it hits the plane z = 0 at
    (0,0,0), so local_lights' target is (0,0,1e-5); depth 1 (no children).
    The light is off the highlight cone of every ray here."""
    w = _world(tmp_path, case, 1.0, plane=True, fillers=fillers, name=name)
    cam = _camera(tmp_path, (0.0, 0.0, 1.0), (1.0, 0.0, 0.0), depth=1)
    sd, cd = _load(w, cam)
    rays = np.array([[0.0, 0.0, -1.0, 0.0, 0.0, 1.0]])       # front, position
    keys = np.array([[0, 0, 0]], np.int32)
    return sd, cd, rays, keys


@pytest.mark.parametrize("case", ["shadow_A", "shadow_B"])
def test_oracle_raises_on_local_lights_factor0_cover(oracle_lib, tmp_path, case):
    from oracle.c_oracle import Oracle
    sd, cd, rays, keys = _shadow_trace(tmp_path, case)
    out, st, rc = Oracle(sd, cd).trace(rays, keys)
    assert rc == 3 and st[0] == 3, (rc, st)
    # control: shifting the light by one ulp leaves the tangency (no raise)
    c = dict(CASES[case])
    c["L"] = [np.nextafter(c["L"][0], 10.0)] + c["L"][1:]
    CASES["_tmp"] = c
    try:
        sd2, cd2, _, _ = _shadow_trace(tmp_path, "_tmp", name="w2.yml")
        out2, st2, rc2 = Oracle(sd2, cd2).trace(rays, keys)
    finally:
        CASES.pop("_tmp")
    if rc2 == 0:
        assert out2[0].max() > 0


PIXEL_CASES = ["pixel_A_back", "pixel_B_front", "pixel_A_far"]


def _pixel_scene(tmp_path, case, fillers=0, sphere=True):
    """The plane, the light and the raising sphere of a pixel case, seen by
    raise_search.PIXEL_CAMERA: PIXEL's primary ray hits the plane at exactly
    the case's T, so its local_lights raises (high-light angle 1 degree: no
    camera or reflected ray is in the light's cone here)."""
    c = CASES[case]
    w = _world(tmp_path, case, 1.0, plane=True, fillers=fillers, sphere=sphere)
    cc = raise_search.PIXEL_CAMERA
    cam = tmp_path / "c.yml"
    cam.write_text(raise_cases.camera_yaml(cc["position"], cc["front"], cc["width"], cc["height"]))
    return _load(w, str(cam))


@pytest.mark.parametrize("case", PIXEL_CASES)
def test_oracles_raise_at_the_pixel_of_a_factor0_cover(oracle_lib, tmp_path, case):
    """A whole render raises Math::DomainError first at PIXEL in both oracles;
    without the sphere it renders."""
    from oracle import rt_ref
    from oracle.c_oracle import Oracle
    c = CASES[case]
    assert c["T"] == list(raise_cases.pixel_T())
    sd, cd = _pixel_scene(tmp_path, case)
    out, status, rc = Oracle(sd, cd).render()
    assert rc == 3, rc
    assert _first_pixel(status, 3) == tuple(raise_search.PIXEL)
    _, cam = rt_ref.load_scene(str(tmp_path / "w.yml"), str(tmp_path / "c.yml"))
    with pytest.raises(Exception) as e:
        for xx in range(cd.width):
            for yy in range(cd.height):
                cam.render_at(xx, yy)
    assert "DomainError" in str(e.value) and (xx, yy) == tuple(raise_search.PIXEL)
    sd2, cd2 = _pixel_scene(tmp_path, case, sphere=False)
    out2, status2, rc2 = Oracle(sd2, cd2).render()
    assert rc2 == 0 and not status2.any()


# ------------------------------------------------------------------ GPU
ENGINES = [(0, {}), (1, {}), (1, dict(lv_split=1)), (1, dict(lv_compact=0)), (1, dict(lv_compact=2)),
           (0, dict(bvh=2)), (1, dict(bvh=2)), (1, dict(bvh=2, sphere_src=2)), (1, dict(bvh=2, sphere_src=4)),
           (1, dict(bvh=0)), (1, dict(bvh=2, sphere_src=4, lv_split=1)),
           (1, dict(lv_hl_cap=1)), (1, dict(lv_hl_cap=1, lv_split=1)),   # deferred-check list overflow: re-render
           (1, dict(lv_sort=1)), (1, dict(lv_sort=1, bvh=2, sphere_src=4))]  # binned levels (SORT kernels)


def _renderer(sd, cd, engine, **opts):
    from raytracing_rb_amd.runtime import Renderer
    r = Renderer(sd, cd, device=0)
    r.set_option("engine", engine)
    for k, v in opts.items():
        r.set_option(k, v)
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("fillers", [0, 40, 300])
def test_gpu_highlight_lit_area_raise_matches_oracle(gpu, tmp_path, fillers):
    """Same raise code and first pixel from the oracle and every engine / walk
    (40 filler spheres: the hierarchy walk of lit_area_raises; 300: k_hl_raise's
    per-lane walk instead of its wave over the spheres, used up to 256 spheres)."""
    from oracle.c_oracle import Oracle
    from raytracing_rb_amd.runtime import RtxError
    sd, cd = _highlight_scene(tmp_path, fillers=fillers)
    _, status, rc = Oracle(sd, cd).render()
    assert rc == 3
    x, y = _first_pixel(status, 3)
    for engine, opts in ENGINES:
        with pytest.raises(RtxError) as e:
            _renderer(sd, cd, engine, **opts).render()
        assert e.value.kind == "domain", (engine, opts, str(e.value))
        m = re.search(r"at pixel \((\d+),(\d+)\)", str(e.value))
        assert m and (int(m.group(1)), int(m.group(2))) == (x, y), (engine, opts, str(e.value), (x, y))
    # control: without the sphere the frame renders and equals the oracle's
    sd2, cd2 = _highlight_scene(tmp_path, fillers=fillers, sphere=False)
    ref, st2, rc2 = Oracle(sd2, cd2).render()
    assert rc2 == 0
    for engine, opts in ENGINES:
        fb = _renderer(sd2, cd2, engine, **opts).render()
        assert np.abs(fb - ref).max() <= 1e-12, (engine, opts)


@pytest.mark.gpu
def test_gpu_highlight_raise_through_trace_and_path_trace(gpu, tmp_path):
    """rtx_trace / rtx_path_trace of a ray from T straight at the light."""
    from raytracing_rb_amd.runtime import RtxError
    c = CASES["highlight"]
    sd, cd = _highlight_scene(tmp_path)
    d = np.subtract(c["L"], c["T"])
    rays = np.array([list(d) + list(c["T"])])
    for engine in (0, 1):
        r = _renderer(sd, cd, engine)
        with pytest.raises(RtxError) as e:
            r.trace(rays, np.array([[0, 0, 0]], np.int32))
        assert e.value.kind == "domain"
        with pytest.raises(RtxError) as e:
            r.path_trace(rays)
        assert e.value.kind == "domain"


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["shadow_A", "shadow_B"])
@pytest.mark.parametrize("fillers", [0, 40, 300, 600])    # (600: 16-bit leaves, per-sphere raise lists)
def test_gpu_local_lights_factor0_raise(gpu, tmp_path, case, fillers):
    """rtx_trace (the lanes engine, every sphere walk): the default
    (exact_raises = 1) reports the raise of the factor-0 cover, as the oracle
    does; exact_raises = 0 returns the colour."""
    from oracle.c_oracle import Oracle
    from raytracing_rb_amd.runtime import RtxError
    sd, cd, rays, keys = _shadow_trace(tmp_path, case, fillers=fillers)
    ref, st, rc = Oracle(sd, cd).trace(rays, keys)
    assert rc == 3
    for engine, opts in ENGINES:
        with pytest.raises(RtxError) as e:
            _renderer(sd, cd, engine, **opts).trace(rays, keys)
        assert e.value.kind == "domain", (engine, opts)
        fb = _renderer(sd, cd, engine, exact_raises=0, **opts).trace(rays, keys)
        assert np.isfinite(fb).all()


@pytest.mark.gpu
@pytest.mark.parametrize("case", PIXEL_CASES)
@pytest.mark.parametrize("fillers", [0, 40, 300, 600])    # (600: 16-bit leaves, per-sphere raise lists)
def test_gpu_local_lights_factor0_raise_in_a_render(gpu, tmp_path, case, fillers):
    """A whole render through every engine / walk / ring / split / sphere mode
    with the default exact_raises = 1 (the light buffer's cell and the raise
    buffer's lists, or the widened hierarchy walk): the same
    Math::DomainError at the same first pixel as the oracle.  With
    exact_raises = 0 the frame renders, and every pixel the oracle does not
    raise at equals the oracle's."""
    from oracle.c_oracle import Oracle
    from raytracing_rb_amd.runtime import RtxError
    sd, cd = _pixel_scene(tmp_path, case, fillers=fillers)
    out, status, rc = Oracle(sd, cd).render()
    assert rc == 3
    x, y = _first_pixel(status, 3)
    ok = status == 0
    for engine, opts in ENGINES:
        with pytest.raises(RtxError) as e:
            _renderer(sd, cd, engine, **opts).render()
        assert e.value.kind == "domain", (engine, opts, str(e.value))
        m = re.search(r"at pixel \((\d+),(\d+)\)", str(e.value))
        assert m and (int(m.group(1)), int(m.group(2))) == (x, y), (engine, opts, str(e.value), (x, y))
        fb = _renderer(sd, cd, engine, exact_raises=0, **opts).render()
        assert np.isfinite(fb).all(), (engine, opts)
        assert np.abs(fb - out)[ok].max() <= 1e-12, (engine, opts)
    # control: without the sphere the frame renders and equals the oracle's, with the check on
    sd2, cd2 = _pixel_scene(tmp_path, case, fillers=fillers, sphere=False)
    ref, st2, rc2 = Oracle(sd2, cd2).render()
    assert rc2 == 0
    for engine, opts in ENGINES:
        fb = _renderer(sd2, cd2, engine, **opts).render()
        assert np.abs(fb - ref).max() <= 1e-12, (engine, opts)
