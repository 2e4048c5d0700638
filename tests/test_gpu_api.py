"""The Ruby API surface (World / Camera / RayTracer / Ray / CLI) over librtx,
checked against the oracle — reads like the reference's call sites
(src/main.rb:15-21, camera.rb:41-110, ray_tracer.rb:16)."""

import os

import numpy as np
import pytest

from conftest import SCENES

pytestmark = pytest.mark.gpu


def _world_camera(**ov):
    from raytracing_rb_amd.api import Camera, World
    world = World(os.path.join(SCENES, "mix_world.yml"))
    cam = Camera(world, os.path.join(SCENES, "mix_camera.yml"), **(ov or {"width": 48, "height": 27}))
    return world, cam


def _oracle(world, cam):
    from oracle.c_oracle import Oracle
    return Oracle(world.scene, cam.desc)


def test_render_at_matches_oracle(gpu):
    world, cam = _world_camera()
    o = _oracle(world, cam)
    for x, y in [(0, 0), (47, 26), (20, 13), (5, 22)]:
        item = cam.render_at(x, y)
        assert item["position"] == [x, cam.height - 1 - y]          # camera.rb:98
        ref, st, rc = o.render_pixels([[x, y]])
        assert np.abs(np.array(item["color"]) - ref[0]).max() <= 1e-9


def test_render_sync_png_and_fork_agree(gpu, tmp_path):
    from raytracing_rb_amd import png
    world, cam = _world_camera()
    fb = cam.render_sync(str(tmp_path / "s.png"))
    img = png.decode_rgb8(str(tmp_path / "s.png"))
    q = np.minimum(np.trunc(fb * 256.0), 255).astype(np.int64)
    assert np.array_equal(img.astype(np.int64), (q * 255) >> 8)       # array_to_color + Color#blend
    fb2 = cam.render_fork(str(tmp_path / "f.png"), 3)                 # 3 workers (tiles) on this node
    assert np.array_equal(fb, fb2)
    assert open(tmp_path / "s.png", "rb").read() == open(tmp_path / "f.png", "rb").read()


def test_trace_sync_matches_oracle(gpu):
    from raytracing_rb_amd.api import Ray
    world, cam = _world_camera()
    o = _oracle(world, cam)
    ray = Ray([1.0, 0.1, -0.05], [0.0, 0.0, 0.0])
    got = cam.ray_tracer.trace_sync(3, 4, ray, 1)
    ref, st, rc = o.trace(np.array([[1.0, 0.1, -0.05, 0.0, 0.0, 0.0]]), np.array([[3, 4, 1]]))
    assert np.abs(np.array(got.to_a()) - ref[0]).max() <= 1e-9


def test_cli(gpu, tmp_path):
    from raytracing_rb_amd import png
    from raytracing_rb_amd.__main__ import main
    cam_yml = tmp_path / "cam.yml"
    src = open(os.path.join(SCENES, "c1_camera.yml")).read()
    src = src.replace("width:            1920", "width:            64").replace("height:           1080",
                                                                                "height:           36")
    cam_yml.write_text(src)
    out = str(tmp_path / "o.png")
    assert main(["s", out, os.path.join(SCENES, "c1_world.yml"), str(cam_yml)]) == 0
    assert png.decode_rgb8(out).shape == (36, 64, 3)
    assert main(["s", out]) == 1                                      # "parameter error"


def test_render_multi_rccl_gather_matches_render(gpu):
    """rtx_render_multi (Camera#render_fork over the node's GPUs, camera.rb:41-68):
    one context per visible GPU, ONE RCCL ncclSend/ncclRecv group to the first
    (on a 1-GPU box a 1-rank clique sending to itself), bit-identical to
    rtx_render; then more workers than GPUs (device copies)."""
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import Renderer, device_count, render_multi
    sd, cd = config.load_scene(os.path.join(SCENES, "c2_world.yml"), os.path.join(SCENES, "c2_camera.yml"),
                               camera_overrides=dict(width=200, height=77))
    n = device_count()
    assert n >= 1
    rs = [Renderer(sd, cd, device=k) for k in range(n)]
    full = rs[0].render(seed=4)
    got = render_multi(rs, tile_rows=8, seed=4)
    assert np.array_equal(got.view(np.uint64), full.view(np.uint64))
    got = render_multi(rs, tile_rows=8, seed=4)            # the cached clique again
    assert np.array_equal(got.view(np.uint64), full.view(np.uint64))
    rs3 = [Renderer(sd, cd, device=k % n) for k in range(3)]
    got3 = render_multi(rs3, tile_rows=5, seed=4)
    assert np.array_equal(got3.view(np.uint64), full.view(np.uint64))


def test_render_multi_plan_lpt_matches_render(gpu):
    """rtx_render_multi_plan (ADVICE / VERDICT r04 item 8): LPT tile lists from
    the measured rays (rtx_tile_rays) and from the probe (rtx_tile_probe, no
    render) for 3 contexts on one device (the device-copy gather) and one per
    visible GPU (RCCL): every frame bit-identical to rtx_render; a plan that
    lists a tile twice or omits one is refused."""
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import Renderer, RtxError, device_count, lpt_plan_native, render_multi_plan
    from raytracing_rb_amd.tiles import lpt_plan, row_tile_costs
    sd, cd = config.load_scene(os.path.join(SCENES, "c2_world.yml"), os.path.join(SCENES, "c2_camera.yml"),
                               camera_overrides=dict(width=200, height=77))
    n = device_count()
    r0 = Renderer(sd, cd, device=0)
    full = r0.render(seed=4)
    rays = row_tile_costs(r0.tile_rays(), 8)
    probe = r0.tile_probe().sum(axis=1)
    assert probe.shape == rays.shape and (probe > 0).any()
    for ranks in (3, n):
        rs = [Renderer(sd, cd, device=k % n) for k in range(ranks)]
        for costs in (rays, probe):
            plan = lpt_plan(costs, ranks)
            assert lpt_plan_native(costs, ranks) == plan
            got = render_multi_plan(rs, plan, tile_rows=8, seed=4)
            assert np.array_equal(got.view(np.uint64), full.view(np.uint64)), (ranks, list(costs))
    rs = [Renderer(sd, cd, device=k % n) for k in range(3)]
    plan = lpt_plan(rays, 3)
    bad = [list(l) for l in plan]
    bad[1][0] = bad[0][0]                               # listed twice (and one tile in no list)
    with pytest.raises(RtxError):
        render_multi_plan(rs, bad, tile_rows=8, seed=4)
