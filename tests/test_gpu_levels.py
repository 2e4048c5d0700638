"""The bounce-level engine (option "engine" = 1) against the
oracle and against the lanes engine.

The two engines run the same binary64 operations on every ray and sum each
camera sample's leaves in trace_sync's order, so their frames must be
identical bit for bit, at every size, batch size and buffer
capacity (overflowing samples are re-rendered by the lanes engine).
"""

import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, SCENES

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4          # north-star tolerance, per channel
MAXABS_TOL = 1e-9


def _scene(world, camera, **ov):
    from raytracing_rb_amd import config
    return config.load_scene(os.path.join(SCENES, world), os.path.join(SCENES, camera), camera_overrides=ov)


def _renderer(sd, cd, engine, **opts):
    from raytracing_rb_amd.runtime import Renderer
    r = Renderer(sd, cd, device=0)
    r.set_option("engine", engine)
    for k, v in opts.items():
        r.set_option(k, v)
    return r


def _same(a, b):
    """Bit-identical frames (also -0.0 vs 0.0 and NaN payloads)."""
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))


def _check(gpu_fb, ref, ok=None, min_exact=0.9):
    ok = np.ones(ref.shape[:2], bool) if ok is None else ok
    d = (gpu_fb - ref)[ok]
    rms = np.sqrt((d ** 2).mean(axis=0))
    assert (rms <= RMS_TOL).all(), rms
    assert np.abs(d).max() <= MAXABS_TOL, np.abs(d).max()
    exact = np.mean(np.all(gpu_fb == ref, axis=-1)[ok])
    assert exact >= min_exact, exact


SCENES_SMALL = [
    ("c1_world.yml", "c1_camera.yml", dict(width=192, height=108)),
    ("c0_world.yml", "camera.yml", dict(width=96, height=54)),
    ("c2_world.yml", "c2_camera.yml", dict(width=160, height=90)),
    ("mix_world.yml", "mix_camera.yml", dict(width=64, height=36)),
    ("mix_world.yml", "mix_camera.yml", dict(width=40, height=22, pre_sample_times=3, max_sample_times=2,
                                             variant_threshold=0.0)),
    ("mix_world.yml", "mix_camera.yml", dict(width=40, height=22, pre_sample_times=2, max_sample_times=5,
                                             variant_threshold=0.0)),
    ("c2_world.yml", "c2_camera.yml", dict(width=48, height=27, pre_sample_times=3, max_sample_times=7,
                                           variant_threshold=1e9)),
    ("mix_world.yml", "mix_camera.yml", dict(width=33, height=19, trace_depth=1)),
    ("mix_world.yml", "mix_camera.yml", dict(width=33, height=19, trace_depth=0)),
    ("mix_world.yml", "mix_camera.yml", dict(width=33, height=19, monte_carlo_diffusion_times=3, trace_depth=4)),
]


@pytest.mark.parametrize("world,camera,ov", SCENES_SMALL)
def test_levels_bit_identical_to_lanes_and_match_oracle(gpu, world, camera, ov):
    from oracle.c_oracle import Oracle
    sd, cd = _scene(world, camera, **ov)
    lanes = _renderer(sd, cd, 0).render(seed=3)
    r = _renderer(sd, cd, 1)
    lv = r.render(seed=3)
    assert _same(lv, lanes)
    st = r.level_stats()
    assert st["redo"] == 0 and st["dropped"] == 0
    ref, status, rc = Oracle(sd, cd).render(seed=3)
    _check(lv, ref, status == 0)


@pytest.mark.parametrize("name", ["c1_64x36", "c0_48x27", "c2_32x18", "mix_24x14", "c4_48x27"])
def test_levels_match_golden(gpu, name):
    if name == "c4_48x27":
        import sys
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import make_scenes
        make_scenes.ensure_c4()
    z = np.load(os.path.join(GOLDEN, "frame_%s.npz" % name))
    sd, cd = _scene(str(z["world"]), str(z["camera"]), **eval(str(z["overrides"]), {}))
    fb = _renderer(sd, cd, 1).render(seed=int(z["seed"]))
    # C4 (depth 8, textured ground): more ocml-vs-glibc ulp differences (as test_gpu_bvh)
    _check(fb, z["frame"], z["status"] == 0, min_exact=0.8 if name == "c4_48x27" else 0.9)
    assert _same(fb, _renderer(sd, cd, 0).render(seed=int(z["seed"])))


@pytest.mark.parametrize("opts", [
    dict(lv_batch=512),                                  # many batches (8x8 tiles x 4 samples = 256 per tile)
    dict(lv_batch=1),                                    # one tile per batch
    dict(lv_stage_pct=5, lv_floor=0),                    # staging overflow: re-rendered by the lanes engine
    dict(lv_rec_pct=101, lv_floor=0),                    # tree-record overflow at level 1
    dict(lv_batch=1000, lv_stage_pct=20, lv_rec_pct=150, lv_floor=0),
    dict(lv_stage_pct=5, lv_floor=0, lv_redo_blocks=1),  # the re-render on a single workgroup
    dict(lv_stage_pct=5, lv_floor=0, lv_redo_blocks=0),  # ... on every resident workgroup
])
def test_levels_batches_and_overflow_change_no_bit(gpu, opts):
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=120, height=70)
    lanes = _renderer(sd, cd, 0).render(seed=5)
    r = _renderer(sd, cd, 1, **opts)
    lv = r.render(seed=5)
    assert _same(lv, lanes)
    st = r.level_stats()
    if "lv_stage_pct" in opts or "lv_rec_pct" in opts:
        assert st["redo"] > 0, st                         # the overflow path ran
    assert sum(st["rays"]) > 0


def test_levels_adaptive_extras_batched(gpu):
    """render_at's extra samples (camera.rb:86-97) in several pass-1 batches."""
    sd, cd = _scene("mix_world.yml", "mix_camera.yml", width=64, height=36, pre_sample_times=2,
                    max_sample_times=6, variant_threshold=1e-4)
    lanes = _renderer(sd, cd, 0).render(seed=9)
    for opts in (dict(), dict(lv_batch=300), dict(lv_batch=64, lv_stage_pct=30, lv_floor=0)):
        assert _same(_renderer(sd, cd, 1, **opts).render(seed=9), lanes), opts


def test_levels_c2_full_frame_identical_to_lanes(gpu):
    """C2 (the metric config) at full 1920x1080, 4xAA, depth 5: every pixel of
    the bounce-level frame equals the lanes engine's, no sample overflowed."""
    sd, cd = _scene("c2_world.yml", "c2_camera.yml")
    lanes = _renderer(sd, cd, 0).render()
    r = _renderer(sd, cd, 1)
    lv = r.render()
    assert _same(lv, lanes)
    st = r.level_stats()
    assert st["redo"] == 0 and st["rays"][0] == 32400 * 256, st


def test_levels_tiles_and_subregions(gpu):
    import torch
    from raytracing_rb_amd import tiles
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=200, height=77)
    r = _renderer(sd, cd, 1)
    full = r.render()
    assert _same(full, _renderer(sd, cd, 0).render())
    for n in (2, 3, 8):
        R = r.rows_per_rank(8, n)
        packed = torch.zeros((n * R, 200, 3), dtype=torch.float64, device="cuda")
        for k in range(n):
            r.render_tiles_device(packed[k * R:(k + 1) * R].data_ptr(), 8, k, n)
        r.sync()
        assert _same(tiles.unpack(packed, 77, 8, n).cpu().numpy(), full), n
    out = torch.zeros((20, 30, 3), dtype=torch.float64, device="cuda")
    r.render_device(out.data_ptr(), x0=10, y0=5, x1=40, y1=25)
    r.sync()
    assert _same(out.cpu().numpy(), full[5:25, 10:40])
    assert _same(r.render_at(33, 17), full[17, 33])


def test_levels_color_gt1_error_reported(gpu, tmp_path):
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import RtxError
    src = open(os.path.join(SCENES, "c1_world.yml")).read()
    src = src.replace("diffuse_rate:           [0.5, 0.5, 0.5]", "diffuse_rate:           [0.99, 0.99, 0.99]")
    src = src.replace("ambient:                [0.05, 0.05, 0.05]", "ambient:                [0.3, 0.3, 0.3]", 1)
    p = tmp_path / "bright.yml"
    p.write_text(src)
    sd, cd = config.load_scene(str(p), os.path.join(SCENES, "c1_camera.yml"), camera_overrides=dict(width=24, height=14))
    msgs = []
    for engine in (0, 1):
        with pytest.raises(RtxError) as e:
            _renderer(sd, cd, engine).render()
        assert e.value.kind == "color_gt1" and "color greater than 1" in str(e.value)
        msgs.append(str(e.value))
    assert msgs[0] == msgs[1]                             # same first erring pixel (render_sync order)


# ---- split phases (option lv_split = 1: trace / shadow / shade launches per level)
@pytest.mark.parametrize("world,camera,ov", SCENES_SMALL)
def test_split_phases_bit_identical(gpu, world, camera, ov):
    sd, cd = _scene(world, camera, **ov)
    lanes = _renderer(sd, cd, 0).render(seed=3)
    r = _renderer(sd, cd, 1, lv_split=1)
    assert _same(r.render(seed=3), lanes)
    st = r.level_stats()
    assert st["redo"] == 0 and st["dropped"] == 0


@pytest.mark.parametrize("opts", [
    dict(lv_batch=512),
    dict(lv_stage_pct=5, lv_floor=0),
    dict(lv_rec_pct=101, lv_floor=0),
    dict(lv_batch=1000, lv_stage_pct=20, lv_rec_pct=150, lv_floor=0),
])
def test_split_phases_batches_and_overflow(gpu, opts):
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=120, height=70)
    lanes = _renderer(sd, cd, 0).render(seed=5)
    r = _renderer(sd, cd, 1, lv_split=1, **opts)
    assert _same(r.render(seed=5), lanes)
    if "lv_stage_pct" in opts or "lv_rec_pct" in opts:
        assert r.level_stats()["redo"] > 0


def test_split_phases_extras_c4_and_errors(gpu, tmp_path):
    import sys
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import RtxError
    sd, cd = _scene("mix_world.yml", "mix_camera.yml", width=64, height=36, pre_sample_times=2,
                    max_sample_times=6, variant_threshold=1e-4)
    lanes = _renderer(sd, cd, 0).render(seed=9)
    for opts in (dict(), dict(lv_batch=300)):
        assert _same(_renderer(sd, cd, 1, lv_split=1, **opts).render(seed=9), lanes), opts
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_scenes
    make_scenes.ensure_c4()
    sd, cd = _scene("c4_world.yml", "c4_camera.yml", width=64, height=36)
    assert _same(_renderer(sd, cd, 1, lv_split=1).render(seed=2), _renderer(sd, cd, 0).render(seed=2))
    src = open(os.path.join(SCENES, "c1_world.yml")).read()
    src = src.replace("diffuse_rate:           [0.5, 0.5, 0.5]", "diffuse_rate:           [0.99, 0.99, 0.99]")
    src = src.replace("ambient:                [0.05, 0.05, 0.05]", "ambient:                [0.3, 0.3, 0.3]", 1)
    p = tmp_path / "bright.yml"
    p.write_text(src)
    sd, cd = config.load_scene(str(p), os.path.join(SCENES, "c1_camera.yml"), camera_overrides=dict(width=24, height=14))
    msgs = []
    for engine, opts in ((0, {}), (1, dict(lv_split=1))):
        with pytest.raises(RtxError) as e:
            _renderer(sd, cd, engine, **opts).render()
        msgs.append(str(e.value))
    assert msgs[0] == msgs[1]


def test_split_phases_c2_full_frame(gpu):
    sd, cd = _scene("c2_world.yml", "c2_camera.yml")
    fused = _renderer(sd, cd, 1, lv_split=0).render()
    r = _renderer(sd, cd, 1, lv_split=1)
    assert _same(r.render(), fused)
    assert r.level_stats()["redo"] == 0


@pytest.mark.parametrize("static", [0, 37, 100])
def test_chunk_schedule_changes_no_bit(gpu, static):
    """Static / sharded-claim chunk schedules (option lv_static) reorder work only."""
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=200, height=96)
    lanes = _renderer(sd, cd, 0).render(seed=4)
    for split in (0, 1):
        assert _same(_renderer(sd, cd, 1, lv_static=static, lv_split=split).render(seed=4), lanes), (static, split)


# ---- hit compaction (option lv_compact: k_level_c parks hits in an LDS ring, shades full waves)
@pytest.mark.parametrize("world,camera,ov", SCENES_SMALL)
def test_compaction_bit_identical(gpu, world, camera, ov):
    sd, cd = _scene(world, camera, **ov)
    lanes = _renderer(sd, cd, 0).render(seed=3)
    for compact in (0, 1, 2):                   # 2: the compact ring (the ray re-derived in the second half)
        for src in (-1, 3, 4):                  # 3: the exact sphere records staged in LDS too; 4: 16-bit leaf records
            r = _renderer(sd, cd, 1, lv_compact=compact, sphere_src=src)
            assert _same(r.render(seed=3), lanes), (compact, src)
        st = r.level_stats()
        assert st["redo"] == 0 and st["dropped"] == 0


@pytest.mark.parametrize("opts", [
    dict(lv_batch=512),
    dict(lv_stage_pct=5, lv_floor=0),                    # children past a slice: re-rendered whole
    dict(lv_rec_pct=101, lv_floor=0),                    # records past the arena
    dict(lv_static=37),                                  # sharded claims: parked hits cross chunk claims
])
def test_compaction_batches_overflow_schedule(gpu, opts):
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=120, height=70)
    lanes = _renderer(sd, cd, 0).render(seed=5)
    for compact in (1, 2):
        r = _renderer(sd, cd, 1, lv_compact=compact, **opts)
        assert _same(r.render(seed=5), lanes), compact
        if "lv_stage_pct" in opts or "lv_rec_pct" in opts:
            assert r.level_stats()["redo"] > 0


def test_compaction_errors_and_c4_fallback(gpu, tmp_path):
    """Raise sites keep their order through the ring (full and compact); C4's
    staged hierarchy leaves no LDS for a ring: with sphere_src 0 the option
    falls back to k_level, with the default (auto: nodes in LDS, leaves from
    global memory) k_level_c runs with the compact ring; the same bits."""
    import sys
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import RtxError
    src = open(os.path.join(SCENES, "c1_world.yml")).read()
    src = src.replace("diffuse_rate:           [0.5, 0.5, 0.5]", "diffuse_rate:           [0.99, 0.99, 0.99]")
    src = src.replace("ambient:                [0.05, 0.05, 0.05]", "ambient:                [0.3, 0.3, 0.3]", 1)
    p = tmp_path / "bright.yml"
    p.write_text(src)
    sd, cd = config.load_scene(str(p), os.path.join(SCENES, "c1_camera.yml"), camera_overrides=dict(width=24, height=14))
    msgs = []
    for engine, opts in ((0, {}), (1, dict(lv_compact=1)), (1, dict(lv_compact=0)), (1, dict(lv_compact=2))):
        with pytest.raises(RtxError) as e:
            _renderer(sd, cd, engine, **opts).render()
        msgs.append(str(e.value))
    assert len(set(msgs)) == 1, msgs
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_scenes
    make_scenes.ensure_c4()
    sd, cd = _scene("c4_world.yml", "c4_camera.yml", width=64, height=36)
    lanes = _renderer(sd, cd, 0).render(seed=2)
    assert _same(_renderer(sd, cd, 1, lv_compact=1).render(seed=2), lanes)
    assert _same(_renderer(sd, cd, 1, lv_compact=1, sphere_src=0).render(seed=2), lanes)
    # the hierarchy's nodes in LDS and its leaves read from global memory
    # (sphere_src 2) leave room for the compact ring: k_level_c on C4
    for src in (1, 2, 4):                       # 4: nodes and 16-bit leaf records in LDS (the auto choice)
        for compact in (0, 1, 2):
            assert _same(_renderer(sd, cd, 1, sphere_src=src, lv_compact=compact).render(seed=2), lanes), (src, compact)


# ---- staged ray records: 80 B (path and root in one word, the RNG key decoded from the root) or 96 B
@pytest.mark.parametrize("world,camera,ov", [
    ("c2_world.yml", "c2_camera.yml", dict(width=160, height=90)),
    ("mix_world.yml", "mix_camera.yml", dict(width=64, height=36)),
    ("mix_world.yml", "mix_camera.yml", dict(width=33, height=19, monte_carlo_diffusion_times=3, trace_depth=4)),
    ("mix_world.yml", "mix_camera.yml", dict(width=40, height=22, pre_sample_times=2, max_sample_times=5,
                                             variant_threshold=0.0)),
])
def test_ray_record_layouts_change_no_bit(gpu, world, camera, ov):
    sd, cd = _scene(world, camera, **ov)
    lanes = _renderer(sd, cd, 0).render(seed=3)
    for rb in (0, 80, 96):
        for opts in (dict(), dict(lv_compact=2), dict(lv_compact=0), dict(lv_split=1), dict(lv_stage_pct=5, lv_floor=0)):
            r = _renderer(sd, cd, 1, lv_ray_bytes=rb, **opts)
            assert r.get_option("lv_ray_bytes_effective") == (96 if rb == 96 else 80)
            assert _same(r.render(seed=3), lanes), (rb, opts)


def test_ray_record_64_bit_paths(gpu):
    """A camera whose ray path ids need more than 32 bits ((pt + 3)^trace_depth
    > 2^32) keeps the 96-B record; asking for 80 B is refused, not truncated."""
    from raytracing_rb_amd.runtime import RtxError
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=32, height=18, trace_depth=17)
    lanes = _renderer(sd, cd, 0).render(seed=3)
    r = _renderer(sd, cd, 1)
    assert r.get_option("lv_ray_bytes_effective") == 96
    assert _same(r.render(seed=3), lanes)
    with pytest.raises(RtxError) as e:
        _renderer(sd, cd, 1, lv_ray_bytes=80).render(seed=3)
    assert e.value.kind == "invalid" and "64 bits" in str(e.value)


def test_compaction_c2_full_frame(gpu):
    sd, cd = _scene("c2_world.yml", "c2_camera.yml")
    plain = _renderer(sd, cd, 1, lv_compact=0).render()
    r = _renderer(sd, cd, 1, lv_compact=1)
    assert _same(r.render(), plain)
    assert r.level_stats()["redo"] == 0


# ---- two halves on two streams (option lv_streams = 2, the default)
@pytest.mark.parametrize("world,camera,ov", SCENES_SMALL)
def test_two_streams_bit_identical(gpu, world, camera, ov):
    sd, cd = _scene(world, camera, **ov)
    lanes = _renderer(sd, cd, 0).render(seed=3)
    stats = []
    for streams in (1, 2, 3, 4):
        r = _renderer(sd, cd, 1, lv_streams=streams)
        assert _same(r.render(seed=3), lanes), streams
        stats.append(r.level_stats())
    assert all(st == stats[0] for st in stats)            # shared totals added atomically by every part


@pytest.mark.parametrize("opts", [
    dict(lv_batch=512),                                   # several batches per half, each half on its stream
    dict(lv_stage_pct=5, lv_floor=0),                     # both halves re-render overflowed samples (own stacks)
    dict(lv_rec_pct=101, lv_floor=0),
    dict(lv_static=37, lv_batch=1000),
])
def test_two_streams_batches_and_overflow(gpu, opts):
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=120, height=70)
    lanes = _renderer(sd, cd, 0).render(seed=5)
    for streams in (2, 4):
        r = _renderer(sd, cd, 1, lv_streams=streams, **opts)
        assert _same(r.render(seed=5), lanes), streams
        if "lv_stage_pct" in opts or "lv_rec_pct" in opts:
            assert r.level_stats()["redo"] > 0


def test_two_streams_extras_tiles_and_errors(gpu, tmp_path):
    """render_at's extra samples: both halves append to one extra list; tile
    shares and raise sites as with one stream."""
    import torch
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import RtxError
    sd, cd = _scene("mix_world.yml", "mix_camera.yml", width=64, height=36, pre_sample_times=2,
                    max_sample_times=6, variant_threshold=1e-4)
    lanes = _renderer(sd, cd, 0).render(seed=9)
    for opts in (dict(), dict(lv_batch=300), dict(lv_streams=3), dict(lv_streams=4, lv_batch=300)):
        assert _same(_renderer(sd, cd, 1, **dict(dict(lv_streams=2), **opts)).render(seed=9), lanes), opts
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=160, height=90)
    one, two = _renderer(sd, cd, 1, lv_streams=1), _renderer(sd, cd, 1, lv_streams=3)
    for k, n in ((0, 3), (2, 3), (1, 8)):
        rows = one.lib.rtx_tiles_rows_per_rank(cd.height, 8, n)
        a = torch.zeros((rows, cd.width, 3), dtype=torch.float64, device="cuda")
        b = torch.zeros_like(a)
        one.render_tiles_device(a.data_ptr(), 8, k, n, seed=2)
        two.render_tiles_device(b.data_ptr(), 8, k, n, seed=2)
        torch.cuda.synchronize()
        assert torch.equal(a.view(torch.int64), b.view(torch.int64)), (k, n)
    src = open(os.path.join(SCENES, "c1_world.yml")).read()
    src = src.replace("diffuse_rate:           [0.5, 0.5, 0.5]", "diffuse_rate:           [0.99, 0.99, 0.99]")
    src = src.replace("ambient:                [0.05, 0.05, 0.05]", "ambient:                [0.3, 0.3, 0.3]", 1)
    p = tmp_path / "bright.yml"
    p.write_text(src)
    sd, cd = config.load_scene(str(p), os.path.join(SCENES, "c1_camera.yml"), camera_overrides=dict(width=24, height=14))
    msgs = []
    for engine, opts in ((0, {}), (1, dict(lv_streams=2)), (1, dict(lv_streams=1))):
        with pytest.raises(RtxError) as e:
            _renderer(sd, cd, engine, **opts).render()
        msgs.append(str(e.value))
    assert msgs[0] == msgs[1] == msgs[2]


def test_two_streams_c2_full_frame_and_kernel_time(gpu):
    sd, cd = _scene("c2_world.yml", "c2_camera.yml")
    one = _renderer(sd, cd, 1, lv_streams=1).render()
    r = _renderer(sd, cd, 1, lv_streams=2)
    assert _same(r.render(), one)
    assert r.level_stats()["redo"] == 0
    r.set_option("kernel_events", 1)
    r.render()
    ms, launches = r.kernel_time()
    assert launches == 10 and 0.5 < ms < 50.0, (ms, launches)   # union of the two halves' level launches


# ---- tree reduction (k_tree_finalize): deep trees, path tracing, extra samples, overflow
@pytest.mark.parametrize("world,camera,ov", [
    ("c2_world.yml", "c2_camera.yml", dict(width=120, height=70)),
    ("mix_world.yml", "mix_camera.yml", dict(width=40, height=22, monte_carlo_diffusion_times=3, trace_depth=6)),
    ("mix_world.yml", "mix_camera.yml", dict(width=40, height=22, pre_sample_times=2, max_sample_times=5,
                                             variant_threshold=0.0)),
])
def test_reduction_changes_no_bit(gpu, world, camera, ov):
    """The tree reduction renders the lanes engine's bits (one and two parts)."""
    sd, cd = _scene(world, camera, **ov)
    lanes = _renderer(sd, cd, 0).render(seed=4)
    for parts in (1, 2):
        r = _renderer(sd, cd, 1, lv_streams=parts)
        assert _same(r.render(seed=4), lanes), parts
        r.close()


def test_reduction_with_overflow(gpu):
    """Re-rendered samples (their trees are not followed) inside reduced tiles."""
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=120, height=70)
    lanes = _renderer(sd, cd, 0).render(seed=6)
    r = _renderer(sd, cd, 1, lv_stage_pct=5, lv_floor=0)
    assert _same(r.render(seed=6), lanes)
    assert r.level_stats()["redo"] > 0
    r.close()


# ---- raises of children the cutoff drops (lv_finish builds only their normalize tests)
HEADON_WORLD = """max_distance: 10000
soft_shadow_exponent: 2
lights:
  - type: Spot
    properties:
      name: side
      position: [2.0, -30.0, 4.0]
      radius: 0.0
      color: [1.0, 1.0, 1.0]
      high_light_rate: 1.0
      high_light_angle: 0.5
world_objects:
  - type: Plane
    properties:
      name: pane
      point: [5.0, 0, 0]
      front: [-1, 0, 0]
      up: [0, 0, 1]
      refractive_rate: 1.5
      diffuse_rate: [0.3, 0.3, 0.3]
      ambient: [0.02, 0.02, 0.02]
      reflective_attenuation: [%s]
      refractive_attenuation: [%s]
"""
HEADON_CAMERA = """position: [0.0, 0.0, 0.0]
up: [0.0, 0.0, 1.0]
front: [1.0, 0.0, 0.0]
retina_width: 0.5
retina_height: 0.5
aperture_radius: 0.0
image_distance: 1.0
focal_distance: 0.5
width: 4
height: 4
pre_sample_times: 1
max_sample_times: 1
variant_threshold: 0.001
trace_depth: %d
monte_carlo_diffusion_times: 1
"""


@pytest.mark.parametrize("refl,refr,depth", [
    ("0.5, 0.5, 0.5", "0.0, 0.0, 0.0", 2),   # refraction child dead: only its normalize test runs
    ("0.5, 0.5, 0.5", "0.5, 0.5, 0.5", 1),   # depth 1: both children dead
    ("0.0, 0.0, 0.0", "0.0, 0.0, 0.0", 2),   # both dead by attenuation
    ("0.5, 0.5, 0.5", "0.5, 0.5, 0.5", 2),   # both alive: the full rays
])
def test_dead_child_raises_match_lanes_and_oracle(gpu, tmp_path, refl, refr, depth):
    """Pixel (2, 2)'s ray is exactly (1, 0, 0) and meets the pane head-on: the
    refraction's (reflection + ray.front).normalize is a zero vector
    (world_object.rb:133), which raises whether or not the refraction ray
    survives the cutoff.  Both engines (and split phases) report the same
    raise at the same pixel as the oracle."""
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import RtxError
    from oracle.c_oracle import Oracle
    w, c = tmp_path / "w.yml", tmp_path / "c.yml"
    w.write_text(HEADON_WORLD % (refl, refr))
    c.write_text(HEADON_CAMERA % depth)
    sd, cd = config.load_scene(str(w), str(c))
    _, status, rc = Oracle(sd, cd).render()
    assert status[2, 2] != 0 and rc != 0
    msgs = []
    for engine, opts in ((0, {}), (1, {}), (1, dict(lv_split=1)), (1, dict(lv_compact=0))):
        with pytest.raises(RtxError) as e:
            _renderer(sd, cd, engine, **opts).render()
        assert e.value.kind == "zero_vec", (engine, opts, str(e.value))
        msgs.append(str(e.value))
    assert len(set(msgs)) == 1, msgs


def test_frames_in_flight_identical(gpu):
    """bench.py's two frames in flight: two contexts on two streams render
    consecutive frames concurrently (one part each); every frame equals the
    one-context render bit for bit."""
    import torch
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=480, height=270)
    ref = _renderer(sd, cd, 1).render(seed=1)
    rs = [_renderer(sd, cd, 1, lv_streams=1) for _ in range(2)]
    ss = [torch.cuda.Stream() for _ in range(2)]
    outs = [torch.zeros((cd.height, cd.width, 3), dtype=torch.float64, device="cuda") for _ in range(2)]
    for i in range(5):
        j = i % 2
        rs[j].render_device(outs[j].data_ptr(), seed=1, stream=ss[j].cuda_stream)
    torch.cuda.synchronize()
    for j in range(2):
        rs[j].sync(ss[j].cuda_stream)
        assert _same(outs[j].cpu().numpy(), ref), j
        rs[j].close()


def test_first_raise_in_render_sync_order(gpu, tmp_path):
    """Two raise sites in one frame: pixel (0, 3) meets a glowing sphere
    (color greater than 1) and pixel (2, 2) meets the pane head-on (zero
    vector).  render_sync walks x outer, y inner (camera.rb:102-103), so the
    call reports (0, 3)'s raise, which a row-major order would not."""
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import RtxError
    from oracle.c_oracle import Oracle
    w, c = tmp_path / "w.yml", tmp_path / "c.yml"
    w.write_text(HEADON_WORLD % ("0.5, 0.5, 0.5", "0.0, 0.0, 0.0") + """  - type: Sphere
    properties:
      name: glow
      center: [3.0, 1.5, -0.75]
      radius: 0.2
      refractive_rate: 1.5
      diffuse_rate: [0.5, 0.5, 0.5]
      ambient: [2.0, 2.0, 2.0]
      reflective_attenuation: [0.0, 0.0, 0.0]
      refractive_attenuation: [0.0, 0.0, 0.0]
""")
    c.write_text(HEADON_CAMERA % 2)
    sd, cd = config.load_scene(str(w), str(c))
    _, status, rc = Oracle(sd, cd).render()
    assert status[3, 0] == 2 and status[2, 2] == 1, status   # color > 1 at (0, 3), zero vector at (2, 2)
    assert rc == 2                                            # the oracle reports in render_sync order too
    msgs = []
    for engine, opts in ((0, {}), (1, {}), (1, dict(lv_split=1))):
        with pytest.raises(RtxError) as e:
            _renderer(sd, cd, engine, **opts).render()
        assert e.value.kind == "color_gt1", (engine, opts, str(e.value))
        msgs.append(str(e.value))
    assert len(set(msgs)) == 1, msgs


PRE_EXTRA_WORLD = """max_distance: 10000
soft_shadow_exponent: 2
lights:
  - type: Spot
    properties:
      name: side
      position: [2.0, -30.0, 4.0]
      radius: 0.0
      color: [1.0, 1.0, 1.0]
      high_light_rate: 1.0
      high_light_angle: 0.5
world_objects:
  - type: Plane
    properties:
      name: wall
      point: [5.0, 0, 0]
      front: [-1, 0, 0]
      up: [0, 0, 1]
      u_unit: 1.0
      v_unit: 1.0
      diffuse_rate: [0.3, 0.3, 0.3]
      ambient: [0.02, 0.02, 0.02]
      reflective_attenuation: [0.0, 0.0, 0.0]
      texture_file_path: %s
      texture_horizontal_scale: 0.0
      texture_vertical_scale: 0.0
  - type: Sphere
    properties:
      name: glow
      center: [3.0, 1.597, 1.51]
      radius: 0.012
      refractive_rate: 1.5
      diffuse_rate: [0.5, 0.5, 0.5]
      ambient: [2.0, 2.0, 2.0]
      reflective_attenuation: [0.0, 0.0, 0.0]
      refractive_attenuation: [0.0, 0.0, 0.0]
"""
PRE_EXTRA_CAMERA = """position: [0.0, 0.0, 0.0]
up: [0.0, 0.0, 1.0]
front: [1.0, 0.0, 0.0]
retina_width: 0.5
retina_height: 0.5
aperture_radius: 0.1
image_distance: 1.0
focal_distance: 0.990099
width: 1
height: 1
pre_sample_times: 1
max_sample_times: 8
variant_threshold: 0.0
trace_depth: 2
monte_carlo_diffusion_times: 1
"""


def test_pre_sample_raise_before_extra_sample_raise(gpu, tmp_path):
    """One pixel, two raise codes: its pre sample meets the wall, whose texture
    scale 0 makes Texture#color's to_i raise FloatDomainError (texture.rb:24,
    code 3); an extra sample (the lens aperture moves it) meets a glowing sphere
    first (color greater than 1, code 2).  render_at traces the pre samples
    before the extra ones (camera.rb:72-97), so the reference raises the domain
    error although its code is the larger one: both engines, split phases and
    no compaction report "domain" as the oracle does (a tie on the
    pixel key used to go to the smaller code)."""
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import RtxError
    from oracle.c_oracle import Oracle
    w, c = tmp_path / "w.yml", tmp_path / "c.yml"
    w.write_text(PRE_EXTRA_WORLD % os.path.join(SCENES, "textures", "checker.png"))
    c.write_text(PRE_EXTRA_CAMERA)
    sd, cd = config.load_scene(str(w), str(c))
    o = Oracle(sd, cd)
    keys = np.array([[0, 0, j] for j in range(8)], np.int32)
    chosen = None
    for seed in range(1, 200):              # a seed whose samples raise: 3, then 2 before any other 3
        rays = np.array([o.lens(0, 0, j, seed) for j in range(8)])
        _, st, _ = o.trace(rays, keys, seed)
        extra = [int(s) for s in st[1:] if s]
        if st[0] == 3 and extra and extra[0] == 2:
            chosen = seed
            break
    assert chosen is not None
    _, status, rc = o.render(seed=chosen)
    assert rc == 3 and status[0, 0] == 3
    for engine, opts in ((0, {}), (1, {}), (1, dict(lv_split=1)), (1, dict(lv_compact=0))):
        with pytest.raises(RtxError) as e:
            _renderer(sd, cd, engine, **opts).render(seed=chosen)
        assert e.value.kind == "domain", (engine, opts, str(e.value))
        assert "pixel (0,0)" in str(e.value)


# ---- tree reduction as a grid-stride loop over the batch's tiles (option lv_fin_grid)
@pytest.mark.parametrize("world,camera,ov", [
    ("c2_world.yml", "c2_camera.yml", dict(width=320, height=181)),       # 920 tiles
    ("mix_world.yml", "mix_camera.yml", dict(width=272, height=153, pre_sample_times=2, max_sample_times=5,
                                             variant_threshold=0.0)),     # 680 tiles; extra samples: pass 1
])
def test_grid_stride_reduction_changes_no_bit(gpu, world, camera, ov):
    """lv_fin_grid = k: k reduction blocks per CU loop over the tiles, reusing
    their LDS column and raise slots between tiles.  With one
    part (lv_streams 1) and k = 1 the grid (one block per CU) is smaller than
    the tile count, so blocks take several tiles each."""
    sd, cd = _scene(world, camera, **ov)
    lanes = _renderer(sd, cd, 0).render(seed=4)
    for k in (1, 4):
        for opts in (dict(), dict(lv_stage_pct=5, lv_floor=0)):
            r = _renderer(sd, cd, 1, lv_fin_grid=k, lv_streams=1, **opts)
            assert _same(r.render(seed=4), lanes), (k, opts)
            r.close()


# ---- ray binning (option lv_sort: levels >= 1 visited bin by bin, records at their dense index)
@pytest.mark.parametrize("world,camera,ov", SCENES_SMALL)
def test_binned_levels_bit_identical(gpu, world, camera, ov):
    sd, cd = _scene(world, camera, **ov)
    lanes = _renderer(sd, cd, 0).render(seed=3)
    for opts in (dict(), dict(lv_compact=0), dict(lv_compact=2), dict(lv_streams=1), dict(lv_sort_copy=1),
                 dict(lv_sort_copy=1, lv_compact=2), dict(lv_sort_copy=1, lv_compact=0)):
        r = _renderer(sd, cd, 1, lv_sort=1, **opts)
        assert r.get_option("lv_sort") == 1
        assert _same(r.render(seed=3), lanes), opts


@pytest.mark.parametrize("opts", [
    dict(lv_batch=512),
    dict(lv_stage_pct=5, lv_floor=0),                    # staging overflow (clamped slices) + re-render
    dict(lv_rec_pct=101, lv_floor=0),
    dict(lv_static=0),                                   # every chunk claimed
    dict(lv_split=1),                                    # split phases: lv_sort has no effect there
    dict(lv_sort_from=2), dict(lv_sort_from=4),          # the first levels in queue order
    dict(lv_sort_from=9),                                # past the last level: nothing binned
    dict(lv_sort_bits=3, lv_sort_from=1), dict(lv_sort_bits=4, lv_sort_from=1),
    dict(lv_sort_copy=1, lv_sort_from=1), dict(lv_sort_copy=1, lv_stage_pct=5, lv_floor=0),   # records moved to bin order
])
def test_binned_levels_batches_overflow_schedule(gpu, opts):
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=120, height=70)
    lanes = _renderer(sd, cd, 0).render(seed=5)
    r = _renderer(sd, cd, 1, lv_sort=1, **opts)
    assert _same(r.render(seed=5), lanes)
    if "lv_stage_pct" in opts:
        assert r.level_stats()["redo"] > 0


def plain_r_last(sd, cd):
    r = _renderer(sd, cd, 1, lv_sort=0)
    r.render()
    return r.get_option("lv_sort_last")


def test_binned_levels_c4_and_c2_full_frame(gpu):
    """Binning on the C4 hierarchy (16-bit leaves, compact ring) and on C2 at
    full size: the same frame as without it."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_scenes
    make_scenes.ensure_c4()
    sd, cd = _scene("c4_world.yml", "c4_camera.yml", width=192, height=108, pre_sample_times=2, max_sample_times=2)
    auto = _renderer(sd, cd, 1)
    assert auto.get_option("lv_sort") == -1 and auto.get_option("lv_sort_effective") == 1   # > 512 spheres
    plain = _renderer(sd, cd, 1, lv_sort=0)
    assert plain.get_option("lv_sort_effective") == 0
    plain = plain.render(seed=4)
    assert _same(auto.render(seed=4), plain) and auto.get_option("lv_sort_last") == cd.trace_depth - 1
    assert _same(_renderer(sd, cd, 1, lv_sort=1, lv_compact=0).render(seed=4), plain)
    assert _same(_renderer(sd, cd, 1, lv_sort_copy=1).render(seed=4), plain)   # records moved to bin order
    sd, cd = _scene("c2_world.yml", "c2_camera.yml")
    plain = _renderer(sd, cd, 1, lv_sort=0)
    assert plain.get_option("lv_sort_effective") == 0
    plain = plain.render()
    assert plain_r_last(sd, cd) == 0
    # 64 spheres: the last level binned (8^3 cells) in batches of >= 2^22 samples: one part per frame
    # (the bench's frames in flight); the default two parts give 4,147,200 samples each, not binned
    r = _renderer(sd, cd, 1)
    assert r.get_option("lv_sort_effective") == 0
    assert _same(r.render(), plain) and r.get_option("lv_sort_last") == 0
    r = _renderer(sd, cd, 1, lv_streams=1)
    assert r.get_option("lv_sort_effective") == 1
    assert _same(r.render(), plain) and r.get_option("lv_sort_last") == 1   # the binning ran
    r = _renderer(sd, cd, 1, lv_sort=1, lv_sort_from=1, lv_sort_bits=4)
    assert _same(r.render(), plain)
    st = r.level_stats()
    assert st["redo"] == 0 and st["dropped"] == 0


def test_binning_options_validated(gpu):
    from raytracing_rb_amd.runtime import RtxError
    sd, cd = _scene("c2_world.yml", "c2_camera.yml", width=32, height=18)
    r = _renderer(sd, cd, 1)
    assert (r.get_option("lv_sort"), r.get_option("lv_sort_from"), r.get_option("lv_sort_bits")) == (-1, 0, 0)
    for k, v in (("lv_sort", 2), ("lv_sort", -2), ("lv_sort_from", -1), ("lv_sort_from", 65), ("lv_sort_bits", 5),
                 ("lv_sort_bits", 2)):
        with pytest.raises(RtxError):
            r.set_option(k, v)
    r.set_option("lv_sort_from", 5)               # past the last level (depth 5: levels 0-4): nothing binned
    assert r.get_option("lv_sort_effective") == 0
    r.set_option("lv_sort_from", 4)
    assert r.get_option("lv_sort_effective") == 1


# ---- the light buffer (option lbuf: shadow walks visit the leaves listed in their cell)
@pytest.mark.parametrize("world,camera,ov", SCENES_SMALL)
def test_light_buffer_bit_identical(gpu, world, camera, ov):
    sd, cd = _scene(world, camera, **ov)
    lanes = _renderer(sd, cd, 0).render(seed=3)
    for opts in (dict(), dict(lv_compact=0), dict(lv_streams=1), dict(lv_sort=1)):
        assert _same(_renderer(sd, cd, 1, lbuf=1, **opts).render(seed=3), lanes), opts
        assert _same(_renderer(sd, cd, 1, lbuf=0, **opts).render(seed=3), lanes), opts


def test_light_buffer_c4_global_table(gpu):
    """C4-sized scenes read a finer table from global memory beside their 16-bit leaves."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_scenes
    make_scenes.ensure_c4()
    sd, cd = _scene("c4_world.yml", "c4_camera.yml", width=160, height=90, pre_sample_times=2, max_sample_times=2)
    plain = _renderer(sd, cd, 1, lbuf=0).render(seed=6)
    assert _same(_renderer(sd, cd, 1).render(seed=6), plain)
    assert _same(_renderer(sd, cd, 1, lv_sort=0).render(seed=6), plain)
    assert _same(_renderer(sd, cd, 0).render(seed=6), plain)


def test_light_buffer_c2_full_frame_and_options(gpu):
    from raytracing_rb_amd.runtime import RtxError
    sd, cd = _scene("c2_world.yml", "c2_camera.yml")
    r = _renderer(sd, cd, 1)
    assert r.get_option("lbuf") == 1
    with pytest.raises(RtxError):
        r.set_option("lbuf", 2)
    assert _same(r.render(), _renderer(sd, cd, 1, lbuf=0).render())
