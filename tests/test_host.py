"""Host-side logic: YAML loader vs the oracle's own loader, PNG codec, C-ABI
exports, frame sharding (incl. a world_size-2 gloo gather)."""

import os
import re

import numpy as np
import pytest

from conftest import REFERENCE, ROOT, SCENES
from raytracing_rb_amd import config, png, tiles
from raytracing_rb_amd._abi import RTX_BOX, RTX_PLANE, RTX_SPHERE


# ------------------------------------------------------------------ config
@pytest.mark.parametrize("world", ["c0_world.yml", "c1_world.yml", "c2_world.yml", "mix_world.yml"])
def test_loader_matches_oracle_loader(world):
    from oracle import rt_ref
    sd, _ = config.load_scene(os.path.join(SCENES, world))
    w = rt_ref.World(rt_ref.load_config(os.path.join(SCENES, world)), lambda p: [[(0, 0, 0)]])
    assert sd.desc.n_objects == len(w.objects) and sd.desc.n_lights == len(w.lights)
    assert sd.desc.max_distance == w.max_distance and sd.desc.soft_shadow_exponent == w.soft_shadow_exponent
    kinds = {"Sphere": RTX_SPHERE, "Plane": RTX_PLANE, "Box": RTX_BOX}
    for d, o in zip(sd.objects, w.objects):
        assert d.type == kinds[type(o).__name__]
        assert list(d.diffuse_rate) == o.diffuse_rate.to_a()
        assert list(d.ambient) == o.ambient.to_a()
        assert list(d.reflective_attenuation) == o.reflective_attenuation.to_a()
        assert bool(d.has_refractive_rate) == (o.refractive_rate is not None)
        if d.type == RTX_SPHERE:
            assert list(d.center) == o.center.to_a() and d.radius == o.radius
        else:
            assert list(d.point) == o.point.to_a() and list(d.front) == o.front.to_a()
    for d, l in zip(sd.lights, w.lights):
        assert list(d.position) == l.position.to_a() and d.radius == l.radius
        assert d.high_light_angle == l.high_light_angle and d.high_light_rate == l.high_light_rate


def test_duplicate_keys_last_wins():
    """config/world.yml's front wall repeats keys; YAML (Psych and PyYAML) keeps the last."""
    sd, _ = config.load_scene(os.path.join(SCENES, "c0_world.yml"))
    wall = sd.objects[1]
    assert list(wall.diffuse_rate) == [0.6, 0.6, 0.6]
    assert list(wall.reflective_attenuation) == [0.39, 0.39, 0.39]
    assert list(wall.ambient) == [0.01, 0.01, 0.01]


@pytest.mark.skipif(not os.path.exists(os.path.join(REFERENCE, "config", "world.yml")),
                    reason="reference checkout not present (GPU box)")
def test_reference_world_yml_equals_restated_c0():
    ref = config.load_yaml(os.path.join(REFERENCE, "config", "world.yml"))
    ours = config.load_yaml(os.path.join(SCENES, "c0_world.yml"))
    for a, b in zip(ref["world_objects"], ours["world_objects"]):
        pa, pb = dict(a["properties"]), dict(b["properties"])
        ta, tb = pa.pop("texture_file_path", None), pb.pop("texture_file_path", None)
        assert pa == pb and a["type"] == b["type"]
        if ta == "./textures/RubyOnRails.png":      # the reference's texture, used as-is
            assert tb == ta
            assert open(os.path.join(REFERENCE, "textures", "RubyOnRails.png"), "rb").read() == \
                open(os.path.join(SCENES, "textures", "RubyOnRails.png"), "rb").read()
    assert ref["lights"] == ours["lights"]
    assert ref["max_distance"] == ours["max_distance"]
    cam_ref = config.load_yaml(os.path.join(REFERENCE, "config", "camera.yml"))
    cam_ours = config.load_yaml(os.path.join(SCENES, "camera.yml"))
    assert {k: float(v) if not isinstance(v, tuple) else v for k, v in cam_ref.items()} == \
        {k: float(v) if not isinstance(v, tuple) else v for k, v in cam_ours.items()}


def test_float_without_dot_is_float(tmp_path):
    p = tmp_path / "c.yml"
    p.write_text("a: 1e-5\nb: 3\nc: [1, 2, 3]\nd: [1, 2]\ne: {f: [0, 0.5, 1]}\n")
    c = config.load_yaml(str(p))
    assert c["a"] == 1e-5 and isinstance(c["a"], float) and c["b"] == 3
    assert c["c"] == (1.0, 2.0, 3.0) and c["d"] == [] and c["e"]["f"] == (0.0, 0.5, 1.0)


@pytest.mark.parametrize("drop,kind", [("refractive_rate", "Sphere"), ("reflective_attenuation", "Sphere"),
                                       ("ambient", "Plane"), ("center", "Sphere")])
def test_missing_required_property_raises(tmp_path, drop, kind):
    src = open(os.path.join(SCENES, "c1_world.yml")).read().splitlines()
    out, in_kind = [], None
    for line in src:
        m = re.match(r"\s*- type: (\w+)", line)
        if m:
            in_kind = m.group(1)
        if in_kind == kind and line.strip().startswith(drop + ":"):
            continue
        out.append(line)
    p = tmp_path / "w.yml"
    p.write_text("\n".join(out) + "\n")
    with pytest.raises(config.ConfigError, match=drop):
        config.load_scene(str(p))


def test_camera_desc():
    _, cam = config.load_scene(os.path.join(SCENES, "c2_world.yml"), os.path.join(SCENES, "c2_camera.yml"))
    assert (cam.width, cam.height, cam.pre_sample_times, cam.max_sample_times, cam.trace_depth) == (1920, 1080, 4, 4, 5)
    assert cam.image_distance == 0.01714573877962683 and cam.focal_distance == 0.017


# ------------------------------------------------------------------ png
@pytest.mark.parametrize("mode,bits", [("RGB", 8), ("RGBA", 8), ("L", 8), ("P", 8), ("RGBA", 16), ("RGB", 16),
                                       ("LA", 8)])
def test_png_decoder_matches_pillow(tmp_path, mode, bits):
    from PIL import Image
    rs = np.random.RandomState(3)
    h, w = 13, 17
    p = str(tmp_path / "t.png")
    if bits == 16:
        a = rs.randint(0, 65536, (h, w, 4 if mode == "RGBA" else 3)).astype(np.uint16)
        png.write(p, a)
        ref = (a[:, :, :3] >> 8).astype(np.uint8)
    else:
        a = rs.randint(0, 256, (h, w, 4)).astype(np.uint8)
        im = Image.fromarray(a, "RGBA").convert(mode)
        im.save(p, optimize=True)
        ref = np.asarray(Image.open(p).convert("RGB"))
    assert np.array_equal(png.decode_rgb8(p), ref)


def test_png_texture_fixture_matches_pillow():
    from PIL import Image
    for name in ("rails_synth.png", "checker.png", "RubyOnRails.png"):
        p = os.path.join(SCENES, "textures", name)
        assert np.array_equal(png.decode_rgb8(p), np.asarray(Image.open(p).convert("RGB")))


def test_reference_texture_decode_is_high_byte():
    """texture.rb:12-20: Vec3((pixel.red >> 8) / 256.0): the reference's own 16-bit
    RubyOnRails.png decodes to the high byte of every 16-bit sample."""
    import struct
    import zlib
    p = os.path.join(SCENES, "textures", "RubyOnRails.png")
    data = open(p, "rb").read()
    w, h, depth, ctype = struct.unpack(">IIBB", data[16:26])
    assert (w, h, depth, ctype) == (122, 158, 16, 6)
    got = png.decode_rgb8(p)
    # independent decode of the first row (filter type + 16-bit big-endian RGBA)
    pos, idat = 8, b""
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        if data[pos + 4:pos + 8] == b"IDAT":
            idat += data[pos + 8:pos + 8 + n]
        pos += 12 + n
    raw = zlib.decompress(idat)
    ftype, line = raw[0], bytearray(raw[1:1 + w * 8])
    assert ftype in (0, 1)                           # row 0: None or Sub (no row above)
    if ftype == 1:
        for i in range(8, len(line)):                # Sub: + the byte one pixel (8 B) left
            line[i] = (line[i] + line[i - 8]) & 0xFF
    row0 = np.frombuffer(bytes(line), ">u2").reshape(w, 4)
    assert np.array_equal(got[0], (row0[:, :3] >> 8).astype(np.uint8))


# ------------------------------------------------------------------ C-ABI
def test_capi_exports_every_declared_symbol():
    import ctypes
    from raytracing_rb_amd import _abi
    hdr = open(os.path.join(ROOT, "include", "rtx.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    declared = set(re.findall(r"\b(rtx_[a-z0-9_]+)\s*\(", hdr))
    assert len(declared) > 30
    lib = ctypes.CDLL(_abi.LIB_PATH)
    missing = [s for s in sorted(declared) if not hasattr(lib, s)]
    assert not missing, missing
    assert declared == {n for n, _, _ in _abi.SIGNATURES}, "ctypes mirror out of sync with rtx.h"


def test_capi_struct_layout_matches_header():
    """Compile a tiny C program against include/rtx.h and compare sizeof/offsetof with ctypes."""
    import ctypes
    import subprocess
    from raytracing_rb_amd import _abi
    checks = {"rtx_object_desc": (_abi.ObjectDesc, ["refractive_rate", "center", "texture_vertical_scale"]),
              "rtx_light_desc": (_abi.LightDesc, ["high_light_angle"]),
              "rtx_scene_desc": (_abi.SceneDesc, ["objects", "textures"]),
              "rtx_camera_desc": (_abi.CameraDesc, ["variant_threshold", "monte_carlo_diffusion_times"]),
              "rtx_texture_desc": (_abi.TextureDesc, ["rgb"])}
    src = ['#include <stdio.h>\n#include <stddef.h>\n#include "rtx.h"\nint main(){']
    for cname, (_, fields) in checks.items():
        src.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f in fields:
            src.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    src.append("return 0;}")
    d = os.path.join(ROOT, "build")
    os.makedirs(d, exist_ok=True)
    c = os.path.join(d, "layout.c")
    open(c, "w").write("\n".join(src))
    exe = os.path.join(d, "layout")
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, c], check=True)
    got = dict(l.split() for l in subprocess.run([exe], capture_output=True, text=True).stdout.splitlines())
    for cname, (ct, fields) in checks.items():
        assert int(got[cname]) == ctypes.sizeof(ct), cname
        for f in fields:
            assert int(got["%s.%s" % (cname, f)]) == getattr(ct, f).offset, (cname, f)


# ------------------------------------------------------------------ sharding
@pytest.mark.parametrize("H,tr,n", [(1080, 8, 8), (1080, 16, 8), (1080, 8, 3), (37, 8, 2), (5, 8, 4), (1080, 8, 1)])
def test_tiles_cover_every_row_once(H, tr, n):
    seen = np.concatenate([tiles.rank_rows(H, tr, r, n) for r in range(n)])
    seen = seen[seen >= 0]
    assert np.array_equal(np.sort(seen), np.arange(H))
    src, dst = tiles.unpack_index(H, tr, n)
    assert np.array_equal(np.sort(dst), np.arange(H)) and len(src) == H


def test_unpack_roundtrip():
    H, W, tr, n = 45, 7, 8, 3
    frame = np.random.RandomState(1).rand(H, W, 3)
    R = tiles.rows_per_rank(H, tr, n)
    packed = np.zeros((n * R, W, 3))
    for r in range(n):
        y = tiles.rank_rows(H, tr, r, n)
        packed[r * R:(r + 1) * R][y >= 0] = frame[y[y >= 0]]
    assert np.array_equal(tiles.unpack(packed, H, tr, n), frame)


def _gloo_worker(rank, world, port, H, W, tr, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.c_oracle import Oracle
    sd, cd = config.load_scene(os.path.join(SCENES, "c2_world.yml"), os.path.join(SCENES, "c2_camera.yml"),
                               camera_overrides={"width": W, "height": H})
    o = Oracle(sd, cd)
    df = tiles.DistributedFrame(W, H, tr, rank, world, "cpu")
    ys = tiles.rank_rows(H, tr, rank, world)
    for i, y in enumerate(ys):                # this rank's tiles, rendered by the CPU oracle
        if y >= 0:
            fb, st, rc = o.render(0, int(y), W, int(y) + 1)
            df.packed[i] = torch.from_numpy(fb[0])
    frame = df.gather()
    if rank == 0:
        q.put(frame.numpy().copy())
    dist.destroy_process_group()


def test_distributed_gather_gloo_world2():
    """world_size-2 tile sharding + the one gather, on CPU (gloo): the frame is
    bit-identical to a single-process render."""
    import multiprocessing as mp
    import socket
    H, W, tr = 20, 12, 8
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, H, W, tr, q)) for r in range(2)]
    for p in ps:
        p.start()
    frame = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle.c_oracle import Oracle
    sd, cd = config.load_scene(os.path.join(SCENES, "c2_world.yml"), os.path.join(SCENES, "c2_camera.yml"),
                               camera_overrides={"width": W, "height": H})
    ref, st, rc = Oracle(sd, cd).render()
    assert np.array_equal(frame, ref)


# ------------------------------------------------------------------ cost-balanced tile lists
@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_lpt_plan_covers_every_tile_once_and_balances(n):
    costs = np.random.default_rng(n).integers(1, 1000, 135)
    plan = tiles.lpt_plan(costs, n)
    assert len(plan) == n and len({len(l) for l in plan}) == 1
    real = sorted(t for l in plan for t in l if t < len(costs))
    assert real == list(range(len(costs)))
    loads = [sum(int(costs[t]) for t in l if t < len(costs)) for l in plan]
    # LPT: no rank exceeds the mean by more than the largest single tile
    assert max(loads) <= sum(loads) / n + costs.max()
    assert plan == tiles.lpt_plan(costs, n)      # deterministic: every rank computes the same plan


def test_row_tile_costs_sums_bands():
    tr8 = np.arange(6 * 4).reshape(6, 4)          # 6 bands of 8x8 tiles, 4 across
    assert list(tiles.row_tile_costs(tr8, 8)) == list(tr8.sum(axis=1))
    assert list(tiles.row_tile_costs(tr8, 16)) == [tr8[0:2].sum(), tr8[2:4].sum(), tr8[4:6].sum()]
    with pytest.raises(ValueError):
        tiles.row_tile_costs(tr8, 4)


def _gloo_plan_worker(rank, world, port, H, W, tr, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ntiles = (H + tr - 1) // tr
    plan = tiles.lpt_plan(np.arange(ntiles)[::-1] % 5 + 1, world)
    df = tiles.DistributedFrame(W, H, tr, rank, world, "cpu", plan=plan)
    for k, t in enumerate(plan[rank]):          # a stub render: each row holds its image row index
        for j in range(tr):
            df.packed[k * tr + j] = float(t * tr + j)
    frame = df.gather()
    if rank == 0:
        q.put(frame.numpy().copy())
    dist.destroy_process_group()


def test_distributed_gather_of_an_lpt_plan_gloo_world3():
    """Per-rank tile lists (lpt_plan) instead of round-robin tiles: the gather's
    unpack puts every packed row at its image row."""
    import multiprocessing as mp
    import socket
    H, W, tr, world = 45, 3, 8, 3
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_plan_worker, args=(r, world, port, H, W, tr, q)) for r in range(world)]
    for p in ps:
        p.start()
    frame = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(frame[:, :, 0], np.repeat(np.arange(H, dtype=np.float64)[:, None], W, 1))


def _gloo_pipeline_worker(rank, world, port, H, W, tr, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    df = tiles.DistributedFrame(W, H, tr, rank, world, "cpu", buffers=2)
    ys = torch.as_tensor(tiles.rank_rows(H, tr, rank, world), dtype=torch.float64)
    frames, pending = [], []
    for i in range(5):                          # bench.py's pipelined step: frame i = row index + 1000 i
        df.packed.copy_((ys + 1000.0 * i)[:, None, None].expand_as(df.packed))
        if pending:
            f = df.gather_finish(pending.pop())
            if rank == 0:
                frames.append(f.clone().numpy())
        pending.append(df.gather_start())
    f = df.gather_finish(pending.pop())
    if rank == 0:
        frames.append(f.clone().numpy())
        q.put(frames)
    dist.destroy_process_group()


def test_distributed_pipelined_gather_gloo_world3():
    """Double-buffered asynchronous gather (frame i's gather overlaps frame
    i + 1's render): every gathered frame is the one its ranks rendered."""
    import multiprocessing as mp
    import socket
    H, W, tr, world = 37, 5, 8, 3
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_pipeline_worker, args=(r, world, port, H, W, tr, q)) for r in range(world)]
    for p in ps:
        p.start()
    frames = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(frames) == 5
    rows = np.repeat(np.arange(H, dtype=np.float64)[:, None], W, 1)
    for i, f in enumerate(frames):
        for c in range(3):
            assert np.array_equal(f[:, :, c], rows + 1000.0 * i), i


def test_bench_launches_its_own_ranks_gloo_stub():
    """bench.py --gpus 2 without torch.distributed.run starts the 2 ranks itself
    (launch_ranks), the world size is checked, the one gather runs and rank 0
    prints the JSON line (stub tile render on CPU/gloo: no GPU, no librtx)."""
    import json
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub", "--gpus", "2", "--steps", "2"],
                         capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["stub"] and line["frame_rows_ok"]


def test_bench_refuses_mismatched_world_size():
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--stub", "--gpus", "2"],
                         capture_output=True, text=True, timeout=120, env=env)
    assert out.returncode == 2 and "refusing" in out.stderr


def test_library_is_the_build_of_this_tree():
    """librtx.so embeds the sha of the sources it was built from (rtx_build_id);
    the loader refuses an in-tree library built from other sources."""
    from raytracing_rb_amd import _abi, _build
    lib = _abi.load_library()
    assert lib.rtx_build_id().decode() == _build.source_sha()


def test_native_lpt_plan_matches_python():
    """rtx_lpt_plan (host C++, used by the CLI's `rtx N`) == tiles.lpt_plan,
    ties included (equal costs, zeros, more ranks than tiles)."""
    from raytracing_rb_amd.runtime import lpt_plan_native
    from raytracing_rb_amd.tiles import lpt_plan
    rs = np.random.RandomState(3)
    for n_tiles, ranks in ((135, 8), (136, 8), (23, 3), (5, 8), (1, 1), (64, 2)):
        for costs in (rs.randint(0, 1000, n_tiles), np.full(n_tiles, 7), rs.randint(0, 3, n_tiles)):
            assert lpt_plan_native(costs, ranks) == lpt_plan(costs, ranks), (n_tiles, ranks)

