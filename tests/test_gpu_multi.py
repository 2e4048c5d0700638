"""The multi-GPU frame step (C3: Camera#render_fork + fork_jobs replaced by
round-robin row tiles and one RCCL gather, camera.rb:41-68, fork_jobs.rb:1-33)
run on a GPU as far as one GPU allows: a 1-rank RCCL (``nccl``) process group
with the gather forced (``force_collective``), two frames in flight on two
contexts and two streams, the asynchronous gather of frame i overlapping frame
i + 1's render, and the packed buffers reused after their gather.  Every
gathered frame must equal one whole-frame render bit for bit.

Only one GPU is available to these tests; the N > 1 data movement itself is
covered by the gloo tests in test_host.py and runs on hardware in the
driver's multi-GPU bench.
"""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, SCENES

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("F", [1, 2])
def test_pipelined_tiles_one_rank_rccl_gather_equals_full_render(gpu, F):
    """F frames in flight; F = 1 reuses the single packed buffer every frame, so
    each render must wait for the previous frame's gather."""
    import torch
    import torch.distributed as dist
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import Renderer
    from raytracing_rb_amd.tiles import PipelinedTiles
    sd, cd = config.load_scene(os.path.join(SCENES, "c2_world.yml"), os.path.join(SCENES, "c2_camera.yml"),
                               camera_overrides={"width": 320, "height": 181})
    env = {"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_port()), "RANK": "0", "WORLD_SIZE": "1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    dist.init_process_group("nccl", device_id=gpu)
    try:
        K = 5
        streams = [torch.cuda.Stream(gpu) for _ in range(F)]
        rs = [Renderer(sd, cd, device=0) for _ in range(F)]
        for r in rs:
            r.set_option("lv_streams", 1)
        frames = []
        pipe = PipelinedTiles(rs, streams, cd.width, cd.height, 8, 0, 1, gpu, seed=1, force_collective=True,
                              on_frame=lambda i, f: frames.append(f.clone()))
        assert pipe.df.collective
        for _ in range(K):
            pipe.step()
        pipe.drain()
        torch.cuda.synchronize(gpu)
        for j, r in enumerate(rs):
            r.sync(streams[j].cuda_stream)
        full = rs[0].render(seed=1)
        assert len(frames) == K
        for i, f in enumerate(frames):
            assert np.array_equal(f.cpu().numpy(), full), i
        for r in rs:
            r.close()
    finally:
        dist.destroy_process_group()
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_bench_force_collective_one_rank():
    """bench.py's own multi-GPU step (PipelinedTiles under a 1-rank RCCL group)
    on the full C2 frame: the timed frames are rendered and gathered, and the
    gathered frame equals a whole-frame render bit for bit (gather_check)."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-collective", "--steps", "4",
                          "--warmup", "1", "--no-cpu-baseline", "--no-projection"],
                         capture_output=True, text=True, timeout=110, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert line["gather_check"] == "bit-identical"
    rb = line["ranks"]                          # per-rank render and measured gather times
    assert len(rb["render_ms"]) == 1 and len(rb["gather_ms"]) == 1
    assert 0.0 < rb["render_ms"][0] < 100.0 and 0.0 <= rb["gather_ms"][0] < 100.0, rb
    assert line["n_gpus"] == 1 and "RCCL" in line["config"]["parallelism"]
    assert line["value"] > 0


def test_lpt_tile_lists_reassemble_bit_exactly(gpu):
    """rtx_tile_rays after a whole-frame render -> lpt_plan for 3 and 8 ranks;
    every rank's tile list rendered with rtx_render_tile_list_device and
    unpacked by the plan equals the whole frame bit for bit."""
    import torch
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import Renderer
    from raytracing_rb_amd.tiles import lpt_plan, plan_unpack_index, row_tile_costs
    sd, cd = config.load_scene(os.path.join(SCENES, "c2_world.yml"), os.path.join(SCENES, "c2_camera.yml"),
                               camera_overrides={"width": 320, "height": 181})
    r = Renderer(sd, cd, device=0)
    full = r.render(seed=1)
    rays = r.tile_rays()
    assert rays.shape == (23, 40) and rays.min() > 0       # every tile traced its camera samples at least
    for n in (3, 8):
        plan = lpt_plan(row_tile_costs(rays, 8), n)
        rows = len(plan[0]) * 8
        packed = torch.zeros((n * rows, cd.width, 3), dtype=torch.float64, device="cuda")
        for k in range(n):
            r.render_tile_list_device(packed[k * rows:(k + 1) * rows].data_ptr(), plan[k], 8, seed=1)
        torch.cuda.synchronize()
        r.sync()
        src, dst = plan_unpack_index(plan, cd.height, 8)
        frame = np.zeros_like(full)
        frame[dst] = packed.cpu().numpy()[src]
        assert np.array_equal(frame.view(np.uint64), full.view(np.uint64)), n
    r.close()


def test_bench_force_collective_lpt_plan():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-collective", "--balance", "lpt",
                          "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-projection"],
                         capture_output=True, text=True, timeout=110, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert line["gather_check"] == "bit-identical" and line["ranks"]["balance"] == "lpt"
