#!/usr/bin/env python3
"""Headline benchmark: Mpixels/s at 1920x1080, 4x AA, depth 5, 64 spheres (C2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
                    [--workload c2|c4] [--emulate-rank k/N] [--no-projection] [--inflight F]

One step = one complete C2 frame (BASELINE.json configs[2]): 1920x1080 pixels,
Camera#render_at with pre = max = 4 samples, trace_depth 5, 64 spheres + ground
plane + area light, counter RNG seed 1, scene resident in HBM before timing.
Frames are pipelined (`--inflight F`, default 2): F independent contexts on F
streams, frame i on context i mod F, so one frame's last levels and tree
reduction overlap the next frame's first levels.  Every one of the K timed
frames is rendered completely (and, multi-GPU, gathered to rank 0) inside the
timed region; `ms_per_step` is the time per frame of that stream of frames,
`frame_latency_ms` one frame rendered alone, as the library renders one frame by default (`frame_latency_parts` parts on the context's streams).

Multi-GPU (C3, BASELINE.json configs[3]): one process per GPU.  Under
torch.distributed.run (WORLD_SIZE set) this process is one rank; with
`--gpus N > 1` and no WORLD_SIZE it launches the N ranks itself
(torch.distributed.run as a child process, started before this process makes
any GPU call) and exits with their status.  A world size that differs from
--gpus is an error, never a silent 1-GPU run.  The frame is split into 8-row
tiles dealt round-robin over the ranks (rtx_render_tiles_device, the
replacement of camera.rb:41-68 / fork_jobs.rb:1-33) and gathered to rank 0
with ONE RCCL gather per frame: strong scaling of the C2 frame.

`--emulate-rank k/N` times rank k's share of an N-rank frame on one GPU;
the default 1-GPU run also reports `projection`: every rank's share for
N = 2, 4, 8 timed on this GPU, the max over ranks, and the projected speedup.

Prints ONE JSON line on rank 0 (contract in the task statement), including
`roofline` (FP64 VALU: hardware FP64 rate from the committed PMC pass of this
kernel build vs 78.6 TF; measured HBM traffic; the reference-work rate and the
HBM-write fraction beside it) and `cpu_baseline` (the C restatement of the
reference with its fork_jobs column bands, on the host cores, bounded sample).
"""

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    "c2": ("c2_world.yml", "c2_camera.yml",
           "C2: 64 spheres + ground plane + area light (soft shadows), 1920x1080, 4x AA, depth 5"),
    "c4": ("c4_world.yml", "c4_camera.yml",
           "C4: 4096 random spheres + textured ground + area light, 3840x2160, 8x AA, depth 8"),
}
WORLD = os.path.join(ROOT, "scenes", WORKLOADS["c2"][0])
CAMERA = os.path.join(ROOT, "scenes", WORKLOADS["c2"][1])
WORKLOAD = WORKLOADS["c2"][2]
METRIC = "Mpixels/sec at 1920×1080, 4× AA, depth 5; per-channel RMS vs ref"
TILE_ROWS = 8
PROJECT_N = (2, 4, 8)
XGMI_LINK_GBS = 153.0            # one xGMI link (MI355X_MICROARCH.md); the gather's estimate only


def host_cores():
    """CPUs this job may use: the affinity mask, capped by a cgroup CPU quota."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = max(1, min(n, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(col_stride=4):
    """Time the C restatement (fork per core, camera.rb:54 column bands) on a
    strided column sample, in a child process started before any GPU init."""
    nprocs = host_cores()
    if WORLD.endswith("c4_world.yml"):
        col_stride = col_stride * 64           # C4: ~300x the work per pixel; keep the sample ~10-30 s of CPU
    code = (
        "import sys, time, json; sys.path.insert(0, %r)\n"
        "from raytracing_rb_amd import config\n"
        "from oracle.c_oracle import Oracle\n"
        "sd, cd = config.load_scene(%r, %r)\n"
        "o = Oracle(sd, cd)\n"
        "t = time.time(); o.render_fork(%d, %d); dt = time.time() - t\n"
        "cols = len(range(0, cd.width, %d))\n"
        "print(json.dumps({'dt': dt, 'px': cols * cd.height}))\n"
    ) % (ROOT, WORLD, CAMERA, nprocs, col_stride, col_stride)
    try:
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600, check=True)
        r = json.loads(out.stdout.strip().splitlines()[-1])
    except Exception as e:  # a reported baseline only: never fail the bench on it
        return {"value": None, "unit": "Mpixels/s", "cores": nprocs, "kind": "port",
                "sample": "failed: %s" % (str(e)[:200],)}
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        pass
    return {"value": round(r["px"] / r["dt"] / 1e6, 5), "unit": "Mpixels/s", "cores": nprocs, "kind": "port",
            "host_cpus": os.cpu_count(),
            "sample": "every %dth column of the %s frame (%d px), %d forked processes (one per CPU this job may "
                      "use: affinity mask / cgroup quota) with camera.rb:54 column bands; %.1f s wall; CPU: %s"
                      % (col_stride, WORKLOAD.split(":")[0], r["px"], nprocs, r["dt"], model)}


FIXTURES = {"c2": ("c2_full_columns64.npz", "c2_world.yml"), "c4": ("c4_full_columns256.npz", "c4_world.yml")}


def fixture_parity(frame, workload):
    """Per-channel RMS, max |delta|, bit-exact fraction and max u8 difference of a
    rendered full-size frame (torch, device) against the committed C-oracle
    fixture columns (tests/golden/make_golden.py; the test tolerance of
    DESIGN.md §6: RMS <= 1e-4).  Bytes as array_to_color (camera.rb:153-156):
    trunc(min(256 c, 255))."""
    import hashlib
    import numpy as np
    name, world = FIXTURES[workload]
    path = os.path.join(ROOT, "tests", "golden", name)
    z = np.load(path)
    with open(os.path.join(ROOT, "scenes", world), "rb") as f:
        if str(z["scene_sha"]) != hashlib.sha256(f.read()).hexdigest():
            return {"fixture": "tests/golden/" + name, "error": "scene differs from the fixture's"}
    cols = z["columns"]
    got = frame[:, cols.tolist(), :].cpu().numpy()
    ref = z["frame"]
    if got.shape != ref.shape:
        return {"fixture": "tests/golden/" + name, "error": "shape %s vs %s" % (got.shape, ref.shape)}
    d = got - ref
    u8 = lambda a: np.trunc(np.minimum(a * 256.0, 255.0)).astype(np.int64)
    rms = np.sqrt((d ** 2).mean(axis=(0, 1)))
    return {"fixture": "tests/golden/" + name, "columns": int(len(cols)), "pixels": int(ref.shape[0] * len(cols)),
            "frame": "the last timed frame", "rms": [float("%.3g" % v) for v in rms],
            "max_abs": float("%.3g" % np.abs(d).max()),
            "bit_exact_frac": round(float(np.all(d == 0, axis=2).mean()), 6),
            "u8_max": int(np.abs(u8(got) - u8(ref)).max()), "tolerance_rms": 1e-4,
            "pass": bool((rms <= 1e-4).all())}


def launch_ranks(args):
    """--gpus N > 1 without torch.distributed.run: start the N ranks as a child
    torch.distributed.run (this process never touches the GPU) and return its status."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def pmc_profile(workload, engine):
    """The committed PMC pass of this kernel build (tools/pmc_json.py), or None."""
    from raytracing_rb_amd import roofline
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % workload)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        pm = json.load(f)
    stale = pm.get("source_sha") != roofline.kernel_source_sha() or pm.get("engine") != engine
    return pm, stale


def stub_main(args, world, rank):
    """Test-only (tests/test_host.py): the rank plumbing of the multi-GPU bench on
    CPU — ranks launched by launch_ranks, a gloo group, a stub tile "render" that
    writes each packed row's image row index, the one gather, the JSON line.
    No GPU and no librtx are touched; the JSON says "stub": true."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from raytracing_rb_amd.tiles import DistributedFrame, rank_rows
    W, H = 40, 37
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus
    df = DistributedFrame(W, H, TILE_ROWS, rank, world, "cpu", buffers=2)
    ys = torch.as_tensor(rank_rows(H, TILE_ROWS, rank, world), dtype=torch.float64)
    t0 = time.perf_counter()
    pending, frame = [], None
    for _ in range(args.steps):                # the GPU bench's pipelined step
        df.packed.copy_(ys[:, None, None].expand_as(df.packed))
        if pending:
            frame = df.gather_finish(pending.pop())
        pending.append(df.gather_start())
    frame = df.gather_finish(pending.pop())
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    if rank == 0:
        ok = bool(np.array_equal(frame[:, :, 0].numpy(), np.repeat(np.arange(H, dtype=np.float64)[:, None], W, 1)))
        print(json.dumps({"metric": METRIC, "value": W * H * args.steps / elapsed / 1e6, "unit": "Mpixels/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "stub": True,
                          "frame_rows_ok": ok}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-projection", action="store_true")
    ap.add_argument("--emulate-rank", default=None, metavar="k/N",
                    help="time rank k's share of an N-rank tiled frame on this one GPU")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2",
                    help="c2: the metric's configuration (default); c4: the 4096-sphere stress scene")
    ap.add_argument("--bvh", type=int, default=1, help="sphere walk: 0 ordered linear, 1 auto, 2 hierarchy")
    ap.add_argument("--option", action="append", default=[], metavar="KEY=VALUE",
                    help="extra rtx_set_option before timing (experiments)")
    ap.add_argument("--inflight", type=int, default=2,
                    help="frames in flight: F contexts, each on its own stream, render consecutive frames "
                         "(frame i on context i mod F; every frame complete, and gathered, inside the timed "
                         "region); 1 = one frame at a time")
    ap.add_argument("--force-collective", action="store_true",
                    help="run the multi-GPU step (tile shares, RCCL gather to rank 0, pipelined) even with one "
                         "rank: a 1-rank RCCL group (evidence that the C3 path runs on ROCm)")
    ap.add_argument("--tile-rows", type=int, default=TILE_ROWS,
                    help="rows per round-robin tile of a rank's share (default %d)" % TILE_ROWS)
    ap.add_argument("--balance", choices=("auto", "rr", "lpt"), default="auto",
                    help="multi-GPU tile split: rr = round-robin tiles; lpt = tile lists balanced by the rays each "
                         "tile traced in one whole-frame render (rtx_tile_rays, longest processing time first); "
                         "auto = lpt from 8 ranks (r08a projection: 8 ranks 5.99x rr / 6.11x lpt, 2 and 4 ranks "
                         "within 1 %%, rr slightly ahead), else rr")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)   # CPU test of the rank plumbing
    args = ap.parse_args()
    globals()["TILE_ROWS"] = args.tile_rows      # every share / gather of this run
    if args.balance == "lpt" and args.tile_rows % 8:
        ap.error("--balance lpt needs --tile-rows a multiple of 8 (its costs are the 8x8 tiles' ray counts)")
    if args.balance == "auto":               # (lpt's costs come in 8x8 tiles: rr for other tile heights)
        args.balance = "lpt" if args.gpus >= 8 and args.tile_rows % 8 == 0 else "rr"

    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        sys.exit(launch_ranks(args))
    world = int(world_env or "1")
    if world != args.gpus:
        print("bench.py: WORLD_SIZE=%d but --gpus %d: refusing to measure a different GPU count"
              % (world, args.gpus), file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub:
        return stub_main(args, world, rank)

    global WORLD, CAMERA, WORKLOAD, METRIC
    if args.workload != "c2":
        if args.workload == "c4":
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import make_scenes
            make_scenes.ensure_c4()
        WORLD = os.path.join(ROOT, "scenes", WORKLOADS[args.workload][0])
        CAMERA = os.path.join(ROOT, "scenes", WORKLOADS[args.workload][1])
        WORKLOAD = WORKLOADS[args.workload][2]
        METRIC = "Mpixels/sec at 3840×2160, 8× AA, depth 8 (C4, 4096 spheres)"

    emulate = None
    if args.force_collective and args.emulate_rank:
        print("bench.py: --force-collective and --emulate-rank exclude each other", file=sys.stderr)
        sys.exit(2)
    if args.emulate_rank:
        k, n = (int(v) for v in args.emulate_rank.split("/"))
        if world != 1 or not (0 <= k < n):
            print("bench.py: --emulate-rank k/N needs one process and 0 <= k < N", file=sys.stderr)
            sys.exit(2)
        emulate = (k, n)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and emulate is None:
        cpu = cpu_baseline()              # before this process touches the GPU

    import numpy as np
    import torch
    import torch.distributed as dist

    from raytracing_rb_amd import config, roofline
    from raytracing_rb_amd.runtime import Renderer
    from raytracing_rb_amd.tiles import PipelinedTiles, lpt_plan, row_tile_costs, rows_per_rank

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    # The frames' streams are this process's first streams, before RCCL makes
    # its own, so every rank sets up its frames exactly as the measured 1-GPU
    # run does (a second pair of contexts and streams in one
    # process was measured to run its two frames one after the other).
    F = max(1, args.inflight)
    frame_streams = [torch.cuda.Stream(dev) for _ in range(F)] if F > 1 else None
    if world > 1 or args.force_collective:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:                     # the multi-rank step under a 1-rank RCCL group
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            if "MASTER_PORT" not in os.environ:
                with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
                    so.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(so.getsockname()[1])
        dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != args.gpus:
            print("bench.py: process group has %d ranks, --gpus %d" % (dist.get_world_size(), args.gpus),
                  file=sys.stderr)
            sys.exit(2)

    scene, cam = config.load_scene(WORLD, CAMERA)
    W, H = cam.width, cam.height
    # F frames in flight: F independent contexts (own level buffers, own
    # camera copy), each on its own stream; frame i renders on context i mod F,
    # so frame i + 1's levels fill the CUs frame i's last levels and tree
    # reduction leave idle.  Each context then renders its frame as one part
    # (lv_streams = 1: the overlap comes from the other frame; two parts per
    # frame on top of that measured slower, profiles/r03x).
    rs = []
    parts_default = None
    for _ in range(F):
        rc = Renderer(scene, cam, device=local_rank)
        rc.set_option("bvh", args.bvh)
        parts_default = rc.get_option("lv_streams")
        if F > 1:
            rc.set_option("lv_streams", 1)
        for kv in args.option:
            key, val = kv.split("=", 1)
            rc.set_option(key, int(val))
        rs.append(rc)
    r = rs[0]
    engine = r.engine()
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    streams = [stream] if F == 1 else frame_streams
    counter = [0]

    def next_ctx():
        j = counter[0] % F
        counter[0] += 1
        return j

    packed_for = {}

    def share_render(k, n, j):
        if (k, n, j) not in packed_for:
            packed_for[(k, n, j)] = torch.empty((rows_per_rank(H, TILE_ROWS, n), W, 3), dtype=torch.float64,
                                                device=dev)
        rs[j].render_tiles_device(packed_for[(k, n, j)].data_ptr(), TILE_ROWS, k, n, seed=1,
                                  stream=streams[j].cuda_stream)

    def share_step(k, n):
        share_render(k, n, next_ctx())

    dist_step = world > 1 or args.force_collective
    if world == 1 and emulate is None:
        frames = [torch.empty((H, W, 3), dtype=torch.float64, device=dev) for _ in range(F)]

        def render_full(j):
            rs[j].render_device(frames[j].data_ptr(), seed=1, stream=streams[j].cuda_stream)

    if world == 1 and emulate is None and not dist_step:
        def step():
            render_full(next_ctx())
    elif world == 1 and emulate is not None:
        def step():
            share_step(*emulate)
    else:
        # Frame i renders on context / stream / packed buffer j = i mod F; its
        # gather overlaps frame i + 1's render (tiles.PipelinedTiles); drain()
        # finishes the last one before the timed region closes: all K frames
        # are rendered AND gathered inside it.
        plan = None
        if args.balance == "lpt":
            # rank 0 renders the whole frame once (outside the timed region),
            # derives the plan from its tiles' ray counts and broadcasts it: one
            # plan for every rank even if ray counts differed between ranks (a
            # re-rendered overflow sample's rays are not counted)
            if rank == 0:
                full0 = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
                rs[0].render_device(full0.data_ptr(), seed=1, stream=streams[0].cuda_stream)
                torch.cuda.synchronize(dev)
                plan = lpt_plan(row_tile_costs(rs[0].tile_rays(), TILE_ROWS), world)
                del full0
            box = [plan]
            if world > 1:
                dist.broadcast_object_list(box, src=0, device=dev)
            plan = box[0]
            assert len({len(l) for l in plan}) == 1, "LPT plan lists must be equally long (one gather size)"
        pipe = PipelinedTiles(rs, streams, W, H, TILE_ROWS, rank, world, dev, seed=1,
                              force_collective=args.force_collective, plan=plan)
        df = pipe.df
        step, drain = pipe.step, pipe.drain

    if not dist_step:
        def drain():
            pass

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local_rank])
        torch.cuda.synchronize(dev)

    def check_raises():
        for j in range(F):
            rs[j].sync(streams[j].cuda_stream)   # raises if a reference raise site fired

    for _ in range(args.warmup):
        step()
    drain()
    barrier()
    check_raises()

    # ---- timed region: exactly K steps, barrier + synchronize on both sides
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    drain()
    barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    check_raises()

    # ---- the last timed frame against the committed oracle fixture (data, not
    # the oracle): every 64th (C2) / 256th (C4) column of the full-size frame
    parity = None
    if rank == 0 and emulate is None:
        last = df.frame if dist_step else frames[(counter[0] - 1) % F]
        parity = fixture_parity(last, args.workload)

    # ---- the gathered frame equals one whole-frame render, bit for bit (rank 0)
    gather_check = None
    if dist_step and rank == 0:
        full = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
        rs[0].render_device(full.data_ptr(), seed=1, stream=stream.cuda_stream)
        torch.cuda.synchronize(dev)
        rs[0].sync(stream.cuda_stream)
        gather_check = "bit-identical" if torch.equal(full, df.frame) else "MISMATCH"
        del full

    # ---- one frame alone (latency; F = 1 semantics), outside the timed region
    # One frame alone renders as the library does by default (lv_streams parts
    # on the context's streams); the contexts of the frames in flight render one
    # part each (the other frame fills the tails), restored afterwards.
    latency_ms, latency_parts = None, None
    if world == 1 and emulate is None:
        parts_inflight = rs[0].get_option("lv_streams")
        if not any(kv.split("=", 1)[0] == "lv_streams" for kv in args.option):
            rs[0].set_option("lv_streams", parts_default)
        latency_parts = rs[0].get_option("lv_streams")
        lat = []
        for _ in range(6):
            torch.cuda.synchronize(dev)
            a = time.perf_counter()
            render_full(0)
            torch.cuda.synchronize(dev)
            lat.append((time.perf_counter() - a) * 1e3)
        latency_ms = float(np.median(lat[1:]))        # (the first: the parts' buffers allocated)
        rs[0].set_option("lv_streams", parts_inflight)

    # ---- the dominant kernel alone: HIP events on its launch stream around
    # every ray-tree kernel launch (rtx_kernel_time), outside the timed region
    r.set_option("kernel_events", 1)
    kern_ms, kern_launches = [], 0
    for _ in range(max(3, min(args.steps, 10))):
        if world == 1 and emulate is None:
            render_full(0)
        elif world == 1:
            share_render(emulate[0], emulate[1], 0)
        else:
            pipe.render_share(0, df.bufs[0])
        ms, kern_launches = r.kernel_time()
        kern_ms.append(ms)
    r.set_option("kernel_events", 0)
    kern_frame_ms = float(np.median(kern_ms))

    # ---- multi-rank step (C3): what each rank's share and the gather cost, so
    # the driver's N-GPU line explains itself: every rank renders its share
    # alone (one frame, context 0, HIP events on its stream), then the
    # ranks time the gather itself (events around a blocking dist.gather on the
    # current stream, after a barrier); rank 0 collects them.
    rank_breakdown = None
    if dist_step:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        rms_ = []
        for _ in range(3):
            ev[0].record(streams[0])
            pipe.render_share(0, df.bufs[0])
            ev[1].record(streams[0])
            ev[1].synchronize()
            rms_.append(ev[0].elapsed_time(ev[1]))
        r.sync(streams[0].cuda_stream)
        gms = []
        for _ in range(3):
            barrier()
            ev[0].record(stream)
            df.gather_finish(df.gather_start(df.bufs[0]))
            ev[1].record(stream)
            ev[1].synchronize()
            gms.append(ev[0].elapsed_time(ev[1]))
        mine = torch.tensor([float(np.median(rms_)), float(np.median(gms))], dtype=torch.float64, device=dev)
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        rank_breakdown = {"render_ms": [round(float(v[0]), 4) for v in allv],
                          "gather_ms": [round(float(v[1]), 4) for v in allv],
                          "packed_bytes_per_rank": int(df.rows * W * 3 * 8), "balance": args.balance,
                          "method": "one frame's share rendered alone on context 0 of each rank (HIP events on its "
                                    "stream, median of 3); the gather of one packed frame to rank 0 after a "
                                    "barrier (events around a blocking dist.gather on the current stream, median "
                                    "of 3; it includes waiting for the slowest rank's enqueue)"}

    # ---- 1-GPU projection of the tile-sharded frame (C3) for N = 2, 4, 8
    projection = None
    if world == 1 and emulate is None and not args.no_projection:
        def timed(fn, nf):
            """Per-frame ms of nf frames of fn(j) in flight (frame i on context i mod F)."""
            a = time.perf_counter()
            for i in range(nf):
                fn(i % F)
            torch.cuda.synchronize(dev)
            return (time.perf_counter() - a) / nf * 1e3

        def warm(fn):
            for j in range(F):
                fn(j)
            torch.cuda.synchronize(dev)
        REPS = 5
        warm(render_full)
        full_ms = float(np.median([timed(render_full, 4 * F) for _ in range(REPS)]))
        tile_rays = rs[0].tile_rays()           # rays per 8x8 tile of context 0's last whole frame

        def plan_render(tiles_k, j):
            key = ("plan", len(tiles_k), j)
            if key not in packed_for:
                packed_for[key] = torch.empty((len(tiles_k) * TILE_ROWS, W, 3), dtype=torch.float64, device=dev)
            rs[j].render_tile_list_device(packed_for[key].data_ptr(), tiles_k, TILE_ROWS, seed=1,
                                          stream=streams[j].cuda_stream)
        projection = {"method": "each rank's share rendered alone on this GPU (rtx_render_tiles_device) with the "
                                "bench's %d frame(s) in flight: every share warmed up once, then %d rounds that "
                                "time every rank's share (%d frames each) in an order rotated by one rank per "
                                "round, so clock or warm-up drift spreads over all ranks; rank_ms = per-rank "
                                "median; projected frame = max over ranks; the RCCL gather is estimated "
                                "separately at %.0f GB/s per xGMI link (the multi-GPU step overlaps it with the "
                                "next frame's render)" % (F, REPS, 4 * F, XGMI_LINK_GBS),
                      "full_frame_ms": round(full_ms, 4), "per_n": {}}
        for n in PROJECT_N:
            fns = [lambda j, k=k: share_render(k, n, j) for k in range(n)]
            for fn in fns:
                warm(fn)
            per = [[] for _ in range(n)]
            for rep in range(REPS):
                for q in range(n):
                    k = (q + rep) % n
                    per[k].append(timed(fns[k], 4 * F))
            shares = [float(np.median(v)) for v in per]
            packed_bytes = rows_per_rank(H, TILE_ROWS, n) * W * 3 * 8
            gather_ms = packed_bytes / (XGMI_LINK_GBS * 1e9) * 1e3
            mx = max(shares)
            med = float(np.median(shares))
            projection["per_n"][str(n)] = {
                "rank_ms": [round(v, 4) for v in shares], "max_rank_ms": round(mx, 4),
                "rank_spread": round((mx - min(shares)) / med, 4),
                "rank_ms_rounds": [[round(x, 4) for x in v] for v in per],
                "gather_est_ms": round(gather_ms, 4),
                "projected_speedup": round(full_ms / (mx + gather_ms), 3),
                "projected_speedup_no_gather": round(full_ms / mx, 3)}
            # the same with cost-balanced tile lists (--balance lpt): the rays
            # per tile of the whole frame, longest processing time first
            plan = lpt_plan(row_tile_costs(tile_rays, TILE_ROWS), n)
            cost = row_tile_costs(tile_rays, TILE_ROWS)
            fns = [lambda j, k=k: plan_render(plan[k], j) for k in range(n)]
            for fn in fns:
                warm(fn)
            per = [[] for _ in range(n)]
            for rep in range(REPS):
                for q in range(n):
                    k = (q + rep) % n
                    per[k].append(timed(fns[k], 4 * F))
            ls = [float(np.median(v)) for v in per]
            lmx, lmed = max(ls), float(np.median(ls))
            lgather = len(plan[0]) * TILE_ROWS * W * 3 * 8 / (XGMI_LINK_GBS * 1e9) * 1e3
            projection["per_n"][str(n)]["lpt"] = {
                "rank_ms": [round(v, 4) for v in ls], "max_rank_ms": round(lmx, 4),
                "rank_spread": round((lmx - min(ls)) / lmed, 4),
                "rank_rays": [int(sum(int(cost[t]) for t in l if t < len(cost))) for l in plan],
                "gather_est_ms": round(lgather, 4),
                "projected_speedup": round(full_ms / (lmx + lgather), 3),
                "projected_speedup_no_gather": round(full_ms / lmx, 3)}

    if rank == 0:
        counts = r.count_work(seed=1)           # one counting launch, outside the timed region
        n_share = emulate[1] if emulate else world
        px_frame = W * H if n_share == 1 else W * H / n_share
        ops_frame = roofline.algorithmic_ops(counts) / n_share
        # whole-frame rates over the timed step (every launch of the frame: level
        # kernels, resets, re-render, tree reduction), not the level kernels alone
        step_s = elapsed / args.steps
        ref_rate_tf = ops_frame / step_s / 1e12
        wr_gbs = px_frame * roofline.FRAMEBUFFER_BYTES_PER_PX / step_s / 1e9
        value = W * H * args.steps / elapsed / 1e6 if emulate is None else None
        pm, stale = pmc_profile(args.workload, engine) if (world == 1 and emulate is None) else (None, None)
        hw = roofline.hw_fp64(pm, kern_frame_ms) if pm else None
        line = {
            "metric": METRIC,
            "value": round(value, 3) if value is not None else None,
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "frames_in_flight": F,
            "frame_latency_ms": round(latency_ms, 4) if latency_ms is not None else None,
            "frame_latency_parts": latency_parts,
            # SURVEY.md §8(d)'s one-frame-at-a-time rate: W*H / frame_latency_ms
            "value_single_frame": round(W * H / latency_ms / 1e3, 3) if latency_ms else None,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": WORKLOAD, "width": W, "height": H, "samples_per_pixel": cam.pre_sample_times,
                       "trace_depth": cam.trace_depth, "objects": scene.n_objects, "seed": 1, "engine": engine,
                       "parallelism": "tiles%d-rr x %d ranks, 1 RCCL gather/frame%s"
                       % (TILE_ROWS, world, " (1-rank group, --force-collective)" if world == 1 else "")
                       if dist_step else "1 GPU"},
            "roofline": {
                "bound": "valu_fp64",
                "unit": "TFLOP/s",
                "achieved": hw["achieved_tflops"] if hw else None,
                "peak": roofline.FP64_PEAK_TFLOPS,
                "frac": hw["frac"] if hw else None,
                "traffic": (int(pm["traffic_bytes_per_frame"]) if pm and pm.get("traffic_bytes_per_frame")
                            else None),
                "kernel": pm["kernel"] if pm else "/".join(np.atleast_1d(roofline.DOMINANT_KERNEL[engine])),
                "kernel_ms_per_frame": round(kern_frame_ms, 4),
                "kernel_launches_per_frame": kern_launches,
                "kernel_avg_ms": round(kern_frame_ms / max(1, kern_launches), 4),
                "kernel_timing": "level kernels only (achieved/frac are the dominant kernel's: its FLOP over its own "
                                 "launches); HIP events around every ray-tree launch of one frame rendered alone on context 0 "
                                 "(lv_streams %d: %d launches that do not overlap); with frames in flight the "
                                 "launches of two frames overlap and each one's span stretches, so the matching "
                                 "rocprofv3 summary is the single-frame run (tools/gpu_session.sh bench: "
                                 "prof_single = bench.py --inflight 1 --option lv_streams=%d)"
                                 % (r.get_option("lv_streams"), kern_launches, r.get_option("lv_streams")),
                "hw": hw,
                "pmc_source": ({"file": "profiles/pmc_%s.json" % args.workload, "stale": stale,
                                "source_sha": pm.get("source_sha"), "session": pm.get("session")}
                               if pm else None),
                "note": "FP64 VALU-bound path (no dense contraction, no MFMA): achieved = FP64 FLOP per frame from "
                        "the committed PMC pass of this kernel build (SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64 x active "
                        "lanes) / the live HIP-event kernel time; peak = MI355X vector FP64 78.6 TF; traffic = "
                        "2 x FETCH_SIZE + WRITE_SIZE per frame (MI355X_MICROARCH.md HBM corrections)",
                "reference_work_rate": {"achieved_tflops": round(ref_rate_tf, 4),
                                        "algorithmic_fp64_ops_per_frame": int(ops_frame),
                                        "note": "the brute-force reference algorithm's ops (device-counted events "
                                                "x frozen cost table, raytracing_rb_amd/roofline.py) per second of "
                                                "the timed step (whole frame): a work rate, not a utilisation (the "
                                                "exact culls and the hierarchy skip most of these ops)"},
                "hbm_write": {"achieved": round(wr_gbs, 3), "peak": roofline.HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(wr_gbs / roofline.HBM_PEAK_GBS, 7),
                              "bytes_per_px": roofline.FRAMEBUFFER_BYTES_PER_PX,
                              "time": "ms_per_step (the whole frame)"},
            },
            "cpu_baseline": cpu,
            "work_counts": counts,
        }
        if parity is not None:
            line["parity"] = parity
        if gather_check is not None:
            line["gather_check"] = gather_check
        if rank_breakdown is not None:
            line["ranks"] = rank_breakdown
        if emulate:
            line["emulate_rank"] = {"rank": emulate[0], "nranks": emulate[1],
                                    "rank_ms_per_frame": round(elapsed / args.steps * 1e3, 4)}
        if projection:
            line["projection"] = projection
        print(json.dumps(line), flush=True)
    for rc in rs:
        rc.close()
    if dist_step:
        dist.barrier(device_ids=[local_rank])
        dist.destroy_process_group()
    if gather_check == "MISMATCH":
        sys.exit(1)


if __name__ == "__main__":
    main()
