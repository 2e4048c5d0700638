#!/usr/bin/env python3
"""BASELINE.md's table, measured on the GPU box (one MI355X + its host cores):

    python tools/baseline_table.py OUT_DIR

* CPU: the C restatement of the reference (oracle/rt_oracle.c, scalar FP64,
  brute force) in the reference's fork_jobs column bands (camera.rb:53-65), one
  process per CPU this job may use; C0 and C1 full frames, C2 every 4th and C4
  every 256th column (extrapolated per pixel); median of 3 (C4: 1).
* GPU: the default engine, whole frames on the device, median of 5 (C4: 3).
* RMS vs oracle: per channel over the pixels the CPU run rendered.
* Multi-GPU: every rank's share of an N-rank tiled frame timed alone on this
  GPU, one frame at a time: every share warmed up once, then 5 rounds with
  the rank order rotated by one per round (drift spreads over all ranks),
  per-rank median; projected frame = max over ranks.  Round-robin 8-row
  tiles (rtx_render_tiles_device) and LPT tile lists by the whole frame's
  measured rays (tiles.lpt_plan, rtx_render_tile_list_device).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

CONFIGS = [  # name, world, camera, CPU column stride, CPU reps, GPU reps
    ("C0", "c0_world.yml", "c0_camera.yml", 1, 3, 5),
    ("C1", "c1_world.yml", "c1_camera.yml", 1, 3, 5),
    ("C2", "c2_world.yml", "c2_camera.yml", 4, 3, 5),
    ("C4", "c4_world.yml", "c4_camera.yml", 256, 1, 3),
]


def main():
    out_dir = sys.argv[1]
    os.makedirs(out_dir, exist_ok=True)
    import numpy as np
    import make_scenes
    make_scenes.ensure_c4()
    from bench import host_cores
    from raytracing_rb_amd import config
    from oracle.c_oracle import Oracle
    cores = host_cores()
    res = {"cores": cores, "host_cpus": os.cpu_count(), "configs": {}}
    cpu_frames = {}
    # CPU first: this process has not touched the GPU yet (fork)
    for name, w, c, stride, reps, _ in CONFIGS:
        sd, cd = config.load_scene(os.path.join(ROOT, "scenes", w), os.path.join(ROOT, "scenes", c))
        o = Oracle(sd, cd)
        ts = []
        for _ in range(reps):
            t = time.time()
            fb = o.render_fork(cores, stride)
            ts.append(time.time() - t)
        cols = np.arange(0, cd.width, stride)
        px = cols.size * cd.height
        cpu_frames[name] = (cols, fb[:, cols, :])
        res["configs"][name] = {"cpu_mpix_s": px / float(np.median(ts)) / 1e6, "cpu_sample_px": int(px),
                                "cpu_col_stride": stride, "cpu_s": float(np.median(ts))}
        print(name, "cpu", res["configs"][name], flush=True)
    import torch
    from raytracing_rb_amd.runtime import Renderer
    from raytracing_rb_amd.tiles import rows_per_rank, lpt_plan, row_tile_costs
    dev = torch.device("cuda", 0)
    for name, w, c, stride, _, greps in CONFIGS:
        sd, cd = config.load_scene(os.path.join(ROOT, "scenes", w), os.path.join(ROOT, "scenes", c))
        r = Renderer(sd, cd)
        W, H = cd.width, cd.height
        frame = torch.empty((H, W, 3), dtype=torch.float64, device=dev)
        r.render_device(frame.data_ptr())
        r.sync()

        def timed(fn, reps):
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t)
            return float(np.median(ts))
        t1 = timed(lambda: r.render_device(frame.data_ptr()), greps)
        fb = frame.cpu().numpy()
        cols, ref = cpu_frames[name]
        d = fb[:, cols, :] - ref
        e = res["configs"][name]
        e.update(gpu_ms=t1 * 1e3, gpu_mpix_s=W * H / t1 / 1e6, engine=r.engine(),
                 rms_vs_oracle=[float(v) for v in np.sqrt((d ** 2).mean(axis=(0, 1)))],
                 maxabs_vs_oracle=float(np.abs(d).max()),
                 exact_px=float(np.mean(np.all(d == 0, axis=2))))
        proj = {}
        if name in ("C2", "C4"):
            rays = r.tile_rays()                     # of the whole-frame renders above
            rounds = 5
            for n in (2, 4, 8):
                plan = lpt_plan(row_tile_costs(rays, 8), n)
                rows = max(rows_per_rank(H, 8, n), len(plan[0]) * 8)
                packed = torch.empty((rows, W, 3), dtype=torch.float64, device=dev)
                for kind in ("rr", "lpt"):
                    def share(k):
                        if kind == "rr":
                            r.render_tiles_device(packed.data_ptr(), 8, k, n)
                        else:
                            r.render_tile_list_device(packed.data_ptr(), plan[k], 8)
                    for k in range(n):
                        timed(lambda k=k: share(k), 1)      # warm-up
                    per = [[] for _ in range(n)]
                    for rnd in range(rounds):
                        for j in range(n):
                            k = (j + rnd) % n
                            per[k].append(timed(lambda k=k: share(k), 1))
                    ms = [float(np.median(v)) for v in per]
                    proj.setdefault(str(n), {})[kind] = {
                        "rank_ms": [round(v * 1e3, 4) for v in ms], "max_rank_ms": max(ms) * 1e3,
                        "rank_spread": (max(ms) - min(ms)) / max(ms), "projected_speedup": t1 / max(ms),
                        "projected_mpix_s": W * H / max(ms) / 1e6}
            e["projection"] = proj
        print(name, "gpu", {k: v for k, v in e.items() if not k.startswith("cpu")}, flush=True)
        r.close()
    with open(os.path.join(out_dir, "baseline_table.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
