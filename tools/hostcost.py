#!/usr/bin/env python3
"""Host cost of enqueueing one frame vs the frame's GPU time (GPU box):
    python tools/hostcost.py [--share k/N] [--reps 20]
Prints the median wall time the render call takes to return (enqueue only,
no synchronisation) next to the median per-frame time of a synchronised run."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--share", default="")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--scene", default="c2")
    a = ap.parse_args()
    import numpy as np
    import torch
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import Renderer
    from raytracing_rb_amd.tiles import rows_per_rank
    sd, cd = config.load_scene(os.path.join(ROOT, "scenes", a.scene + "_world.yml"),
                               os.path.join(ROOT, "scenes", a.scene + "_camera.yml"))
    r = Renderer(sd, cd)
    r.set_option("lv_streams", 1)
    s = torch.cuda.current_stream()
    if a.share:
        k, n = (int(v) for v in a.share.split("/"))
        out = torch.empty((rows_per_rank(cd.height, 8, n), cd.width, 3), dtype=torch.float64, device="cuda")
        fn = lambda: r.render_tiles_device(out.data_ptr(), 8, k, n, stream=s.cuda_stream)
    else:
        out = torch.empty((cd.height, cd.width, 3), dtype=torch.float64, device="cuda")
        fn = lambda: r.render_device(out.data_ptr(), stream=s.cuda_stream)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    enq, frame = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e3)
        frame.append((t2 - t0) * 1e3)
    # back-to-back without synchronisation between frames
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("scene %s share %s: enqueue %.3f ms (median), frame %.3f ms (median, synchronised); back-to-back: "
          "enqueue %.3f ms/frame, %.3f ms/frame total" % (a.scene, a.share or "-", float(np.median(enq)),
                                                         float(np.median(frame)), (t1 - t0) * 1e3 / a.reps,
                                                         (t2 - t0) * 1e3 / a.reps), flush=True)


if __name__ == "__main__":
    main()
