#!/usr/bin/env python3
"""Does splitting a share into concurrently running halves on two HIP streams
pay?  (GPU box)  For N in --n: time rank 0's share of N ranks alone (one
context, one stream), then the same rows as two shares of 2N ranks (ranks 0
and N of 2N) rendered by two contexts on two streams at once.

    python tools/concur.py --scene c2 --n 1 8
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="c2")
    ap.add_argument("--n", type=int, nargs="+", default=[1, 8])
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    import numpy as np
    import torch
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import Renderer
    sd, cd = config.load_scene(os.path.join(ROOT, "scenes", a.scene + "_world.yml"),
                               os.path.join(ROOT, "scenes", a.scene + "_camera.yml"))
    W, H, TR = cd.width, cd.height, 8
    r1, r2 = Renderer(sd, cd, device=0), Renderer(sd, cd, device=0)
    s1 = torch.cuda.Stream()
    s2 = torch.cuda.Stream()
    big = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
    o1 = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
    o2 = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        return float(np.median(ts)) * 1e3

    for n in a.n:
        def alone():
            r1.render_tiles_device(big.data_ptr(), TR, 0, n, seed=1, stream=s1.cuda_stream)

        def pair():
            r1.render_tiles_device(o1.data_ptr(), TR, 0, 2 * n, seed=1, stream=s1.cuda_stream)
            r2.render_tiles_device(o2.data_ptr(), TR, n, 2 * n, seed=1, stream=s2.cuda_stream)

        def serial():
            r1.render_tiles_device(o1.data_ptr(), TR, 0, 2 * n, seed=1, stream=s1.cuda_stream)
            r2.render_tiles_device(o2.data_ptr(), TR, n, 2 * n, seed=1, stream=s1.cuda_stream)
        ta, tp, ts = timed(alone), timed(pair), timed(serial)
        print("%s n=%d  share alone %.3f ms | two halves on two streams %.3f ms | two halves one stream %.3f ms"
              % (a.scene, n, ta, tp, ts), flush=True)


if __name__ == "__main__":
    main()
