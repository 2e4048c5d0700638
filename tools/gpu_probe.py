#!/usr/bin/env python3
"""GPU exploration: parity vs the C oracle on small frames + timing of kernel variants."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from raytracing_rb_amd import config
from raytracing_rb_amd.runtime import Renderer
from oracle.c_oracle import Oracle

def scene(name, **ov):
    return config.load_scene(os.path.join(ROOT, "scenes", "%s_world.yml" % name),
                             os.path.join(ROOT, "scenes", "%s_camera.yml" % name if name != "c0" else "camera.yml"),
                             camera_overrides=ov)

def parity(name, **ov):
    sd, cd = scene(name, **ov)
    r = Renderer(sd, cd)
    t = time.time(); g = r.render(); tg = time.time() - t
    ref, st, rc = Oracle(sd, cd).render()
    ok = st == 0
    d = np.abs(g - ref)[ok]
    rms = np.sqrt(((g - ref)[ok] ** 2).mean(axis=0))
    exact = np.mean(np.all(g == ref, axis=2)[ok])
    print("parity %-3s %s: rc=%d oracle-errs=%d rms=%s maxabs=%.3g bit-exact-px=%.5f (gpu %.2fs)" % (
        name, ov, rc, (~ok).sum(), rms, d.max(), exact, tg), flush=True)

def timing(name, variants, reps=3, **ov):
    sd, cd = scene(name, **ov)
    r = Renderer(sd, cd)
    W, H = cd.width, cd.height
    out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    for key, val in variants:
        if key: r.set_option(key, val)
        r.render_device(out.data_ptr(), stream=s.cuda_stream); r.sync(s.cuda_stream)
        ts = []
        for _ in range(reps):
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s); r.render_device(out.data_ptr(), stream=s.cuda_stream); e1.record(s); e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = min(ts)
        print("timing %s %dx%d %s=%s: %.2f ms  %.1f Mpix/s" % (name, W, H, key, val, ms, W * H / ms / 1e3), flush=True)
    return r

if __name__ == "__main__":
    torch.cuda.init()
    print(torch.cuda.get_device_name(0), flush=True)
    parity("c1", width=192, height=108)
    parity("c0", width=96, height=54)
    parity("c2", width=128, height=72)
    timing("c1", [(None, None)])
    r = timing("c2", [("waves_per_simd", 2), ("waves_per_simd", 1), ("waves_per_simd", 3), ("waves_per_simd", 4)])
    print("counts", r.count_work(), flush=True)
