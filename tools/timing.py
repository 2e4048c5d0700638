#!/usr/bin/env python3
"""Time k_render on one scene under several runtime options (GPU box).

    python tools/timing.py --scene c2 [--size 1920x1080] [--reps 5] '{"bvh": 0}' '{"bvh": 2}'

Prints per-option min/median kernel ms (HIP events on the launch stream) and a
hash of the frame (every option must render the same bits).
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="c2")
    ap.add_argument("--size", default="")
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--share", default="", help="k/N: time rank k's share of N ranks (--tile-rows-row tiles)")
    ap.add_argument("--tile-rows", type=int, default=8, help="rows per round-robin tile of --share")
    ap.add_argument("--dummy-streams", type=int, default=0,
                    help="with --inflight: create this many unused streams before each option set's streams")
    ap.add_argument("--keep", action="store_true", help="with --inflight: keep every option set's contexts open")
    ap.add_argument("--inflight", type=int, default=1,
                    help="frames in flight: K contexts on K streams render consecutive frames (throughput per frame)")
    ap.add_argument("opts", nargs="*")
    a = ap.parse_args()
    import torch
    from raytracing_rb_amd import config
    from raytracing_rb_amd.runtime import Renderer
    if a.scene == "c4":
        import make_scenes
        make_scenes.ensure_c4()
    ov = {}
    if a.size:
        w, h = a.size.split("x")
        ov.update(width=int(w), height=int(h))
    if a.spp:
        ov.update(pre_sample_times=a.spp, max_sample_times=a.spp)
    sd, cd = config.load_scene(os.path.join(ROOT, "scenes", a.scene + "_world.yml"),
                               os.path.join(ROOT, "scenes", a.scene + "_camera.yml"), camera_overrides=ov)
    out = torch.empty((cd.height, cd.width, 3), dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream()
    share = tuple(int(v) for v in a.share.split("/")) if a.share else None

    def render(r):
        if share:
            r.render_tiles_device(out.data_ptr(), a.tile_rows, share[0], share[1], stream=s.cuda_stream)
        else:
            r.render_device(out.data_ptr(), stream=s.cuda_stream)
    kept = []
    for o in (a.opts or ["{}"]):
        opts = json.loads(o)
        if a.inflight > 1:
            # K independent contexts (own buffers and camera copy), frame i on context/stream i mod K
            rs, ss, outs = [], [], []
            dummies = [torch.cuda.Stream() for _ in range(a.dummy_streams)]   # (hardware-queue mapping probe)
            for _ in range(a.inflight):
                r = Renderer(sd, cd)
                for k, v in opts.items():
                    r.set_option(k, v)
                rs.append(r)
                ss.append(torch.cuda.Stream())
                outs.append(torch.empty_like(out))
            def frame(i):
                k = i % a.inflight
                if share:
                    rs[k].render_tiles_device(outs[k].data_ptr(), a.tile_rows, share[0], share[1], stream=ss[k].cuda_stream)
                else:
                    rs[k].render_device(outs[k].data_ptr(), stream=ss[k].cuda_stream)
            for i in range(2 * a.inflight):
                frame(i)
            torch.cuda.synchronize()
            ts = []
            nf = 8 * a.inflight
            for _ in range(a.reps):
                t = time.perf_counter()
                for i in range(nf):
                    frame(i)
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t) * 1e3 / nf)
            if a.keep:
                kept.extend(rs)
            else:
                for r in rs:
                    r.close()
            ts.sort()
            sha = hashlib.sha1(outs[0].cpu().numpy().tobytes()).hexdigest()[:12]
            print("%-8s %-40s min %9.3f ms  median %9.3f ms  %8.2f Mpix/s  sha %s  (%d frames in flight, per frame)%s" % (
                a.scene, o, ts[0], ts[len(ts) // 2], cd.width * cd.height / ts[len(ts) // 2] / 1e3, sha, a.inflight,
                "  (share %s)" % a.share if share else ""), flush=True)
            continue
        r = Renderer(sd, cd)              # a fresh context per option set: options do not carry over
        for k, v in opts.items():
            r.set_option(k, v)
        render(r)
        r.sync(s.cuda_stream)
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            render(r)
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        r.sync(s.cuda_stream)
        st = r.level_stats() if r.engine() == "levels" else None
        r.close()
        ts.sort()
        sha = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
        print("%-8s %-40s min %9.3f ms  median %9.3f ms  %8.2f Mpix/s  sha %s%s" % (
            a.scene, o, ts[0], ts[len(ts) // 2], cd.width * cd.height / ts[len(ts) // 2] / 1e3, sha,
            "  (share %s: Mpix/s of the whole frame)" % a.share if share else ""), flush=True)
        if st:
            print("         levels: rays per level %s, redo %d, dropped %d" % (st["rays"], st["redo"], st["dropped"]),
                  flush=True)


if __name__ == "__main__":
    main()
