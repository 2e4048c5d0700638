#!/usr/bin/env python3
"""Build kernel variants (compile-time macros) and time them on the GPU.

  python tools/variants.py build NAME=DEF1,DEF2 ...   (here, CPU)
  python tools/variants.py time [--scene c2] [--rounds 3]   (on the GPU box)
Each variant is timed in its own child process (a library is loaded once per
process); rounds are interleaved across variants (methodology rule 24).
"""
import glob, json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VDIR = os.path.join(ROOT, "_variants")       # not under build/: variants must travel to the GPU box
sys.path.insert(0, ROOT)

CHILD = r"""
import os, sys, json, torch
sys.path.insert(0, %(root)r)
from raytracing_rb_amd import config
from raytracing_rb_amd.runtime import Renderer
sd, cd = config.load_scene(os.path.join(%(root)r, 'scenes', '%(scene)s_world.yml'),
                           os.path.join(%(root)r, 'scenes', '%(scene)s_camera.yml'))
r = Renderer(sd, cd)
opts = json.loads(%(opts)r)
for k, v in opts.items(): r.set_option(k, v)
out = torch.empty((cd.height, cd.width, 3), dtype=torch.float64, device='cuda')
s = torch.cuda.current_stream()
r.render_device(out.data_ptr(), stream=s.cuda_stream); r.sync(s.cuda_stream)
ts = []
for _ in range(%(reps)d):
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(s); r.render_device(out.data_ptr(), stream=s.cuda_stream); b.record(s); b.synchronize()
    ts.append(a.elapsed_time(b))
import hashlib
print(json.dumps({'ms': sorted(ts), 'sha': hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]}))
"""

def build(specs):
    from raytracing_rb_amd import _build
    os.makedirs(VDIR, exist_ok=True)
    for spec in specs:
        name, _, defs = spec.partition("=")
        defs = [d for d in defs.split(",") if d]
        out = os.path.join(VDIR, "librtx_%s.so" % name)
        print("building", name, defs, flush=True)
        _build.build(force=True, out=out, defines=defs)

def time_all(scene="c2", rounds=3, reps=5, opts="{}"):
    libs = sorted(glob.glob(os.path.join(VDIR, "librtx_*.so")))
    res = {os.path.basename(l)[7:-3]: [] for l in libs}
    shas = {}
    for rnd in range(rounds):
        for lib in libs:
            name = os.path.basename(lib)[7:-3]
            env = dict(os.environ, RTX_LIB=lib)
            code = CHILD % dict(root=ROOT, scene=scene, reps=reps, opts=opts)
            out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            if out.returncode:
                print(name, "FAILED", out.stderr[-2000:], flush=True)
                continue
            r = json.loads(out.stdout.strip().splitlines()[-1])
            res[name].append(r["ms"][0])
            shas[name] = r["sha"]
            print("round %d %-20s %.3f ms  sha %s" % (rnd, name, r["ms"][0], r["sha"]), flush=True)
    for k, v in res.items():
        if v:
            print("SUMMARY %-20s min %.3f ms  median %.3f ms  sha %s" % (k, min(v), sorted(v)[len(v) // 2], shas.get(k)))

if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:])
    else:
        import argparse
        ap = argparse.ArgumentParser()
        ap.add_argument("cmd"); ap.add_argument("--scene", default="c2"); ap.add_argument("--rounds", type=int, default=3)
        ap.add_argument("--opts", default="{}"); ap.add_argument("--reps", type=int, default=5)
        a = ap.parse_args()
        if a.scene == "c4":
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import make_scenes
            make_scenes.ensure_c4()
        time_all(a.scene, a.rounds, reps=a.reps, opts=a.opts)
