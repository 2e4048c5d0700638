#!/usr/bin/env python3
"""Phase breakdown of k_render from a -DRTX_STAMPS=1 build (diagnostic only)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from raytracing_rb_amd import config, _abi
from raytracing_rb_amd.runtime import Renderer
scene = sys.argv[1] if len(sys.argv) > 1 else "c2"
ov = dict(width=960, height=540) if scene == "c4" else {}
sd, cd = config.load_scene(os.path.join(ROOT, "scenes", scene + "_world.yml"), os.path.join(ROOT, "scenes", scene + "_camera.yml"), camera_overrides=ov)
r = Renderer(sd, cd)
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    r.set_option(k, int(v))
lib = _abi.load_library()
out = torch.empty((cd.height, cd.width, 3), dtype=torch.float64, device="cuda")
r.render_device(out.data_ptr()); r.sync()
st = (ctypes.c_ulonglong * 16)()
lib.rtxdbg_read_stamps(st, 1)
r.render_device(out.data_ptr()); r.sync()
lib.rtxdbg_read_stamps(st, 1)
tA, tB, tC, tD, iters, waves, wexact, lexact, w0, w1, busy, lanes, live, dry0, dry1, maxitem = list(st)[:16]
tot = tA + tB + tC + tD
print("waves %d  iterations/wave %.1f" % (waves, iters / waves))
for n, v in (("A fetch/pop/lens/highlight", tA), ("B query (object walk)", tB), ("C hit_info/lights", tC), ("D shade_finish", tD)):
    print("%-28s %5.1f%%  %.0f cycles/wave  %.0f cycles/iteration" % (n, 100 * v / tot, v / waves, v / iters))
print("of A: work refill (global atomic) %.1f%% of all, %.0f cycles/iteration" % (100 * wexact / tot, wexact / iters))
span = w1 - w0
print("kernel span %.3f ms (100 MHz clock); lanes %d" % (span / 1e5, lanes))
print("lane busy (start -> pool empty) %.1f%% of lanes x span; lane resident %.1f%%" % (
    100.0 * busy / (lanes * span), 100.0 * live / (lanes * span)))
print("pool empty at %.1f%% of the span; last lane done at %.1f%%; longest item %.3f ms" % (
    100.0 * (dry0 - w0) / span, 100.0 * (dry1 - w0) / span, maxitem / 1e5))
