#!/usr/bin/env python3
"""Phase breakdown of k_level from a -DRTX_STAMPS=1 build, and / or the hierarchy
walks' lane occupancy from a -DRTX_WALKSTATS=1 build (diagnostic only):
    RTX_LIB=_variants/librtx_stamps.so python tools/stamps_levels.py c2 [option=value ...]
Per-wave shader-clock cycles (s_memtime) summed over every level launch of one frame;
walk counters: wave iterations of the inner-node loop and of the leaf visits, and the
lanes active in each (query_bvh)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch
from raytracing_rb_amd import config, _abi
from raytracing_rb_amd.runtime import Renderer
scene = sys.argv[1] if len(sys.argv) > 1 else "c2"
if scene == "c4":
    import make_scenes
    make_scenes.ensure_c4()
ov = dict(width=960, height=540) if scene == "c4" else {}
sd, cd = config.load_scene(os.path.join(ROOT, "scenes", scene + "_world.yml"),
                           os.path.join(ROOT, "scenes", scene + "_camera.yml"), camera_overrides=ov)
r = Renderer(sd, cd)
r.set_option("engine", 1)
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    r.set_option(k, int(v))
lib = _abi.load_library()
out = torch.empty((cd.height, cd.width, 3), dtype=torch.float64, device="cuda")
r.render_device(out.data_ptr()); r.sync()
st = (ctypes.c_ulonglong * 16)()
lv = (ctypes.c_ulonglong * 64)()
ws = (ctypes.c_ulonglong * 8)()
lib.rtxdbg_read_stamps(st, 1)
lib.rtxdbg_read_level_stamps(lv, 1)
lib.rtxdbg_read_walkstats(ws, 1)
r.render_device(out.data_ptr()); r.sync()
lib.rtxdbg_read_stamps(st, 1)
lib.rtxdbg_read_level_stamps(lv, 1)
lib.rtxdbg_read_walkstats(ws, 1)
v = list(st)
tot = sum(v[:6]) or 1          # (0 without RTX_STAMPS: e.g. a walk-counter build alone)
names = ["A claim/load/lens/highlight", "B EXTEND walk", "C hit_info/normal/cos", "D SHADOW walks + lights",
         "E (unused)", "F mask, slot alloc, children, leaf, record"]
print("waves %d  chunks %d  cycles/chunk %.0f" % (v[7], v[6], tot / max(1, v[6])))
for n, x in zip(names, v[:6]):
    print("%-38s %5.1f%%  %8.0f cycles/chunk" % (n, 100.0 * x / tot, x / max(1, v[6])))
ch = max(1, v[6])
print("lanes per chunk: with a ray %.1f, EXTEND walk %.1f, hit (shading, SHADOW walks) %.1f" % (
    v[8] / ch, v[9] / ch, v[10] / ch))
if v[13]:
    print("k_tree_finalize: %d waves, per wave %.0f cycles slice layout + %.0f cycles tree walks"
          " (of which LDS gather %.0f)" % (v[13], v[11] / v[13], v[12] / v[13], v[14] / v[13]))


print("per level: cycles per chunk by phase A-F, chunks, hit lanes per chunk")
for d in range(8):
    row = list(lv[8 * d: 8 * d + 8])
    if not row[6]:
        continue
    c = row[6]
    print("  level %d%s: chunks %8d  hit %5.1f  total %7.0f  A %6.0f B %6.0f C %6.0f D %6.0f E %6.0f F %6.0f" % (
        d, "+" if d == 7 else " ", c, row[7] / c, sum(row[:6]) / c, *[x / c for x in row[:6]]))

w = list(ws)
if w[0]:
    for name, o in (("EXTEND", 0), ("SHADOW", 4)):
        print("%s walks: inner-node loop %d wave iterations, %.1f lanes each; leaf visits %d wave iterations, %.1f lanes each"
              % (name, w[o], w[o + 1] / max(1, w[o]), w[o + 2], w[o + 3] / max(1, w[o + 2])))
