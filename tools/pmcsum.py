#!/usr/bin/env python3
"""Summarize tools/pmc.sh output per kernel (summed over its dispatches, divided by --frames).

    python tools/pmcsum.py gpurun_out/TAG [--frames N] [--match k_lv]

Derived per kernel: active lanes per VALU instruction (SQ_THREAD_CYCLES_VALU /
SQ_ACTIVE_INST_VALU), the share of wave time waiting (SQ_WAIT_ANY /
SQ_WAVE_CYCLES) and issuing VALU, and HBM bytes (2 x FETCH_SIZE + WRITE_SIZE,
KB units, the gfx950 corrections of MI355X_MICROARCH.md)."""
import argparse, collections, csv, glob, re

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--frames", type=float, default=2.0)
ap.add_argument("--match", default="k_")
a = ap.parse_args()

tot = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(dict)
for f in sorted(glob.glob(a.dir + "/pmc_*/*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if a.match not in name:
            continue
        k = re.sub(r"\(.*", "", name).replace("void ", "").replace("rtx::", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[k][(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, c in sorted(tot.items()):
    n = a.frames
    ms = sum(dur[k].values()) / len(set(x for x in dur[k])) * (len(dur[k]) / max(1, len(set(f for f, _ in dur[k]))) / n) \
        if dur[k] else 0
    print("== %s   (%.3f ms per frame)" % (k, ms))
    for name, v in sorted(c.items()):
        print("   %-28s %.4g" % (name, v / n))
    wc = c.get("SQ_WAVE_CYCLES", 0)
    if c.get("SQ_ACTIVE_INST_VALU"):
        print("   active lanes / VALU instr  %.1f" % (c["SQ_THREAD_CYCLES_VALU"] / c["SQ_ACTIVE_INST_VALU"]))
    if wc:
        print("   wait / wave time           %.2f   VALU issue / wave time %.2f" % (
            c.get("SQ_WAIT_ANY", 0) / wc, c.get("SQ_ACTIVE_INST_VALU", 0) / wc))
    if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
        print("   HBM bytes per frame        %.3g" % ((2 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024 / n))
