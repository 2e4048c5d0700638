#!/usr/bin/env python3
"""Per-kernel totals of a rocprofv3 kernel trace: python tools/ktsum.py DIR [--frames N]"""
import collections, csv, glob, re, sys
d = sys.argv[1]
frames = float(sys.argv[sys.argv.index("--frames") + 1]) if "--frames" in sys.argv else 1.0
f = glob.glob(d + "/*kernel_trace.csv")[0]
tot = collections.OrderedDict()
for r in csv.DictReader(open(f)):
    k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("rtx::", "")
    t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    n, s = tot.get(k, (0, 0.0))
    tot[k] = (n + 1, s + t)
for k, (n, s) in tot.items():
    print("%-44s launches %5.0f  total %9.3f ms  avg %8.4f ms" % (k, n / frames, s / frames, s / n))
