#!/usr/bin/env python3
"""FETCH_SIZE per access pattern from a tools/fetch_probe.hip run.

    python tools/fetch_probe_json.py OUT_DIR/fetch_probe OUT_DIR/fetch_probe.log profiles/fetch_probe.json

For each probe kernel: the algorithmic bytes it read (printed by the probe),
FETCH_SIZE (KiB, summed over the XCDs by rocprofv3) and their ratio
counted / true.  MI355X_MICROARCH.md's read correction (bytes = 2 x
FETCH_SIZE) holds where the ratio is 0.5.
"""
import csv
import glob
import json
import os
import sys


def main(d, log, out):
    true = {}
    order = []
    for line in open(log):
        if " bytes " in line and line.split()[0].startswith("k_"):
            name, _, b = line.split()
            order.append(name)
            true.setdefault(name, []).append(int(b))
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "FETCH_SIZE" and r["Kernel_Name"].lstrip("void ").startswith("k_"):
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    res = {}
    for (_, kname, kib), name in zip(rows, order):
        short = kname.replace("void ", "").split("(")[0].replace("char const*", "").strip()
        assert short.split("<")[0] == name.split("<")[0], (short, name)
        b = true[name][0]
        res.setdefault(name, []).append({"true_bytes": b, "fetch_size_bytes": kib * 1024.0,
                                         "counted_over_true": kib * 1024.0 / b})
    summary = {k: round(sum(x["counted_over_true"] for x in v) / len(v), 4) for k, v in res.items()}
    doc = {"what": "FETCH_SIZE (rocprofv3, KiB x 1024) over the bytes each probe kernel reads exactly once from a "
                   "2 GiB arena (tools/fetch_probe.hip); two repetitions each",
           "patterns": {"k_stream": "16-B vector loads, consecutive lanes consecutive",
                        "k_scatter<32>": "one 32-B record per lane at a permuted slot (k_tree_finalize's tree records)",
                        "k_runs<32>": "32-B records in runs of 64 per wave, runs permuted",
                        "k_scatter<80>": "one 80-B record per lane at a permuted slot",
                        "k_runs<80>": "80-B records in runs of 64 per wave (k_level_c's staged rays)"},
           "counted_over_true": summary, "runs": res}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(summary))


if __name__ == "__main__":
    main(*sys.argv[1:4])
