#!/usr/bin/env python3
"""Per-launch HBM traffic of k_render from two rocprofv3 PMC passes.

    python tools/pmc_json.py FETCH_DIR WRITE_DIR OUT.json --workload c2

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch
(memory-side L2 requests).  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports
half the bytes of wide (16 B/lane) coalesced reads, so the corrected read bytes
are 2 x FETCH_SIZE; WRITE_SIZE reads 16 B/lane stores exactly.  Other access
widths are uncalibrated there, so both the raw and the corrected values are
kept.  Counting launches (k_render<true,...>) are excluded.
"""
import argparse
import csv
import glob
import json
import os


def per_launch(d, counter):
    vals = {}
    for f in glob.glob(os.path.join(d, "*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if r["Counter_Name"] != counter or "k_render" not in name or "k_renderILb1E" in name:
                continue
            key = (f, r["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    v = sorted(vals.values())
    if not v:
        return None, 0
    v = v[1:] if len(v) > 2 else v          # drop the first (cold) launch
    return sum(v) / len(v), len(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("out")
    ap.add_argument("--workload", default="c2")
    a = ap.parse_args()
    fk, nf = per_launch(a.fetch_dir, "FETCH_SIZE")
    wk, nw = per_launch(a.write_dir, "WRITE_SIZE")
    out = {
        "workload": a.workload,
        "kernel": "k_render",
        "fetch_size_kib": fk, "write_size_kib": wk, "launches": [nf, nw],
        "read_bytes": None if fk is None else 2.0 * fk * 1024,
        "write_bytes": None if wk is None else wk * 1024,
        "correction": "read = 2 x FETCH_SIZE (gfx950, MI355X_MICROARCH.md HBM section); write = WRITE_SIZE",
        "source": [os.path.relpath(a.fetch_dir), os.path.relpath(a.write_dir)],
    }
    out["traffic_bytes"] = None if fk is None or wk is None else out["read_bytes"] + out["write_bytes"]
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
