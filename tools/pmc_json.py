#!/usr/bin/env python3
"""Per-frame PMC counters of the ray-tree kernel from rocprofv3 passes.

    python tools/pmc_json.py OUT.json --workload c2 --engine lanes --frames 4 --skip 1 \
        --session r02a PASS_DIR [PASS_DIR ...]

Each PASS_DIR is one `rocprofv3 --pmc ... -d PASS_DIR` run of
`tools/timing.py --reps F-1` (F frames: one warm-up + F-1 timed).  Counter
values of every dispatch of the engine's ray-tree kernel are summed; the first
`--skip` frames' dispatches are dropped (launches per frame = dispatches /
frames) and the rest averaged per frame.

HBM traffic: FETCH_SIZE / WRITE_SIZE are KiB per dispatch (memory-side L2
requests).  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half the bytes of
wide (16 B/lane) coalesced reads, so read bytes = 2 x FETCH_SIZE; WRITE_SIZE
reads 16 B/lane stores exactly.  Raw values are kept beside the corrected ones.
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dispatch_values(d, kernel, seen=None):
    """{counter: [value per dispatch in dispatch order]} for kernels whose short name is `kernel`
    (a name or a tuple of names; counting launches, k_render<true,...>, excluded).  The short
    names that matched are added to `seen`."""
    names = (kernel,) if isinstance(kernel, str) else tuple(kernel)
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            short = name.split("(")[0].split("<")[0].strip()
            if short.split("::")[-1] not in names or "k_renderILb1E" in name or "<true" in name:
                continue
            if seen is not None:
                seen.add(short.split("::")[-1])
            key = int(r["Dispatch_Id"])
            per.setdefault(r["Counter_Name"], {}).setdefault(key, 0.0)
            if r["Counter_Name"].startswith("GRBM_"):   # one row per dispatch, already summed over the 8 XCDs by rocprofv3 (roofline.valu_busy)
                per[r["Counter_Name"]][key] = max(per[r["Counter_Name"]][key], float(r["Counter_Value"]))
            else:
                per[r["Counter_Name"]][key] += float(r["Counter_Value"])
    return {c: [v[k] for k in sorted(v)] for c, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--engine", default="lanes")
    ap.add_argument("--frames", type=int, required=True)
    ap.add_argument("--skip", type=int, default=1)
    ap.add_argument("--session", default="")
    a = ap.parse_args()
    from raytracing_rb_amd import roofline
    kernel = roofline.DOMINANT_KERNEL[a.engine]
    per_frame, launches, seen = {}, None, set()
    for d in a.dirs:
        for c, vals in dispatch_values(d, kernel, seen).items():
            if len(vals) % a.frames:
                raise SystemExit("%s: %d dispatches of %s is not a multiple of %d frames" % (d, len(vals), c, a.frames))
            lpf = len(vals) // a.frames
            launches = lpf
            kept = vals[a.skip * lpf:]
            per_frame[c] = sum(kept) / (a.frames - a.skip)
    if not seen:
        raise SystemExit("no dispatch of %s in %s" % (kernel, a.dirs))
    out = {"workload": a.workload, "engine": a.engine, "kernel": "/".join(sorted(seen)), "session": a.session,
           "source_sha": roofline.kernel_source_sha(), "launches_per_frame": launches,
           "frames": a.frames - a.skip, "per_frame": per_frame,
           "source": [os.path.relpath(d, ROOT) for d in a.dirs]}
    if "FETCH_SIZE" in per_frame and "WRITE_SIZE" in per_frame:
        # The x2 read correction (MI355X_MICROARCH.md) holds for 128-B requests:
        # streaming loads and records read in runs (profiles/fetch_probe_r07a.json:
        # FETCH_SIZE = 0.50 x the bytes of k_stream, k_runs<32>, k_runs<80>).  A
        # scattered 32-B record is a 64-B request, counted at its full 64 B (2.0 x
        # the record): there FETCH_SIZE itself is the HBM read traffic.  The level
        # kernels read their staged rays in runs of 64 (chunks): x2.
        fs = per_frame["FETCH_SIZE"] * 1024
        rd, wr = 2.0 * fs, per_frame["WRITE_SIZE"] * 1024
        out.update(read_bytes_per_frame=rd, write_bytes_per_frame=wr, traffic_bytes_per_frame=rd + wr,
                   read_bytes_if_all_64B_requests=fs,
                   correction="read = 2 x FETCH_SIZE (gfx950: 128-B requests counted at half, MI355X_MICROARCH.md "
                              "HBM section; checked for runs of records by tools/fetch_probe.hip, "
                              "profiles/fetch_probe_r07a.json); scattered 32-B records (64-B requests) are "
                              "counted in full: read_bytes_if_all_64B_requests is the lower bound; write = WRITE_SIZE")
    lanes, how = roofline.active_lanes(per_frame)
    if lanes:
        out.update(active_lanes=lanes, active_lanes_from=how)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
