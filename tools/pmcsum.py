#!/usr/bin/env python3
"""Summarize tools/pmc.sh output: per-counter value of the last k_render dispatch."""
import collections, csv, glob, sys
d = sys.argv[1]
tot = {}
for f in sorted(glob.glob(d + '/pmc_*/*_counter_collection.csv')):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if 'k_render' in r['Kernel_Name']:
            agg[int(r['Dispatch_Id'])][r['Counter_Name']] += float(r['Counter_Value'])
    if agg:
        tot.update(agg[max(agg)])
for k, v in sorted(tot.items()):
    print('%-26s %.4g' % (k, v))
if 'SQ_WAVE_CYCLES' in tot and 'GRBM_GUI_ACTIVE' in tot:
    per_xcd = tot['GRBM_GUI_ACTIVE'] / 8
    print('occupancy (waves per SIMD, of 2): %.2f' % (tot['SQ_WAVE_CYCLES'] * 4 / (per_xcd * 1024)))
    print('wait_any %.2f wait_inst %.2f active_any %.2f active_valu %.2f' % tuple(
        tot.get(k, 0) / tot['SQ_WAVE_CYCLES'] for k in ('SQ_WAIT_ANY', 'SQ_WAIT_INST_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_ACTIVE_INST_VALU')))
