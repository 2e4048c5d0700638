#!/bin/bash
# Round 5, session r10b: where ray binning's time goes (r10a: C2 4.62 -> 7.72 ms although the walks'
# wave iterations fell 18-21 %).  One part per frame (no second stream to overlap or to block the
# binning kernels), kernel traces with and without binning, C2 and C4.
#   bash tools/sessions/r10b_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{"lv_streams": 1}' '{"lv_streams": 1, "lv_sort": 1}' '{"lv_streams": 1}' '{"lv_streams": 1, "lv_sort": 1}' > $OUT/timing_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_plain -o kt --output-format csv -- python3 tools/timing.py --scene c2 --reps 5 '{"lv_streams": 1}' > $OUT/prof_plain.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_sort -o kt --output-format csv -- python3 tools/timing.py --scene c2 --reps 5 '{"lv_streams": 1, "lv_sort": 1}' > $OUT/prof_sort.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4_plain -o kt --output-format csv -- python3 tools/timing.py --scene c4 --reps 1 '{"lv_streams": 1}' > $OUT/prof_c4_plain.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4_sort -o kt --output-format csv -- python3 tools/timing.py --scene c4 --reps 1 '{"lv_streams": 1, "lv_sort": 1}' > $OUT/prof_c4_sort.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
