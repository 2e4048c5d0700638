#!/bin/bash
# Round 5, session r10a: ray binning (option lv_sort: levels >= 1 visited bin by bin, one counting-sort
# pass per level; the wave emulator tools/wave_sim.cpp ranked it first).  The binning tests, C2 / C4
# timing with and without it on one box, the walks' lane counters (RTX_WALKSTATS build) with and
# without it, and a kernel trace of the binned C2 frame.
#   bash tools/sessions/r10a_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_levels.py -k binned -x -v --timeout 120 --timeout-method thread > $OUT/pytest_binned.log 2>&1 && \
RTX_LIB=_variants/librtx_walkstats.so timeout -k 10 200 python3 tools/stamps_levels.py c2 > $OUT/walk_c2.log 2>&1 && \
RTX_LIB=_variants/librtx_walkstats.so timeout -k 10 200 python3 tools/stamps_levels.py c2 lv_sort=1 > $OUT/walk_c2_sort.log 2>&1 && \
RTX_LIB=_variants/librtx_walkstats.so timeout -k 10 300 python3 tools/stamps_levels.py c4 > $OUT/walk_c4.log 2>&1 && \
RTX_LIB=_variants/librtx_walkstats.so timeout -k 10 300 python3 tools/stamps_levels.py c4 lv_sort=1 > $OUT/walk_c4_sort.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"lv_sort": 1}' '{}' '{"lv_sort": 1}' > $OUT/timing_c2.log 2>&1 && \
timeout -k 10 500 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"lv_sort": 1}' > $OUT/timing_c4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_sort -o run -- python3 tools/timing.py --scene c2 --reps 5 '{"lv_sort": 1}' > $OUT/prof_sort.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
