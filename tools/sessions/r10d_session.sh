#!/bin/bash
# Round 5, session r10d: ray binning, keys written by the producing level, one contiguous range of chunks per
# binning workgroup (r10c: counting from the staged rays cost 0.1 ms per C2 level).
# Binning tests, C2 / C4 timing with and without it (default two parts), kernel traces of one part.
#   bash tools/sessions/r10c_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_levels.py -k binned -x -v --timeout 120 --timeout-method thread > $OUT/pytest_binned.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"lv_sort": 1}' '{}' '{"lv_sort": 1}' > $OUT/timing_c2.log 2>&1 && \
timeout -k 10 500 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"lv_sort": 1}' > $OUT/timing_c4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_sort -o kt --output-format csv -- python3 tools/timing.py --scene c2 --reps 5 '{"lv_streams": 1, "lv_sort": 1}' > $OUT/prof_sort.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4_sort -o kt --output-format csv -- python3 tools/timing.py --scene c4 --reps 1 '{"lv_streams": 1, "lv_sort": 1}' > $OUT/prof_c4_sort.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
