#!/bin/bash
# Round 5, session r10k: C2 with binning of the deep levels only (option lv_sort_from: r10b showed the
# binned level kernels gain most on the last level, -10 %, and nothing on level 1), 32,768 bins (in-tree)
# and 4,096 bins (_variants/librtx_cb3.so), then the binning tests.
#   bash tools/sessions/r10k_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
OPTS=('{}' '{"lv_sort": 1}' '{"lv_sort": 1, "lv_sort_from": 3}' '{"lv_sort": 1, "lv_sort_from": 4}')
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 "${OPTS[@]}" "${OPTS[@]}" > $OUT/timing_c2_cb4.log 2>&1 && \
RTX_LIB=_variants/librtx_cb3.so timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 "${OPTS[@]}" "${OPTS[@]}" > $OUT/timing_c2_cb3.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_levels.py -k binned -x -v --timeout 120 --timeout-method thread > $OUT/pytest_binned.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
