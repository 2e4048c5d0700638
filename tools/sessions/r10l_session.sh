#!/bin/bash
# Round 5, session r10l: binning by default everywhere (auto: C4-sized scenes every level >= 1 with 16^3
# origin cells, small scenes the last level only with 8^3; r10k: C2 4.60 -> 4.57 ms).  Every GPU test,
# then C2 / C4 timing of the auto policy against binning off and against the other resolution.
#   bash tools/sessions/r10l_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"lv_sort": 0}' '{"lv_sort_bits": 4}' '{}' '{"lv_sort": 0}' '{"lv_sort_bits": 4}' > $OUT/timing_c2.log 2>&1 && \
timeout -k 10 500 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"lv_sort_bits": 3}' > $OUT/timing_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
