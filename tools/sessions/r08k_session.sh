#!/bin/bash
# Round-4: C4 batch size sweep (option lv_batch: camera samples per bounce-level batch).
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 500 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"lv_batch": 16777216}' '{"lv_batch": 33554432}' '{"lv_batch": 67108864}' '{}' > $OUT/timing_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
