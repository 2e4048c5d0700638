#!/bin/bash
# Round-4: C4 schedule options on the final build (parts on streams, static share of chunks).
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"lv_streams": 1}' '{"lv_streams": 3}' '{"lv_static": 100}' '{"lv_static": 50}' '{"lv_batch": 33554432, "lv_streams": 1}' '{}' > $OUT/timing_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
