#!/bin/bash
# Round 5, session r10s2: C4 runtime-option sweep on the final build (no rebuild): ray-bin grid,
# static chunk share, streams, batch, light-buffer on/off.
#   bash tools/sessions/r10s2_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u tools/timing.py --scene c4 --reps 4 '{}' '{"lv_sort_bits": 3}' '{"lv_static": 100}' \
    '{"lv_static": 0}' '{"lv_streams": 1}' '{"lv_streams": 4}' '{"lv_batch": 8388608}' '{"lv_sort_from": 2}' '{}' \
    > $OUT/timing_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
