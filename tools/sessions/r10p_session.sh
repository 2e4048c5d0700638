#!/bin/bash
# Round 5, session r10p: last-level binning on small shares (C2 1/8, 1/4, 1/2 of the frame, one part each as
# the in-flight bench renders them): default (binned) against lv_sort 0, two interleaved pairs.
#   bash tools/sessions/r10p_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for sh in 0/8 0/4 0/2; do
  timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 9 --share $sh --tile-rows 8 \
    '{"lv_streams": 1}' '{"lv_streams": 1, "lv_sort": 0}' '{"lv_streams": 1}' '{"lv_streams": 1, "lv_sort": 0}' \
    >> $OUT/timing_c2_shares.log 2>&1 || exit 1
done
echo "session $TAG rc=0"
