#!/bin/bash
# Round 6, session r11ag: the C2 1/8 share's chunk schedule (verdict r5 item 5):
# static vs claimed chunks (lv_static), grid size (lv_grid_div), one frame at
# a time, two interleaved rounds; then the full frame with the best candidates.
#   bash tools/sessions/r11ag_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 9 --share 0/8 '{}' '{"lv_static": 0}' '{"lv_static": 50}' \
  '{"lv_static": 75}' '{}' '{"lv_static": 0}' '{"lv_static": 50}' '{"lv_static": 75}' > $OUT/timing_share8.log 2>&1 &&
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 9 '{}' '{"lv_static": 0}' '{"lv_static": 50}' \
  '{}' '{"lv_static": 0}' '{"lv_static": 50}' > $OUT/timing_c2.log 2>&1
rc=$?
cat $OUT/timing_share8.log $OUT/timing_c2.log | grep -v amdgpu.ids | grep -v levels:
echo "session $TAG rc=$rc"
exit $rc
