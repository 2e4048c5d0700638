#!/bin/bash
# Round 6, session r11j: the C2 1/8 share one frame at a time (VERDICT r5 item
# 5): its time under the part count (lv_streams 1-4), then a kernel trace of
# the default share for its timeline (tools/share_timeline.py).
#   bash tools/sessions/r11j_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 240 python3 tools/timing.py --scene c2 --share 0/8 --reps 15 '{}' '{"lv_streams": 1}' \
  '{"lv_streams": 3}' '{"lv_streams": 4}' '{}' '{"lv_streams": 1}' '{"lv_streams": 3}' '{"lv_streams": 4}' \
  > $OUT/timing_share8.log 2>&1 &&
timeout -k 10 240 python3 tools/timing.py --scene c2 --reps 9 '{}' '{"lv_streams": 1}' '{"lv_streams": 3}' \
  > $OUT/timing_full.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/share8 -o share8 -- \
  python3 tools/timing.py --scene c2 --share 0/8 --reps 9 '{}' > $OUT/share8_trace.log 2>&1
rc=$?
cat $OUT/timing_share8.log $OUT/timing_full.log | grep -v amdgpu.ids | grep -v levels:
echo "session $TAG rc=$rc"
exit $rc
