#!/bin/bash
# Round 6, session r11t: the final build (entries keep their l-interval, the device tests the sort key only;
# tangency bounds from the builder): C4 and C2 frames alone with
# exact_raises 0 and 1.
#   bash tools/sessions/r11t_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 tools/timing.py --scene c4 --reps 3 '{"exact_raises": 0}' '{"exact_raises": 1}' \
  '{"exact_raises": 0}' '{"exact_raises": 1}' > $OUT/timing_c4.log 2>&1 &&
timeout -k 10 240 python3 tools/timing.py --scene c2 --reps 9 '{"exact_raises": 0}' '{"exact_raises": 1}' \
  '{"exact_raises": 0}' '{"exact_raises": 1}' > $OUT/timing_c2.log 2>&1
rc=$?
cat $OUT/timing_c4.log $OUT/timing_c2.log | grep -v amdgpu.ids | grep -v levels:
echo "session $TAG rc=$rc"
exit $rc
