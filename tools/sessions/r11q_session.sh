#!/bin/bash
# Round 6, session r11q: the floor terms read with the light data (one round trip less)
# (C4: 40 cells per face side): the raise GPU tests (600 filler spheres run
# them), then C4 frames alone with exact_raises 0 and 1.
#   bash tools/sessions/r11q_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_raises.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_raises.log 2>&1 &&
timeout -k 10 300 python3 tools/timing.py --scene c4 --reps 3 '{"exact_raises": 0}' '{"exact_raises": 1}' \
  '{"exact_raises": 0}' '{"exact_raises": 1}' > $OUT/timing_c4.log 2>&1 &&
timeout -k 10 240 python3 tools/timing.py --scene c2 --reps 9 '{"exact_raises": 0}' '{"exact_raises": 1}' \
  '{"exact_raises": 0}' '{"exact_raises": 1}' > $OUT/timing_c2.log 2>&1
rc=$?
tail -2 $OUT/pytest_raises.log
cat $OUT/timing_c4.log $OUT/timing_c2.log | grep -v amdgpu.ids | grep -v levels:
echo "session $TAG rc=$rc"
exit $rc
