#!/bin/bash
# Round 6, session r11f: C4 and C2 frames alone with exact_raises 0 and 1 in
# alternation, ql from the bits of |d|^2, exact log2 only past a gate (tools/timing.py checks
# both options render the same bits).
#   bash tools/sessions/r11f_session.sh TAG
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
cat $OUT/timing_c4.log $OUT/timing_c2.log 2>/dev/null | grep -v amdgpu.ids | tail -20
echo "session $TAG rc=$rc"
exit $rc
