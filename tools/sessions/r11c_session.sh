#!/bin/bash
# Round 6, session r11c: C4 and C2 frames alone with exact_raises 0 and 1 in
# alternation, raise-buffer entries read four at a time (tools/timing.py
# checks both options render the same bits); then diagnostic builds of
# the C2 exact_raises kernel without its band test / raise lists (_variants).
#   bash tools/sessions/r11c_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 tools/timing.py --scene c4 --reps 3 '{"exact_raises": 0}' '{"exact_raises": 1}' \
  '{"exact_raises": 0}' '{"exact_raises": 1}' > $OUT/timing_c4.log 2>&1 &&
timeout -k 10 240 python3 tools/timing.py --scene c2 --reps 9 '{"exact_raises": 0}' '{"exact_raises": 1}' \
  '{"exact_raises": 0}' '{"exact_raises": 1}' > $OUT/timing_c2.log 2>&1 &&
timeout -k 10 400 python3 tools/variants.py time --scene c2 --rounds 3 --reps 7 > $OUT/variants_c2.log 2>&1
rc=$?
grep SUMMARY $OUT/variants_c2.log
cat $OUT/timing_c4.log $OUT/timing_c2.log 2>/dev/null | grep -v amdgpu.ids | tail -20
echo "session $TAG rc=$rc"
exit $rc
