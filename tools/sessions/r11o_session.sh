#!/bin/bash
# Round 6, session r11o: where C4's exact_raises time goes: the diagnostic
# builds of r11c (_variants: base, without the band test, without the raise
# lists, without both; wrong results on raise inputs only) on C4.
#   bash tools/sessions/r11o_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python3 tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1
rc=$?
grep SUMMARY $OUT/variants_c4.log
echo "session $TAG rc=$rc"
exit $rc
