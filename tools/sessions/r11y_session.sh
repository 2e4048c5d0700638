#!/bin/bash
# Round 6, session r11y: the raise buffer's resolution on C4 with the
# lane-per-walk lists (_variants: w0n40, w0n80, w0n160 = 40 / 80 / 160 raise
# cells per face side, RTX_XR_WAVE=0), C4 frames alone, interleaved rounds.
#   bash tools/sessions/r11y_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1000 python3 tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1
rc=$?
grep SUMMARY $OUT/variants_c4.log
echo "session $TAG rc=$rc"
exit $rc
