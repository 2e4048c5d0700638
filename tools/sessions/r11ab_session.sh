#!/bin/bash
# Round 6, session r11ab: the raise buffer at 80 and 160 cells per face side on
# C4 (_variants n80, n160; both with the one-round-trip bin scan and the
# threaded raise-buffer builder), C4 frames alone, interleaved rounds.
#   bash tools/sessions/r11ab_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python3 tools/variants.py time --scene c4 --rounds 3 --reps 2 > $OUT/variants_c4.log 2>&1
rc=$?
grep SUMMARY $OUT/variants_c4.log
echo "session $TAG rc=$rc"
exit $rc
