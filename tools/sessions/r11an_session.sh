#!/bin/bash
# Round 6, session r11an: the overflow re-walk of query_lbuf without the raise
# band test (RTX_OVF_XR=0: the light buffer's band tests and the raise lists
# have checked every factor-0 raise already) against with it (=1): C4 and C2
# frames alone for _variants ovf0 / ovf1, interleaved rounds.
#   bash tools/sessions/r11an_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python3 tools/variants.py time --scene c4 --rounds 3 --reps 2 > $OUT/variants_c4.log 2>&1 &&
timeout -k 10 600 python3 tools/variants.py time --scene c2 --rounds 3 --reps 9 > $OUT/variants_c2.log 2>&1
rc=$?
grep SUMMARY $OUT/variants_c4.log $OUT/variants_c2.log
echo "session $TAG rc=$rc"
exit $rc
