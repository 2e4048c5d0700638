#!/bin/bash
# Round-4 A/B of compile-time variants (tools/variants.py: every library under
# _variants/), rounds interleaved: C2 and C4 frames alone.   bash tools/sessions/r08f_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python tools/variants.py time --scene c2 --rounds 4 --reps 7 > $OUT/variants_c2.log 2>&1 && \
timeout -k 10 400 python tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
