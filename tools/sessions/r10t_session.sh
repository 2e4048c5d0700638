#!/bin/bash
# Round 5, session r10t: C4's global light-buffer resolution, 96 / 128 / 160 cells per face side
# (lbuf_check: 2.0 / 1.6 / 1.4 leaves per lookup), interleaved rounds on one box.
#   bash tools/sessions/r10t_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python3 tools/variants.py time --scene c4 --rounds 3 --reps 2 > $OUT/variants_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
