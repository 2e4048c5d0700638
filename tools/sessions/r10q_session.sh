#!/bin/bash
# Round 5, session r10q: small scenes bin their last level only in batches of >= 2^22 samples (r10p).
# Every GPU test, smoke, C2 PMC passes + bench + traces, C4 bench, then BASELINE.md's table.
#   bash tools/sessions/r10q_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
bash tools/gpu_session.sh $TAG full && bash tools/gpu_session.sh $TAG baseline
rc=$?
echo "session $TAG rc=$rc"
exit $rc
