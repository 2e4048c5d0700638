#!/bin/bash
# Round 5, session r10n: the final bench line (frame latency now as one frame renders by default),
# C4's PMC passes, bench line and single-frame kernel trace for this build.
#   bash tools/sessions/r10n_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
bash tools/gpu_session.sh $TAG bench && WL=c4 bash tools/gpu_session.sh $TAG pmcbench
rc=$?
echo "session $TAG rc=$rc"
exit $rc
