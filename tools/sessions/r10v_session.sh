#!/bin/bash
# Round 5, session r10v: C4's PMC passes, bench line and single-frame trace for the final build, then
# BASELINE.md's table.
#   bash tools/sessions/r10v_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
WL=c4 bash tools/gpu_session.sh $TAG pmcbench && bash tools/gpu_session.sh $TAG baseline
rc=$?
echo "session $TAG rc=$rc"
exit $rc
