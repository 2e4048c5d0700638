#!/bin/bash
# Round-4 evidence session (one build, one sha):
#   bash tools/sessions/r08_final.sh TAG a   tests, smoke, option A/B (refill), C2 PMC passes + bench + kernel traces
#   bash tools/sessions/r08_final.sh TAG b   C4 PMC passes + bench line + single-frame kernel trace
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$2" = a ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
  timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"lv_refill": 16}' '{}' > $OUT/timing_c2.log 2>&1 && \
  timeout -k 10 400 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"lv_batch": 8388608}' '{}' > $OUT/timing_c4.log 2>&1 && \
  WL=c2 bash tools/gpu_session.sh $TAG pmcbench
else
  WL=c4 bash tools/gpu_session.sh ${TAG}4 pmcbench
fi
rc=$?
echo "session $TAG $2 rc=$rc"
exit $rc
