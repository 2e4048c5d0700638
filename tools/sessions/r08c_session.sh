#!/bin/bash
# Round-4 GPU session (refill): the refill tests first, then every GPU test,
# then the C2 / C4 A/B of option lv_refill (drain / save).   bash tools/sessions/r08c_session.sh TAG [notests]
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_levels.py -k "refill" -x -v --timeout 120 --timeout-method thread > $OUT/pytest_refill.log 2>&1 && \
{ if [ "$2" = notests ]; then true; else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; fi; } && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"lv_refill": 8}' '{"lv_refill": 16}' '{"lv_refill": 32}' '{"lv_refill": 16, "lv_refill_save": 1}' '{}' > $OUT/timing_c2.log 2>&1 && \
timeout -k 10 400 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"lv_refill": 8}' '{"lv_refill": 16}' '{"lv_refill": 32}' '{}' > $OUT/timing_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
