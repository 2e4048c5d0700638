#!/bin/bash
# Round-4: refill with a whole-wave pre-pass and an LDS list (library _variants/librtx_rq.so):
# its refill tests, then C4 / C2 timings with and without lv_refill.
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
export RTX_LIB=$PWD/_variants/librtx_rq.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_levels.py -k "refill" -x -v --timeout 120 --timeout-method thread > $OUT/pytest_refill.log 2>&1 && \
timeout -k 10 400 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"lv_refill": 8}' '{"lv_refill": 16}' '{"lv_refill": 32}' '{}' > $OUT/timing_c4.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"lv_refill": 8}' '{"lv_refill": 16}' '{}' > $OUT/timing_c2.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
