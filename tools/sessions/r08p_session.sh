#!/bin/bash
# Round-4: the hierarchy tests (incl. the refused-quantization fallback) on the final build.
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bvh.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_bvh.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
