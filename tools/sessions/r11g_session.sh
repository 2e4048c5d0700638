#!/bin/bash
# Round 6, session r11g: the GPU test suite on the exact_raises-by-default
# build (raise buffer with 16-bit gates), then the bench line (C2, defaults).
#   bash tools/sessions/r11g_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
tail -3 $OUT/pytest_gpu.log
tail -c 600 $OUT/bench.json
echo "session $TAG rc=$rc"
exit $rc
