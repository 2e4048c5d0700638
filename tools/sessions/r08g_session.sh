#!/bin/bash
# Round-4: the raise tests on the new k_hl_raise, then the A/B of _variants/
# (base: the walk per entry; flat: a wave per entry; nohlr: no highlight raise check).
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_raises.py tests/test_gpu_bvh.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_raises.log 2>&1 && \
timeout -k 10 400 python tools/variants.py time --scene c2 --rounds 4 --reps 7 > $OUT/variants_c2.log 2>&1 && \
timeout -k 10 400 python tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
