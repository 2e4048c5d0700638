#!/bin/bash
# Round-4: in-place raise check on LDSX scenes (_variants/librtx_inl.so): its raise / level tests,
# then the A/B against the in-tree build (_variants/librtx_base.so).
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
RTX_LIB=$PWD/_variants/librtx_inl.so timeout -k 10 500 python -u -m pytest tests/test_raises.py tests/test_gpu_levels.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_inl.log 2>&1 && \
timeout -k 10 400 python tools/variants.py time --scene c2 --rounds 4 --reps 7 > $OUT/variants_c2.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
