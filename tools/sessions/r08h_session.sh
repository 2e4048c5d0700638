#!/bin/bash
# Round-4: raise tests (k_hl_raise's wave-split walk), then the A/B of _variants/
# (base: a lane's walk per entry on C4; split: a wave per entry).
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_raises.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_raises.log 2>&1 && \
timeout -k 10 400 python tools/variants.py time --scene c4 --rounds 3 --reps 2 > $OUT/variants_c4.log 2>&1 && \
timeout -k 10 400 python tools/variants.py time --scene c2 --rounds 3 --reps 7 > $OUT/variants_c2.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
