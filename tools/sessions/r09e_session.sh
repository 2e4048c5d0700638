#!/bin/bash
# Round 5, session e: World#high_lights' lit_area raise checked inline in the level kernels with the fused
# walk (RTX_HL_INLINE, no k_hl_raise), the walk's slab constants kept const (no scratch).  Every GPU test,
# then C2 / C4 on one box: this build (new), the deferred k_hl_raise build (hl0) and round 4 (r4).
#   bash tools/sessions/r09e_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 400 python3 tools/variants.py time --scene c2 --rounds 4 --reps 7 > $OUT/variants_c2.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"exact_raises": 1}' '{}' '{"exact_raises": 1}' > $OUT/timing_c2_xr.log 2>&1 && \
timeout -k 10 500 python3 tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
