#!/bin/bash
# Round 5, session c: the fused raise check as a compile-time kernel variant (k_level_c<..., XR>), band
# half-width 32 float32 ulps, per-nappe cone bounds.  Raise tests, every GPU test, then C2 / C4 timing
# with exact_raises on (default) and off in one process, and the round-4 library beside this one.
#   bash tools/sessions/r09c_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_raises.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_raises.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"exact_raises": 0}' '{}' '{"exact_raises": 0}' > $OUT/timing_c2_xr.log 2>&1 && \
timeout -k 10 300 python3 tools/variants.py time --scene c2 --rounds 3 --reps 7 > $OUT/variants_c2.log 2>&1 && \
timeout -k 10 400 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"exact_raises": 0}' '{}' '{"exact_raises": 0}' > $OUT/timing_c4_xr.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
