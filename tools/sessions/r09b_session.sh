#!/bin/bash
# Round 5, session b: exact_raises on by default, fused into the shadow walk: every GPU
# test (the raise tests first), smoke, the bench line, then on one box: the round-4 library, the pruned
# build without the fused check (cur) and this one (xr) on C2 and C4 (tools/variants.py), and this build
# with exact_raises 0 / 1 (tools/timing.py, same process).
#   bash tools/sessions/r09b_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_raises.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_raises.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 python3 tools/variants.py time --scene c2 --rounds 3 --reps 7 > $OUT/variants_c2.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"exact_raises": 0}' '{}' '{"exact_raises": 0}' > $OUT/timing_c2_xr.log 2>&1 && \
timeout -k 10 500 python3 tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
