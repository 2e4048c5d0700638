#!/bin/bash
# Round 5, session a: the pruned build (no refill / LDS-gathered reduction, lanes-engine stack depth as a
# launch parameter): every GPU test, smoke, the bench line (fixture parity fields), then C2 / C4 timing of
# the round-4 library against this one on one box (tools/variants.py: interleaved rounds, one process each).
#   bash tools/sessions/r09a_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 python3 tools/variants.py time --scene c2 --rounds 3 --reps 7 > $OUT/variants_c2.log 2>&1 && \
timeout -k 10 400 python3 tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
