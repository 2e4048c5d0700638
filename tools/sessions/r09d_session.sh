#!/bin/bash
# Round 5, session d: exact_raises off by default (its fused check a kernel variant), rtx_render_multi_plan /
# rtx_tile_probe / rtx_lpt_plan, the CLI's LPT split.  Every GPU test, smoke, the bench line, then C2 / C4
# with exact_raises 0 (default) / 1 in one process, and the round-4 library beside this one on C2.
#   bash tools/sessions/r09d_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"exact_raises": 1}' '{}' '{"exact_raises": 1}' > $OUT/timing_c2_xr.log 2>&1 && \
timeout -k 10 300 python3 tools/variants.py time --scene c2 --rounds 3 --reps 7 > $OUT/variants_c2.log 2>&1 && \
timeout -k 10 400 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"exact_raises": 1}' '{}' '{"exact_raises": 1}' > $OUT/timing_c4_xr.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
