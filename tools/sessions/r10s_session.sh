#!/bin/bash
# Round 5, session r10s: the light buffer for C4-sized scenes (a 96 x 96-per-face table read from global
# memory beside the 16-bit leaves; C2 keeps its LDS table).  The level / raise / parity GPU tests, then C4
# and C2 timing with and without it.
#   bash tools/sessions/r10s_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_levels.py tests/test_raises.py tests/test_gpu_parity.py tests/test_gpu_bvh.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 500 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"lbuf": 0}' > $OUT/timing_c4.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 9 '{}' '{"lbuf": 0}' '{}' '{"lbuf": 0}' > $OUT/timing_c2.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
