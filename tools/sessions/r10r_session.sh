#!/bin/bash
# Round 5, session r10r: the light buffer (option lbuf, DESIGN.md §3.18: C2's shadow walks visit only the
# leaves listed in their cube-map cell as seen from the light).  The level / raise / parity GPU tests,
# then C2 timing with and without it (two interleaved pairs) and a single-frame kernel trace.
#   bash tools/sessions/r10r_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_levels.py tests/test_raises.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 9 '{}' '{"lbuf": 0}' '{}' '{"lbuf": 0}' > $OUT/timing_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_single -o kt --output-format csv -- python3 tools/timing.py --scene c2 --reps 5 '{"lv_streams": 1}' > $OUT/prof_single.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
