#!/bin/bash
# Round 5, session r10y: the LDS prefetch of queue-order chunks (option lv_prefetch): its parity
# tests, then C2 whole-frame and 1/8-share timings with it off and on (interleaved).
# (The option existed only in the build this session measured; it was reverted)
#   bash tools/sessions/r10y_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_levels.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "prefetch or light_buffer or binn or c2_full" > $OUT/pytest_pf.log 2>&1 && \
timeout -k 10 300 python -u tools/timing.py --scene c2 --reps 9 --inflight 2 '{"lv_prefetch": 0}' '{"lv_prefetch": 1}' \
    '{"lv_prefetch": 0}' '{"lv_prefetch": 1}' > $OUT/timing_c2.log 2>&1 && \
timeout -k 10 300 python -u tools/timing.py --scene c2 --reps 9 '{"lv_prefetch": 0}' '{"lv_prefetch": 1}' \
    '{"lv_prefetch": 0}' '{"lv_prefetch": 1}' > $OUT/timing_c2_single.log 2>&1 && \
timeout -k 10 300 python -u tools/timing.py --scene c2 --reps 9 --share 0/8 --inflight 2 '{"lv_prefetch": 0}' \
    '{"lv_prefetch": 1}' '{"lv_prefetch": 0}' '{"lv_prefetch": 1}' > $OUT/timing_c2_share.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
