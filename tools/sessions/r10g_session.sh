#!/bin/bash
# Round 5, session r10g: ray-bin resolution, 8^3 (cb3: 4,096 bins) against 16^3 origin cells (cb4: 32,768
# bins, the new default; the emulator: C4 walk time 0.822 -> 0.788 of the unbinned order), same box,
# interleaved rounds; then the binning tests on the in-tree (cb4) build.
#   bash tools/sessions/r10g_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 500 python3 tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1 && \
timeout -k 10 300 python3 tools/variants.py time --scene c2 --rounds 2 --reps 5 --opts '{"lv_sort": 1}' > $OUT/variants_c2_sort.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_levels.py -k binned -x -v --timeout 120 --timeout-method thread > $OUT/pytest_binned.log 2>&1
rc=$?
echo "session $TAG rc=$rc"
exit $rc
