#!/bin/bash
# Round 6, session r11x: per-sphere raise lists spread over the wave
# (raise_lists_wave, RTX_XR_WAVE): the raise, light-buffer and hierarchy GPU
# tests on the default build, C4 frames alone with exact_raises 0 and 1, then
# the variants (_variants: w0 = the lane-per-walk lists, w1 = the wave's queue,
# w1n80 = the queue with 80 raise cells per face side) on C4.
#   bash tools/sessions/r11x_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_raises.py \
  tests/test_lbuf.py tests/test_gpu_bvh.py > $OUT/pytest.log 2>&1 &&
timeout -k 10 300 python3 tools/timing.py --scene c4 --reps 3 '{"exact_raises": 0}' '{"exact_raises": 1}' \
  '{"exact_raises": 0}' '{"exact_raises": 1}' > $OUT/timing_c4.log 2>&1 &&
timeout -k 10 900 python3 tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
cat $OUT/timing_c4.log | grep -v amdgpu.ids | grep -v levels:
grep SUMMARY $OUT/variants_c4.log
echo "session $TAG rc=$rc"
exit $rc
