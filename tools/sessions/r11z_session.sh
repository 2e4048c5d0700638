#!/bin/bash
# Round 6, session r11z: k_hl_raise through the light and raise buffers on
# small scenes too (RTX_HL_BUF_SMALL; C2 checked a listed ray with a wave over
# its 64 spheres before): the raise and level GPU tests on the default build,
# C2 frames alone for the variants (_variants: hl0 = the wave per entry, hl1 =
# the buffers), then C2 with exact_raises 0 and 1.
#   bash tools/sessions/r11z_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_raises.py \
  tests/test_gpu_levels.py > $OUT/pytest.log 2>&1 &&
timeout -k 10 600 python3 tools/variants.py time --scene c2 --rounds 3 --reps 9 > $OUT/variants_c2.log 2>&1 &&
timeout -k 10 240 python3 tools/timing.py --scene c2 --reps 9 '{"exact_raises": 0}' '{"exact_raises": 1}' \
  '{"exact_raises": 0}' '{"exact_raises": 1}' > $OUT/timing_c2.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
grep SUMMARY $OUT/variants_c2.log
cat $OUT/timing_c2.log | grep -v amdgpu.ids | grep -v levels:
echo "session $TAG rc=$rc"
exit $rc
