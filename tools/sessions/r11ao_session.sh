#!/bin/bash
# Round 6, session r11ao: query_lbuf's cover lists that overflow (> COVER_K
# covers on one shadow ray) summed in ordered passes over the light buffer's
# cell (RTX_OVF_PASSES=1) instead of the ordered linear walk over every object
# (=0): the raise, light-buffer, hierarchy and level GPU tests on the passes
# build, then C4 and C2 frames alone for _variants old / pass / novf (novf:
# diagnostic, no re-walk at all: wrong where a ray meets > COVER_K covers).
#   bash tools/sessions/r11ao_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
RTX_LIB=_variants/librtx_pass.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_raises.py tests/test_lbuf.py tests/test_gpu_bvh.py tests/test_gpu_levels.py tests/test_gpu_parity.py \
  > $OUT/pytest.log 2>&1 &&
timeout -k 10 600 python3 tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1 &&
timeout -k 10 600 python3 tools/variants.py time --scene c2 --rounds 3 --reps 9 > $OUT/variants_c2.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
grep SUMMARY $OUT/variants_c4.log $OUT/variants_c2.log
echo "session $TAG rc=$rc"
exit $rc
