#!/bin/bash
# Round 6, sessions r11ai, r11aj: raise lists starting 16-byte aligned, four entries
# per load (rtx_scene.h rbuf_head): the raise, light-buffer and hierarchy GPU
# tests on the default build, then C4 and C2 frames alone for _variants al0
# (entries loaded one at a time), al1 (16-byte loads in every kernel; the
# default build of r11ai) and al2 (16-byte loads in the large-scene kernels
# only; the default build of r11aj), interleaved.
#   bash tools/sessions/r11ai_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_raises.py \
  tests/test_lbuf.py tests/test_gpu_bvh.py > $OUT/pytest.log 2>&1 &&
timeout -k 10 600 python3 tools/variants.py time --scene c4 --rounds 3 --reps 2 > $OUT/variants_c4.log 2>&1 &&
timeout -k 10 600 python3 tools/variants.py time --scene c2 --rounds 3 --reps 9 > $OUT/variants_c2.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
grep SUMMARY $OUT/variants_c4.log $OUT/variants_c2.log
echo "session $TAG rc=$rc"
exit $rc
