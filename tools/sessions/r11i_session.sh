#!/bin/bash
# Round 6, session r11i: ray records moved into bin order by the binning pass
# (option lv_sort_copy): the binned-level GPU tests, then
# C4 frames alone with the copy off and on (auto: on above 512 spheres), and
# C2 with one part per frame (its last level binned) off and on.
#   bash tools/sessions/r11i_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_levels.py -m gpu -x -q -k "binned or binning" --timeout 200 \
  --timeout-method thread > $OUT/pytest_binned.log 2>&1 &&
timeout -k 10 300 python3 tools/timing.py --scene c4 --reps 3 '{"lv_sort_copy": 0}' '{"lv_sort_copy": 1}' \
  '{"lv_sort_copy": 0}' '{"lv_sort_copy": 1}' > $OUT/timing_c4.log 2>&1 &&
timeout -k 10 240 python3 tools/timing.py --scene c2 --reps 9 '{"lv_streams": 1, "lv_sort_copy": 0}' \
  '{"lv_streams": 1, "lv_sort_copy": 1}' '{"lv_streams": 1, "lv_sort_copy": 0}' '{"lv_streams": 1, "lv_sort_copy": 1}' \
  > $OUT/timing_c2.log 2>&1
rc=$?
tail -2 $OUT/pytest_binned.log
cat $OUT/timing_c4.log $OUT/timing_c2.log 2>/dev/null | grep -v amdgpu.ids | grep -v levels: | tail -12
echo "session $TAG rc=$rc"
exit $rc
