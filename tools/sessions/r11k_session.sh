#!/bin/bash
# Round 6, session r11k: the parts' launch steps issued in turn (launch_levels):
# GPU tests, the C2 1/8 share and the full frame one at a time, C4 alone, a
# kernel trace of the share, the default bench line.
#   bash tools/sessions/r11k_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 240 python3 tools/timing.py --scene c2 --share 0/8 --reps 15 '{}' '{"lv_streams": 1}' '{}' \
  '{"lv_streams": 1}' > $OUT/timing_share8.log 2>&1 &&
timeout -k 10 240 python3 tools/timing.py --scene c2 --reps 9 '{}' '{"lv_streams": 1}' '{}' > $OUT/timing_full.log 2>&1 &&
timeout -k 10 300 python3 tools/timing.py --scene c4 --reps 3 '{}' > $OUT/timing_c4.log 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/share8 -o share8 -- \
  python3 tools/timing.py --scene c2 --share 0/8 --reps 9 '{}' > $OUT/share8_trace.log 2>&1 &&
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
tail -2 $OUT/pytest_gpu.log
cat $OUT/timing_share8.log $OUT/timing_full.log $OUT/timing_c4.log | grep -v amdgpu.ids | grep -v levels:
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['value_single_frame'], {n: (v['projected_speedup'], v['lpt']['projected_speedup']) for n, v in d['projection']['per_n'].items()})"
echo "session $TAG rc=$rc"
exit $rc
