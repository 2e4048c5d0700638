#!/bin/bash
# Round 6, session r11h: C2 bench-step A/B on the exact_raises-by-default
# build: last-level binning on/off under frames in flight, 2 vs 3 frames in
# flight, exact_raises 0 for reference; two interleaved rounds.
#   bash tools/sessions/r11h_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
b() {  # name args...
  local n=$1; shift
  timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-projection --steps 40 "$@" > $OUT/$n.json 2> $OUT/$n.err &&
  python3 -c "import json,sys; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('%-12s %8.2f Mpix/s %.4f ms/step single %.2f' % ('$n', d['value'], d['ms_per_step'], d['value_single_frame']))"
}
for r in 1 2; do
  b def$r && b nosort$r --option lv_sort=0 && b xr0_$r --option exact_raises=0 && b f3_$r --inflight 3 &&
  b f3nosort$r --inflight 3 --option lv_sort=0 || exit 1
done
echo "session $TAG rc=0"
