#!/bin/bash
# Round 5, session r10z: kernel traces of the C2 frame with the LDS prefetch off and on (per-level
# k_level_c durations), run twice each in alternation.
# (The option existed only in the build this session measured; it was reverted)
#   bash tools/sessions/r10z_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
tr() {  # name option-json
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/$1 -o $1 -- \
    python3 tools/timing.py --scene c2 --reps 9 "$2" > $OUT/$1.log 2>&1
}
tr pf0a '{"lv_prefetch": 0}' && tr pf1a '{"lv_prefetch": 1}' && tr pf0b '{"lv_prefetch": 0}' && tr pf1b '{"lv_prefetch": 1}'
rc=$?
echo "session $TAG rc=$rc"
exit $rc
