#!/bin/bash
# Kernel-trace profile of both engines on one scene: bash tools/prof_levels.sh TAG SCENE [timing.py args]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; SCENE=${2:-c2}; shift; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python tools/timing.py --scene $SCENE "$@" '{"engine": 0}' '{"engine": 1}' > $O/timing_$SCENE.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$SCENE -o kt --output-format csv -- \
  python3 tools/timing.py --scene $SCENE --reps 3 "$@" '{"engine": 1}' > $O/prof_$SCENE.log 2>&1
rc=$?
cat $O/timing_$SCENE.log
f=$(ls $O/prof_$SCENE/*kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && cut -d, -f1-8 "$f" | head -12
exit $rc
