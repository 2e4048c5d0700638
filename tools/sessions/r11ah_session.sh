#!/bin/bash
# Round 6, session r11ah: the tree reduction's record loads (RTX_FIN_LOADS:
# 1 = a record as two 16-byte loads and one prefetch for a single child,
# 0 = header, first-leaf pair and third component apart, two prefetches):
# C2 and C4 frames alone for the variants (_variants fin0, fin1), then a
# kernel trace of C2 frames for each to read k_tree_finalize's time.
#   bash tools/sessions/r11ah_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python3 tools/variants.py time --scene c2 --rounds 3 --reps 9 > $OUT/variants_c2.log 2>&1 &&
timeout -k 10 600 python3 tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1 &&
for v in fin0 fin1; do
  RTX_LIB=_variants/librtx_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt_$v -o kt -- \
    python3 tools/timing.py --scene c2 --reps 9 '{"lv_streams": 1}' > $OUT/kt_$v.log 2>&1 || exit 1
done
rc=$?
grep SUMMARY $OUT/variants_c2.log $OUT/variants_c4.log
for v in fin0 fin1; do f=$(find $OUT/kt_$v -name '*kernel_stats.csv' | head -1); echo "$v: $(grep tree_finalize $f | cut -d, -f1-4)"; done
echo "session $TAG rc=$rc"
exit $rc
