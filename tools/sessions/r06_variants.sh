# Interleaved timing of the in-tree build against diagnostic variants in var/ (C2 frame alone)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 9 '{}' >> $OUT/timing_head.log 2>&1 || exit 1
  for v in var/*.so; do
    RTX_LIB=$v timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 9 '{}' >> $OUT/timing_$(basename $v .so).log 2>&1 || exit 1
  done
done
