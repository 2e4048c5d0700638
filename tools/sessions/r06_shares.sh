set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
for tr in 8 4 2; do
  for k in 0 1 2 3 4 5 6 7; do
    timeout -k 10 120 python3 tools/timing.py --scene c2 --reps 6 --inflight 2 --share $k/8 --tile-rows $tr '{}' >> $OUT/shares_tr$tr.log 2>&1 || exit 1
  done
done
