# Round-3 closing GPU session, part B: C2 bench with 8- and 4-row share tiles, C4 PMC + bench
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench_tr8.json 2> $OUT/bench_tr8.err && \
timeout -k 10 400 python bench.py --no-cpu-baseline --tile-rows 4 > $OUT/bench_tr4.json 2> $OUT/bench_tr4.err && \
WL=c4 bash tools/gpu_session.sh $TAG pmcbench
