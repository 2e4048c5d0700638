#!/bin/bash
# One GPU session (round evidence): tests, smoke, PMC traffic passes, bench, kernel-trace stats.
#   bash tools/gpu_session.sh TAG
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o pf --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 && \
timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o pw --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1 && \
python tools/pmc_json.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_k_render.json --workload c2 > /dev/null && \
mkdir -p profiles && cp $OUT/pmc_k_render.json profiles/pmc_k_render.json && \
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof_bench.log 2>&1 && \
timeout -k 10 600 python bench.py --workload c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
rc=$?
echo "session rc=$rc"
exit $rc
