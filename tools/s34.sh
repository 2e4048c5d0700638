set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s34; mkdir -p $O
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_20.json 2> $O/bench_20.err &&
timeout -k 10 200 python bench.py --steps 3000 --warmup 3 --no-cpu-baseline > $O/bench_3000.json 2> $O/bench_3000.err &&
(timeout 5 rocm-smi --showclocks --showpower --showtemp > $O/smi_after.txt 2>&1 || true) &&
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_20_after.json 2> $O/bench_20_after.err
echo rc=$?
