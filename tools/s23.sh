set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s23; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_bench.log 2>&1
echo rc=$?
