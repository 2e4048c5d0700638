set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s28; mkdir -p $O
timeout -k 10 300 python tools/timing.py --scene c2 --reps 7 '{}' '{"postpone": 16}' '{"postpone": 8}' '{"tile_order": 0}' '{}' > $O/timing_c2.log 2>&1 &&
timeout -k 10 400 python tools/timing.py --scene c4 --reps 1 '{}' '{"tile_order": 1}' '{"postpone": 24}' '{"postpone": 8}' > $O/timing_c4.log 2>&1
echo rc=$?
timeout -k 10 300 python -u -m pytest tests/test_gpu_bvh.py -x -q --timeout 120 --timeout-method thread > $O/pytest_bvh.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o kt --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_bench.log 2>&1
echo rc2=$?
