set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_levels.py tests/test_gpu_parity.py tests/test_gpu_bvh.py > $O/pytest.log 2>&1 &&
timeout -k 10 300 python tools/timing.py --scene c2 --reps 9 '{"lv_ray_bytes":96}' '{"lv_ray_bytes":80}' '{"lv_ray_bytes":96}' '{"lv_ray_bytes":80}' > $O/timing_c2.log 2>&1 &&
timeout -k 10 300 python tools/timing.py --scene c2 --share 0/8 --reps 15 '{"lv_ray_bytes":96}' '{"lv_ray_bytes":80}' '{"lv_ray_bytes":96}' '{"lv_ray_bytes":80}' > $O/timing_share8.log 2>&1 &&
timeout -k 10 300 python bench.py --emulate-rank 0/8 --no-projection --steps 200 --inflight 2 > $O/share8_f2.json 2> $O/share8_f2.err &&
timeout -k 10 300 python bench.py --emulate-rank 0/8 --no-projection --steps 200 --inflight 3 > $O/share8_f3.json 2> $O/share8_f3.err &&
timeout -k 10 300 python bench.py --emulate-rank 0/8 --no-projection --steps 200 --inflight 4 > $O/share8_f4.json 2> $O/share8_f4.err &&
timeout -k 10 500 python tools/timing.py --scene c4 --reps 2 '{"lv_ray_bytes":96}' '{"lv_ray_bytes":80}' > $O/timing_c4.log 2>&1
rc=$?
[ $rc = 0 ] && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_single -o kt --output-format csv -- \
    python3 bench.py --inflight 1 --option lv_streams=1 --steps 5 --warmup 2 --no-cpu-baseline --no-projection \
    > $O/prof_single.json 2> $O/prof_single.err
echo "r05p rc=$rc $?"
