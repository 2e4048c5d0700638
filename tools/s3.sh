set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bvh.py -x -v --timeout 120 --timeout-method thread > $O/pytest_bvh.log 2>&1; echo "bvh rc=$?"
timeout -k 10 120 python tools/timing.py --scene c2 '{"bvh":0}' '{"bvh":2}' '{"bvh":2,"sphere_src":1}' > $O/timing_c2.log 2>&1 && \
timeout -k 10 180 python tools/timing.py --scene c4 --reps 3 '{"bvh":2}' '{"bvh":2,"sphere_src":1}' > $O/timing_c4.log 2>&1
echo rc=$?
