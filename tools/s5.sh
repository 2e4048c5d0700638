set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s5; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "gpu rc=$?"
timeout -k 10 120 python tools/timing.py --scene c2 '{"bvh":0}' '{"bvh":2}' > $O/timing_c2.log 2>&1 && \
timeout -k 10 180 python tools/timing.py --scene c4 --reps 3 '{"bvh":2}' > $O/timing_c4.log 2>&1
echo rc=$?
