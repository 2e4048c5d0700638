set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s7; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "gpu rc=$?"
timeout -k 10 200 python tools/timing.py --scene c2 '{"bvh":0,"lds_stack":0}' '{"bvh":0,"lds_stack":-1}' '{"bvh":2,"lds_stack":0}' '{"bvh":2,"lds_stack":1}' '{"bvh":2,"lds_stack":-1}' > $O/timing_c2.log 2>&1 && \
timeout -k 10 180 python tools/timing.py --scene c4 --reps 3 '{"bvh":2}' > $O/timing_c4.log 2>&1
echo rc=$?
