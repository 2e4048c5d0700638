set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 9 '{}' '{}' '{"bvh": 0}' > $O/timing_c2.log 2>&1 && \
timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 15 --share 0/8 '{}' '{}' > $O/timing_c2_share8.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c4 --reps 2 '{}' > $O/timing_c4.log 2>&1
