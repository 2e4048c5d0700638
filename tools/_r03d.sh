set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 7 '{"lv_compact": 0}' '{"lv_compact": 1}' '{"lv_compact": 0}' '{"lv_compact": 1}' > $O/timing_c2.log 2>&1 && \
true && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_levels.py -x -v --timeout 120 --timeout-method thread > $O/pytest_levels.log 2>&1
