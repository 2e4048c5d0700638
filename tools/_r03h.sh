set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_levels.py -x -v --timeout 120 --timeout-method thread > $O/pytest_levels.log 2>&1 && \
timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 9 '{"lv_streams": 1}' '{"lv_streams": 2}' '{"lv_streams": 3}' '{"lv_streams": 4}' '{"lv_streams": 2}' '{"lv_streams": 3}' > $O/timing_c2.log 2>&1 && \
timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 15 --share 0/8 '{"lv_streams": 1}' '{"lv_streams": 2}' '{"lv_streams": 3}' '{"lv_streams": 4}' '{"lv_streams": 2}' '{"lv_streams": 3}' '{"lv_streams": 4}' > $O/timing_c2_share8.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c4 --reps 2 '{"lv_streams": 2}' '{"lv_streams": 3}' '{"lv_streams": 4}' > $O/timing_c4.log 2>&1
