set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 9 '{"lv_grid_div": 1}' '{"lv_grid_div": 2}' '{"lv_grid_div": 1, "lv_streams": 1}' '{"lv_grid_div": 1}' '{"lv_grid_div": 2}' > $O/timing_c2.log 2>&1 && \
timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 15 --share 0/8 '{"lv_grid_div": 1}' '{"lv_grid_div": 2}' '{"lv_grid_div": 1}' '{"lv_grid_div": 2}' '{"lv_grid_div": 2, "lv_static": 80}' '{"lv_grid_div": 1, "lv_static": 80}' > $O/timing_c2_share8.log 2>&1
