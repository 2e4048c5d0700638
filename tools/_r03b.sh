set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 7 '{"lv_compact": 0}' '{"lv_compact": 1}' '{"lv_compact": 0}' '{"lv_compact": 1}' > gpurun_out/r03b/timing_c2.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03b/prof -o kt --output-format csv -- python3 tools/timing.py --scene c2 --reps 2 '{"lv_compact": 1}' > gpurun_out/r03b/prof.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c4 --reps 2 '{"lv_compact": 0}' '{"lv_compact": 1}' > gpurun_out/r03b/timing_c4.log 2>&1
