set -o pipefail
O=gpurun_out/s17; mkdir -p $O
timeout -k 10 300 python tools/timing.py --scene c2 --reps 7 '{}' '{"lds_stack": 1}' '{"lds_stack": 2}' '{"lds_stack": -1}' '{"lds_stack": 0}' > $O/timing_c2.log 2>&1
echo rc=$?
