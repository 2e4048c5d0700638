set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s33; mkdir -p $O
timeout -k 10 400 python tools/timing.py --scene c2 --reps 7 '{}' '{"lds_stack": -1}' '{"lds_stack": 2}' '{"bvh": 0}' '{}' '{"lds_stack": -1}' '{"lds_stack": 2}' '{"bvh": 0}' > $O/timing_c2.log 2>&1
echo rc=$?
