set -o pipefail
O=gpurun_out/s17; mkdir -p $O
timeout -k 10 200 python tools/timing.py --scene c2 '{"bvh":0}' '{"bvh":2}' '{"bvh":2,"lds_stack":0}' '{"bvh":0}' '{"bvh":2}' > $O/timing_c2.log 2>&1
timeout -k 10 200 python tools/timing.py --scene c4 --reps 3 '{"bvh":2}' '{"bvh":2,"sphere_src":1}' > $O/timing_c4.log 2>&1
echo rc=$?
