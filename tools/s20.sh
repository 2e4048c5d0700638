set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s20; mkdir -p $O
timeout -k 10 300 python tools/timing.py --scene c2 --reps 7 '{"tile_order": 0}' '{"tile_order": 1}' '{"tile_order": 0}' '{"tile_order": 1}' > $O/timing_c2.log 2>&1 &&
timeout -k 10 400 python tools/timing.py --scene c4 --reps 2 '{"tile_order": 0}' '{"tile_order": 1}' > $O/timing_c4.log 2>&1
echo rc=$?
