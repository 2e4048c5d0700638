set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03e; mkdir -p $O
(timeout -k 5 -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true)
grep -i -A12 "pc_sampling\|PC sampling" $O/avail.txt > $O/pcs_avail.txt || true
timeout -k 5 -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $O/pcs -o pcs --output-format csv -- python3 tools/timing.py --scene c2 --reps 2 '{"lv_compact": 1}' > $O/pcs.log 2>&1
echo "pcs rc=$?"
