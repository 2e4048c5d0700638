set -o pipefail
# sample-level work items: full GPU tests, timing C2 / C4, lane utilisation stamps.
O=gpurun_out/s15; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python tools/timing.py --scene c2 --reps 7 > $O/timing_c2.log 2>&1 &&
timeout -k 10 300 python tools/timing.py --scene c4 --reps 2 > $O/timing_c4.log 2>&1 &&
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 200 python tools/stamps.py c2 > $O/stamps_c2.log 2>&1 &&
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 300 python tools/stamps.py c4 > $O/stamps_c4.log 2>&1
echo rc=$?
