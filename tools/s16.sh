set -o pipefail
O=gpurun_out/s16; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 &&
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 200 python tools/stamps.py c2 > $O/stamps_c2.log 2>&1
echo rc=$?
