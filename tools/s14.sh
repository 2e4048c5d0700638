set -o pipefail
O=gpurun_out/s14; mkdir -p $O
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 200 python tools/stamps.py c2 > $O/stamps_c2.log 2>&1 &&
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 300 python tools/stamps.py c4 > $O/stamps_c4.log 2>&1
echo rc=$?
