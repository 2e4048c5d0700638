set -o pipefail
O=gpurun_out/s8; mkdir -p $O
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 120 python tools/stamps.py c2 bvh=2 > $O/stamps_c2_bvh.log 2>&1
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 120 python tools/stamps.py c2 bvh=0 > $O/stamps_c2_lin.log 2>&1
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 120 python tools/stamps.py c4 bvh=2 > $O/stamps_c4_bvh.log 2>&1
echo rc=$?
