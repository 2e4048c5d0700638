set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s21; mkdir -p $O
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 200 python tools/stamps.py c2 tile_order=0 > $O/stamps_c2_0.log 2>&1 &&
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 200 python tools/stamps.py c2 tile_order=1 > $O/stamps_c2_1.log 2>&1 &&
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 200 python tools/stamps.py c4 tile_order=0 > $O/stamps_c4_0.log 2>&1 &&
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 200 python tools/stamps.py c4 tile_order=1 > $O/stamps_c4_1.log 2>&1
echo rc=$?
