set -o pipefail
O=gpurun_out/s16; mkdir -p $O
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 120 python tools/stamps.py c2 > $O/stamps_c2.log 2>&1
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 120 python tools/stamps.py c4 > $O/stamps_c4.log 2>&1
bash tools/pmc.sh s16pmc --scene c2 --reps 2
echo rc=$?
