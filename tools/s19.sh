set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s19; mkdir -p $O
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 200 python tools/stamps.py c2 > $O/stamps_c2.log 2>&1 &&
bash tools/pmc.sh s19 --scene c2 --reps 2 && python tools/pmcsum.py gpurun_out/s19 > $O/pmcsum.log 2>&1
echo rc=$?
