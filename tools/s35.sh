set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s35; mkdir -p $O
timeout -k 10 400 python tools/variants.py time --scene c2 --rounds 4 --reps 5 > $O/variants_c2.log 2>&1
echo rc=$?
