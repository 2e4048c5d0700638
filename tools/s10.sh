set -o pipefail
O=gpurun_out/s10; mkdir -p $O
timeout -k 10 300 python tools/variants.py time --scene c2 --rounds 3 > $O/variants_c2.log 2>&1
echo rc=$?
