set -o pipefail
# Compiler scheduling-strategy variants, C2 then C4 (interleaved rounds; output sha must match).
O=gpurun_out/s13; mkdir -p $O
timeout -k 10 400 python tools/variants.py time --scene c2 --rounds 3 > $O/variants_c2.log 2>&1 &&
timeout -k 10 600 python tools/variants.py time --scene c4 --rounds 1 --reps 2 > $O/variants_c4.log 2>&1
echo rc=$?
