set -o pipefail
# SAH vs median hierarchy: GPU bit-identity tests, then interleaved timing on C2 and C4.
O=gpurun_out/s11; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bvh.py -x -q --timeout 120 --timeout-method thread > $O/pytest_bvh.log 2>&1 &&
timeout -k 10 300 python tools/variants.py time --scene c2 --rounds 3 > $O/variants_c2.log 2>&1 &&
timeout -k 10 500 python tools/variants.py time --scene c4 --rounds 2 --reps 2 > $O/variants_c4.log 2>&1
echo rc=$?
