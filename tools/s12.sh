set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s12; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "gpu rc=$?"
timeout -k 10 300 python tools/variants.py time --scene c2 --rounds 3 > $O/variants_c2.log 2>&1
timeout -k 10 300 python tools/variants.py time --scene c4 --rounds 2 > $O/variants_c4.log 2>&1
echo rc=$?
