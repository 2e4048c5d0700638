set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s15; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "gpu rc=$?"
timeout -k 10 300 python tools/variants.py time --scene c2 --rounds 3 > $O/variants_c2.log 2>&1
timeout -k 10 100 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $O/pmc_write -o pw --output-format csv -- python3 tools/timing.py --scene c2 --reps 2 > $O/pmc_w.log 2>&1
timeout -k 10 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_fetch -o pf --output-format csv -- python3 tools/timing.py --scene c2 --reps 2 > $O/pmc_f.log 2>&1
echo rc=$?
