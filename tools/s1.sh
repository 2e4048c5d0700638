set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
RTX_LIB=build/diag/librtx_stamps.so timeout -k 10 120 python tools/stamps.py c2 > $O/stamps1.log 2>&1 && \
RTX_LIB=build/diag/librtx_stamps2.so timeout -k 10 120 python tools/stamps.py c2 > $O/stamps2.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo rc=$?
