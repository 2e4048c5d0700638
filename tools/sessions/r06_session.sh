set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 && \
for i in 1 2; do
RTX_LIB=var/librtx_base.so timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 9 '{}' >> $OUT/timing_base.log 2>&1 && \
timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 9 '{}' '{"sphere_src": 0}' >> $OUT/timing_new.log 2>&1 || exit 1
done
RTX_LIB=var/librtx_base.so timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 9 --share 0/8 '{}' >> $OUT/timing_base.log 2>&1 && \
timeout -k 10 200 python3 tools/timing.py --scene c2 --reps 9 --share 0/8 '{}' >> $OUT/timing_new.log 2>&1
