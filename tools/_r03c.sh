set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c; mkdir -p $O
RTX_LIB=_variants/librtx_stamps.so timeout -k 10 120 python3 tools/stamps_levels.py c2 lv_compact=0 > $O/stamps_c2_nocompact.log 2>&1 && \
RTX_LIB=_variants/librtx_stamps.so timeout -k 10 120 python3 tools/stamps_levels.py c2 lv_compact=1 > $O/stamps_c2_compact.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof8 -o kt --output-format csv -- python3 bench.py --emulate-rank 0/8 --steps 5 --warmup 2 --no-cpu-baseline --no-projection > $O/rank0of8.json 2> $O/rank0of8.err
