set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r07f; mkdir -p $OUT
timeout -k 10 300 python tools/variants.py time --scene c2 --rounds 4 --reps 7 > $OUT/variants_c2.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"lv_fin_cap": 0}' '{"lv_fin_cap": 4096}' '{}' > $OUT/timing_fin_c2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_fin0 -o kt --output-format csv -- \
    python3 bench.py --inflight 1 --option lv_streams=1 --option lv_fin_cap=0 --steps 5 --warmup 2 --no-cpu-baseline --no-projection \
    > $OUT/prof_fin0.json 2> $OUT/prof_fin0.err
echo rc=$?
