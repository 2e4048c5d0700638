# Instruction-cache counters of the level kernels (diagnostic): two rocprofv3 --pmc passes
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 5 -s KILL 180 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --kernel-trace -d $OUT/ic1 -o ic1 --output-format csv -- \
  python3 tools/timing.py --scene c2 --reps 3 '{}' > $OUT/ic1.log 2>&1 && \
timeout -k 5 -s KILL 180 rocprofv3 --pmc SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d $OUT/ic2 -o ic2 --output-format csv -- \
  python3 tools/timing.py --scene c2 --reps 3 '{}' > $OUT/ic2.log 2>&1
