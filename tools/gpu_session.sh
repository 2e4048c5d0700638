#!/bin/bash
# One GPU session (round evidence), run on the GPU box from the repo root:
#   bash tools/gpu_session.sh TAG [MODE] [ENGINE]
# MODE: full (default) = tests, smoke, PMC passes, bench (+ projection), kernel-trace stats, C4 bench
#       quick          = tests + bench
#       pmc            = PMC passes + bench + kernel-trace stats
#       bench          = bench + kernel-trace stats
#       levels         = the bounce-level GPU tests only
#       timing         = option sweep: bash tools/gpu_session.sh TAG timing SCENE REPS SHARE OPT...
#                        (SHARE = k/N for one rank's share, or - for the whole frame; each OPT a JSON
#                        option set; output $OUT/timing_SCENE[_shareN].log)
#       baseline       = BASELINE.md's table (tools/baseline_table.py: CPU restatement + 1-GPU + projections)
#       stamps         = phase stamps of the levels engine (diagnostic build diag/librtx_stamps.so):
#                        bash tools/gpu_session.sh TAG stamps SCENE OPT...   (OPT as key=value)
# ENGINE: rtx engine option for the PMC passes (0 lanes, 1 levels; default: the library default)
# WL (environment): workload of the pmc / pmcbench modes, c2 (default) or c4
#       pmcbench       = PMC passes + the workload's bench line + its single-frame kernel-trace summary
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}
MODE=${2:-full}
shift 2 2>/dev/null || shift $#
ENGINE=
if [ "$MODE" != timing ] && [ "$MODE" != stamps ]; then ENGINE=${1:-}; fi
OUT=gpurun_out/$TAG
mkdir -p $OUT profiles
ENGOPT='{}'
WL=${WL:-c2}
ENGNAME=$(python3 -c "import sys; sys.path.insert(0,'.'); print({'0':'lanes','1':'levels'}.get('$ENGINE','default'))")
if [ -n "$ENGINE" ]; then ENGOPT="{\"engine\": $ENGINE}"; fi

tests() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
}
smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
}
pmcpass() {  # name counters...   (one rocprofv3 run per pass; 1 warm-up + 3 timed frames)
  local n=$1; shift
  timeout -k 5 -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/pmc_$n -o $n --output-format csv -- \
    python3 tools/timing.py --scene $WL --reps 3 "$ENGOPT" > $OUT/pmc_$n.log 2>&1
}
pmc() {
  (timeout -k 5 -s KILL 60 rocprofv3 -L > $OUT/rocprof_counters.txt 2>&1 || true) && \
  pmcpass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY && \
  pmcpass b SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR && \
  pmcpass c FETCH_SIZE GRBM_GUI_ACTIVE && \
  pmcpass d WRITE_SIZE && \
  pmcpass f SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY && \
  { if grep -q "SQ_INST_CYCLES_VALU" $OUT/rocprof_counters.txt; then pmcpass e SQ_INST_CYCLES_VALU SQ_INSTS_VALU; else true; fi; } && \
  DIRS="$OUT/pmc_a $OUT/pmc_b $OUT/pmc_c $OUT/pmc_d $OUT/pmc_f" && \
  { [ -d $OUT/pmc_e ] && DIRS="$DIRS $OUT/pmc_e"; true; } && \
  python3 tools/pmc_json.py $OUT/pmc_$WL.json $DIRS --workload $WL --frames 4 --skip 1 --session $TAG \
    --engine $(python3 -c "
import sys; sys.path.insert(0,'.')
from raytracing_rb_amd import config
from raytracing_rb_amd.runtime import Renderer
import json
sd, cd = config.load_scene('scenes/c2_world.yml', 'scenes/${WL}_camera.yml', camera_overrides={'width': 8, 'height': 8})
r = Renderer(sd, cd)
for k, v in json.loads('$ENGOPT').items(): r.set_option(k, v)
print(r.engine())") > $OUT/pmc_json.log 2>&1 && \
  cp $OUT/pmc_$WL.json profiles/pmc_$WL.json
}
bench() {
  timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-projection > $OUT/prof_bench.log 2>&1 && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_single -o kt --output-format csv -- \
    python3 bench.py --inflight 1 --option lv_streams=1 --steps 5 --warmup 2 --no-cpu-baseline --no-projection \
    > $OUT/prof_single.json 2> $OUT/prof_single.err
}
bench_c4() {
  timeout -k 10 600 python bench.py --workload c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
}
bench_c4_single() {   # the C4 roofline's kernel time: one frame alone, one context (as prof_single for C2)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_single_c4 -o kt --output-format csv -- \
    python3 bench.py --workload c4 --inflight 1 --option lv_streams=1 --steps 2 --warmup 1 --no-cpu-baseline \
    --no-projection > $OUT/prof_single_c4.json 2> $OUT/prof_single_c4.err
}

levels() {
  timeout -k 10 400 python -u -m pytest tests/test_gpu_levels.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_levels.log 2>&1
}
timing() {  # SCENE REPS SHARE OPT...
  local scene=$1 reps=$2 share=$3; shift 3
  local log=$OUT/timing_$scene.log sh=()
  if [ "$share" != - ]; then sh=(--share $share); log=$OUT/timing_${scene}_share${share#*/}.log; fi
  timeout -k 10 300 python3 tools/timing.py --scene $scene --reps $reps "${sh[@]}" "$@" >> $log 2>&1
}
stamps() {  # SCENE OPT...
  local scene=$1; shift
  RTX_LIB=${STAMPS_LIB:-diag/librtx_stamps.so} timeout -k 10 120 python3 tools/stamps_levels.py $scene "$@" \
    > $OUT/stamps_${scene}_$(echo "$@" | tr ' =' '_-').log 2>&1
}

baseline() {
  timeout -k 10 900 python3 tools/baseline_table.py $OUT > $OUT/baseline.log 2>&1
}

case $MODE in
  levels) levels ;;
  baseline) baseline ;;
  timing) timing "$@" ;;
  stamps) stamps "$@" ;;
  full)  tests && smoke && pmc && bench && bench_c4 ;;
  quick) tests && timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err ;;
  pmc)   pmc && bench ;;
  pmcbench) if [ "$WL" = c4 ]; then pmc && bench_c4 && bench_c4_single; else pmc && bench; fi ;;
  bench) bench ;;
  *) echo "unknown mode $MODE"; false ;;
esac
rc=$?
echo "session $TAG $MODE rc=$rc"
exit $rc
