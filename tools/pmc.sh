#!/bin/bash
# PMC passes (one rocprofv3 run per pass, counters within the per-block slot limits)
# over a few C2 frames: tools/pmc.sh TAG [timing.py args...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
ARGS=("$@")
run() {  # name counters...
  local n=$1; shift
  timeout -k 5 -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d $O/pmc_$n -o $n --output-format csv -- python3 tools/timing.py "${ARGS[@]}" > $O/pmc_$n.log 2>&1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY && \
run b SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_INT32 && \
run c SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY && \
run d FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT && \
run e WRITE_SIZE
