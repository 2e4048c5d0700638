#!/bin/bash
# Round 6, session r11r: what exact_raises adds to a C4 frame, by counters:
# two PMC passes each with exact_raises 0 and 1 (instruction mix, waits).
#   bash tools/sessions/r11r_session.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
pass() {  # name option counters...
  local n=$1 o=$2; shift 2
  timeout -k 5 -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/pmc_$n -o $n --output-format csv -- \
    python3 tools/timing.py --scene c4 --reps 1 "$o" > $OUT/pmc_$n.log 2>&1
}
pass a0 '{"exact_raises": 0}' SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY &&
pass a1 '{"exact_raises": 1}' SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY &&
pass b0 '{"exact_raises": 0}' SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY &&
pass b1 '{"exact_raises": 1}' SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY
rc=$?
python3 - <<'PY'
import csv, glob, collections
for n in ("a0", "a1", "b0", "b1"):
    tot = collections.Counter()
    for f in glob.glob("gpurun_out/%s/pmc_%s/*counter_collection.csv" % ("$TAG", n)):
        for r in csv.DictReader(open(f)):
            if "k_level_c" in r.get("Kernel_Name", ""):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print(n, {k: "%.4g" % v for k, v in sorted(tot.items())})
PY
echo "session $TAG rc=$rc"
exit $rc
