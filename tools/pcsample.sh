#!/bin/bash
# PC-sampling probe of the level kernels on one scene (diagnostic):
#   bash tools/pcsample.sh TAG [SCENE] [OPTS_JSON]
# rocprofv3's stochastic (hardware) sampler first; the host-trap sampler if that
# configuration is not available.  Output: gpurun_out/TAG/pcs*/ (csv), then
# tools/pcsum.py maps the samples to the ISA of the sampled code objects.
set -o pipefail
export TMPDIR=/tmp
TAG=$1; SCENE=${2:-c2}; OPTS=${3:-'{}'}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 5 -s KILL 60 rocprofv3 -L > $OUT/rocprof_list.txt 2>&1 || true
timeout -k 5 -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
  --pc-sampling-unit cycles --pc-sampling-interval 65536 -d $OUT/pcs_stoch -o pcs --output-format csv -- \
  python3 tools/timing.py --scene $SCENE --reps 2 "$OPTS" > $OUT/pcs_stoch.log 2>&1
rc=$?
echo "stochastic rc=$rc" >> $OUT/pcs_stoch.log
if [ $rc -ne 0 ] && [ $rc -ne 124 ] && [ $rc -ne 137 ] && [ $rc -ne 134 ] && [ $rc -ne 139 ]; then
  timeout -k 5 -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
    --pc-sampling-unit time --pc-sampling-interval 1 -d $OUT/pcs_trap -o pcs --output-format csv -- \
    python3 tools/timing.py --scene $SCENE --reps 2 "$OPTS" > $OUT/pcs_trap.log 2>&1
  rc=$?
  echo "host_trap rc=$rc" >> $OUT/pcs_trap.log
fi
exit $rc
