#!/bin/bash
# Round-4 GPU session (C4 quantized leaves): GPU tests, C4 A/B of the sphere
# modes (auto = SPH_BVH_QLDS vs sphere_src 2 = nodes in LDS, leaves global),
# then the C4 PMC passes + bench line + single-frame kernel trace.
#     bash tools/sessions/r08_session.sh TAG [nopmc]
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 400 python3 tools/timing.py --scene c4 --reps 3 '{}' '{"sphere_src": 2}' '{}' > $OUT/timing_c4.log 2>&1 && \
timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' > $OUT/timing_c2.log 2>&1 && \
{ if [ "$2" = nopmc ]; then true; else WL=c4 bash tools/gpu_session.sh ${TAG}4 pmcbench; fi; }
rc=$?
echo "session $TAG rc=$rc"
exit $rc
