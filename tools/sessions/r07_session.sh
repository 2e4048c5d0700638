# Round-4 GPU session: tests, smoke, variant A/B (tools/variants.py: every
# library under _variants/), C2 bench, single-frame kernel-trace summary,
# C4 variants.     bash tools/sessions/r07_session.sh TAG [exact]
#   (exact: also time option exact_raises on C2 / C4)
set -o pipefail
export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 300 python tools/variants.py time --scene c2 --rounds 3 --reps 7 > $OUT/variants_c2.log 2>&1 && \
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_single -o kt --output-format csv -- \
    python3 bench.py --inflight 1 --option lv_streams=1 --steps 5 --warmup 2 --no-cpu-baseline --no-projection \
    > $OUT/prof_single.json 2> $OUT/prof_single.err && \
timeout -k 10 300 python tools/variants.py time --scene c4 --rounds 2 --reps 2 > $OUT/variants_c4.log 2>&1 && \
{ if [ "$2" = exact ]; then
    timeout -k 10 300 python3 tools/timing.py --scene c2 --reps 7 '{}' '{"exact_raises": 1}' > $OUT/timing_c2.log 2>&1 && \
    timeout -k 10 300 python3 tools/timing.py --scene c4 --reps 2 '{}' '{"exact_raises": 1}' > $OUT/timing_c4.log 2>&1
  else true; fi; }
rc=$?
echo "session $TAG rc=$rc"
exit $rc
