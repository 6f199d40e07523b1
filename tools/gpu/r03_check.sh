#!/bin/bash
# round 3 state check: the full GPU suite (benched-step parity in the session process, last),
# smoke, and the default bench (no CPU baseline); EXTRA = an optional script run after them
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} \
   > gpurun_out/r03_gputest.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r03_gputest.log | tail -2
grep -E "FAILED|ERROR" gpurun_out/r03_gputest.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r03_bench.err; exit 1; }
cat gpurun_out/r03_bench.json
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 600 bash -c "$EXTRA" > gpurun_out/r03_extra.log 2>&1 || { echo EXTRAFAIL; tail -20 gpurun_out/r03_extra.log; exit 1; }
  tail -8 gpurun_out/r03_extra.log
fi
