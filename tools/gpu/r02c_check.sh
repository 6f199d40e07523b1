#!/bin/bash
# session-c state check: the full GPU suite, smoke, and the default bench (no CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r02c_gputest.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r02c_gputest.log | tail -2
grep -E "FAILED|ERROR" gpurun_out/r02c_gputest.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02c_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r02c_smoke.log; exit 1; }
tail -1 gpurun_out/r02c_smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/r02c_bench.json 2> gpurun_out/r02c_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r02c_bench.err; exit 1; }
cat gpurun_out/r02c_bench.json
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 400 python -u $EXTRA > gpurun_out/r02c_extra.log 2>&1 || { echo EXTRAFAIL; tail -20 gpurun_out/r02c_extra.log; exit 1; }
  tail -8 gpurun_out/r02c_extra.log
fi
