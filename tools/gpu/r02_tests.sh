#!/bin/bash
# full GPU test suite (every test, measurements -> gpurun_out/parity_report.json), smoke, bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r02_gputest.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/r02_gputest.log | tail -5
grep -E "FAILED|ERROR" gpurun_out/r02_gputest.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r02_smoke.log; exit 1; }
tail -2 gpurun_out/r02_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r02_bench1.json 2> gpurun_out/r02_bench1.err || { echo BENCHFAIL; tail -20 gpurun_out/r02_bench1.err; exit 1; }
cat gpurun_out/r02_bench1.json
exit $rc
