#!/bin/bash
# round 3: graph node census, engine rebuild / recapture churn, then the GPU suite with the
# benched-step parity test in the session process (last), smoke, bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 300 python -u tools/graph_probe.py audit > gpurun_out/r03_audit.log 2>&1 || { echo AUDITFAIL; tail -20 gpurun_out/r03_audit.log; exit 1; }
grep -E "^(bench|small)" gpurun_out/r03_audit.log
timeout -k 10 400 python -u tools/graph_probe.py churn ${CHURN:-40} > gpurun_out/r03_churn.log 2>&1 || { echo CHURNFAIL rc=$?; tail -20 gpurun_out/r03_churn.log; exit 1; }
tail -3 gpurun_out/r03_churn.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r03_gputest.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r03_gputest.log | tail -2
grep -E "FAILED|ERROR" gpurun_out/r03_gputest.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; tail -30 gpurun_out/r03_gputest.log; exit $rc; fi
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r03_bench.err; exit 1; }
cat gpurun_out/r03_bench.json
