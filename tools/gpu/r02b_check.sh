#!/bin/bash
# session re-entry check: GPU suite, smoke, per-call timings of the benched (tuned) step
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r02b_gputest.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r02b_gputest.log | tail -2
grep -E "FAILED|ERROR" gpurun_out/r02b_gputest.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02b_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r02b_smoke.log; exit 1; }
tail -1 gpurun_out/r02b_smoke.log
timeout -k 10 300 python tools/callprof.py 64 --autotune > gpurun_out/r02b_callprof.log 2>&1 || { echo CPFAIL; tail -30 gpurun_out/r02b_callprof.log; exit 1; }
tail -25 gpurun_out/r02b_callprof.log
