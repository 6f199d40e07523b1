#!/bin/bash
# the full GPU suite (parity report) + smoke, the first half of r03_record.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r03_gputest.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_gputest.log | tail -20; exit 1; }
grep -E "passed|failed" gpurun_out/r03_gputest.log | tail -1
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
