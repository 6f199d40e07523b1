#!/bin/bash
# the full GPU suite alone (one process), with the per-test memory log
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json gpurun_out/gpu_mem.log
VQA_TEST_NO_GC=${VQA_TEST_NO_GC:-0} AMD_LOG_LEVEL=1 timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r02_gputest.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r02_gputest.log | tail -2
grep -E "FAILED|ERROR|Fatal|:1:" gpurun_out/r02_gputest.log | head -20
echo "pytest rc=$rc"; exit $rc
