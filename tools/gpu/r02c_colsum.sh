#!/bin/bash
# GPU suite, then same-box A/B of the off-chain column sums (VQA_COLSUM_SIDE)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r02c_gputest.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r02c_gputest.log | tail -1
grep -E "FAILED|ERROR" gpurun_out/r02c_gputest.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash tools/gpu/ab_env.sh VQA_COLSUM_SIDE=0 VQA_COLSUM_SIDE=1
