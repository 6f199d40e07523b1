#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider \
   -k "golden or multistep" > gpurun_out/r02_parity.log 2>&1
rc=$?
tail -5 gpurun_out/r02_parity.log
exit $rc
