#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 400 python -u -m pytest tests/test_vit_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02_vit.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r02_vit.log | tail -12; grep -E "^E " gpurun_out/r02_vit.log | head -30; exit $rc
