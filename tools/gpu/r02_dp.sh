#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_a_dp2_gpu.py tests/test_dp_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02_dp.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r02_dp.log | tail -12; grep -E "^E " gpurun_out/r02_dp.log | head -20; exit $rc
