#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_a_dp2_gpu.py tests/test_dp_gpu.py tests/test_parity_gpu.py -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider -k "dp or grouping" > gpurun_out/r02_dpcheck.log 2>&1
rc=$?; tail -3 gpurun_out/r02_dpcheck.log; grep -E "^E " gpurun_out/r02_dpcheck.log | head -10; exit $rc
