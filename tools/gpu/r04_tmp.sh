#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py tests/test_a_dp2_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_tmp_tests.log 2>&1 || { echo TESTFAIL; grep -E "Error|assert" gpurun_out/r04_tmp_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r04_tmp_tests.log
timeout -k 10 1100 bash tools/gpu/ab.sh "" "--dp" "--hw-queues 8" "--dp --hw-queues 8" > gpurun_out/r04_ab_dp12.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/r04_ab_dp12.log; exit 1; }
cat gpurun_out/r04_ab_dp12.log
