#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 1000 python -u -m pytest tests/test_vit_gpu.py tests/test_z_vit_bench_step_gpu.py tests/test_z_c5_bench_step_gpu.py tests/test_z_dp_bench_step_gpu.py -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_par_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r04_par_tests.log | tail -30
exit $rc
