#!/bin/bash
# GEMM GPU tests, then the phase-stamp micro benchmark
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02c_gemmtest.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r02c_gemmtest.log; exit 1; }
tail -1 gpurun_out/r02c_gemmtest.log
timeout -k 10 120 tools/micro/gemm_stamps
