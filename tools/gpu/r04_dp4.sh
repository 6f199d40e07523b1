#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cp t5-resnet-vqa_amd/lib/libvqa_hip.so tools/patches/libvqa_hip_wt.so
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gemm_tests.log 2>&1 || { echo GEMMFAIL; tail -40 gpurun_out/r04_gemm_tests.log; exit 1; }
tail -1 gpurun_out/r04_gemm_tests.log
timeout -k 10 900 python -u -m pytest tests/test_dp_gpu.py tests/test_a_dp2_gpu.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_dp4_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r04_dp4_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r04_dp4_tests.log | tail -12
timeout -k 10 900 bash tools/gpu/ab_lib.sh tools/patches/libvqa_hip_wt.so tools/patches/libvqa_hip_plain.so 2 > gpurun_out/r04_ab_wt.log 2>&1 || { echo ABWTFAIL; tail -20 gpurun_out/r04_ab_wt.log; exit 1; }
cat gpurun_out/r04_ab_wt.log
timeout -k 10 900 bash tools/gpu/ab.sh "" "--dp" > gpurun_out/r04_ab_dp4.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/r04_ab_dp4.log; exit 1; }
cat gpurun_out/r04_ab_dp4.log
