#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
cp t5-resnet-vqa_amd/lib/libvqa_hip.so tools/patches/libvqa_hip_wt.so
timeout -k 10 900 python -u -m pytest tests/test_dp_gpu.py tests/test_a_dp2_gpu.py tests/test_z_dp_bench_step_gpu.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_dp5_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r04_dp5_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r04_dp5_tests.log | tail -14
timeout -k 10 900 bash tools/gpu/ab.sh "" "--dp" > gpurun_out/r04_ab_dp5.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/r04_ab_dp5.log; exit 1; }
cat gpurun_out/r04_ab_dp5.log
timeout -k 10 900 bash tools/gpu/ab_lib.sh tools/patches/libvqa_hip_wt.so tools/patches/libvqa_hip_plain.so 2 > gpurun_out/r04_ab_wt.log 2>&1 || { echo ABWTFAIL; tail -20 gpurun_out/r04_ab_wt.log; exit 1; }
cat gpurun_out/r04_ab_wt.log
