#!/bin/bash
# r04: DP schedule tests (world 1 RCCL, world 2 gloo incl. config 5, B=64 parity), ViT layer
# diagnostic, engine vs --dp bench, epilogue-patch library A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_a_dp2_gpu.py tests/test_dp_gpu.py tests/test_z_dp_bench_step_gpu.py -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_dp_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r04_dp_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r04_dp_tests.log | tail -12
cp gpurun_out/parity_report.json gpurun_out/r04_dp_parity.json 2>/dev/null
timeout -k 10 300 python tools/vit_layer_diag.py gpurun_out/r04_vit_layer_diag.json > gpurun_out/r04_vit_diag.log 2>&1 || { echo DIAGFAIL; tail -20 gpurun_out/r04_vit_diag.log; exit 1; }
tail -4 gpurun_out/r04_vit_diag.log
timeout -k 10 900 bash tools/gpu/ab.sh "" "--dp" > gpurun_out/r04_ab_dp.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/r04_ab_dp.log; exit 1; }
tail -4 gpurun_out/r04_ab_dp.log
timeout -k 10 900 bash tools/gpu/ab_lib.sh tools/patches/libvqa_hip_base.so tools/patches/libvqa_hip_epi.so 3 2>&1 | tail -6
