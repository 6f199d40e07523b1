#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_dp2_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/r04_dp2_tests.log; exit 1; }
tail -1 gpurun_out/r04_dp2_tests.log
timeout -k 10 900 bash tools/gpu/ab.sh "" "--dp" > gpurun_out/r04_ab_dp2.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/r04_ab_dp2.log; exit 1; }
cat gpurun_out/r04_ab_dp2.log
TAG=trace_dp BENCH_ARGS=--dp timeout -k 10 400 bash tools/gpu/trace.sh && TAG=trace_eng timeout -k 10 400 bash tools/gpu/trace.sh
timeout -k 10 300 python tools/vit_layer_diag.py gpurun_out/r04_vit_layer_diag2.json > gpurun_out/r04_vit_diag2.log 2>&1 || { echo DIAGFAIL; tail -20 gpurun_out/r04_vit_diag2.log; exit 1; }
tail -9 gpurun_out/r04_vit_diag2.log
