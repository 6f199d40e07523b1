#!/bin/bash
# the norm kernel tests, then one probe script (PROBE=tools/x.py)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "norm" > gpurun_out/r02c_normtest.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02c_normtest.log; exit 1; }
tail -1 gpurun_out/r02c_normtest.log
timeout -k 10 500 python -u $PROBE > gpurun_out/r02c_probe.log 2>&1 || { echo PROBEFAIL; tail -30 gpurun_out/r02c_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r02c_probe.log | grep -v "^autotune" | tail -20
