#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for c in mixs mix; do
  timeout -k 10 120 python -u tools/micro/rccl_capture_probe.py $c > gpurun_out/r04_rccl_probe_$c.log 2>&1 || { echo "PROBEFAIL $c"; grep -v amdgpu.ids gpurun_out/r04_rccl_probe_$c.log | tail -8; exit 1; }
  grep -v amdgpu.ids gpurun_out/r04_rccl_probe_$c.log | grep capture
done
timeout -k 10 300 python -u -m pytest "tests/test_dp_gpu.py::test_dp_world1_matches_single_gpu[True-False]" "tests/test_dp_gpu.py::test_dp_world1_matches_single_gpu[True-True]" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_dp6_tt.log 2>&1 || { echo TTFAIL; grep -E "PASS|FAIL|Error|error" gpurun_out/r04_dp6_tt.log | head; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r04_dp6_tt.log
