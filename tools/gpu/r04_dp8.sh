#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py tests/test_a_dp2_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_dp8_tests.log 2>&1 || { echo TESTFAIL; grep -E "FAIL|Error" gpurun_out/r04_dp8_tests.log | head -20; tail -30 gpurun_out/r04_dp8_tests.log; exit 1; }
tail -1 gpurun_out/r04_dp8_tests.log
timeout -k 10 1000 bash tools/gpu/ab.sh "" "--dp-groups" "--dp" > gpurun_out/r04_ab_dp11.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/r04_ab_dp11.log; exit 1; }
cat gpurun_out/r04_ab_dp11.log
python -c "import json;d=json.load(open('gpurun_out/ab_6.json'));print(json.dumps(d['dp']))"
TAG=trace_dps BENCH_ARGS=--dp timeout -k 10 400 bash tools/gpu/trace.sh > gpurun_out/r04_trace_dps.out 2>&1 || { echo TRFAIL; tail -20 gpurun_out/r04_trace_dps.out; exit 1; }
head -7 gpurun_out/steptrace_trace_dps.txt
rm -rf gpurun_out/trace_dps
