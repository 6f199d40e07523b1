#!/bin/bash
# where the step's time goes: stand-alone ResNet call times, then a kernel trace of the benched
# step and its per-kernel list (tools/steptrace.py)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/res_micro.py > gpurun_out/r02c_res_micro.txt 2>&1 || { echo RESFAIL; tail -20 gpurun_out/r02c_res_micro.txt; exit 1; }
tail -3 gpurun_out/r02c_res_micro.txt
rm -rf gpurun_out/r02c_trace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r02c_trace -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-rooflines > gpurun_out/r02c_trace.log 2>&1 || { echo BFAIL; tail -30 gpurun_out/r02c_trace.log; exit 1; }
tail -1 gpurun_out/r02c_trace.log | cut -c1-200
db=$(find gpurun_out/r02c_trace -name "*.db" | head -1)
python tools/steptrace.py $db --list > gpurun_out/r02c_steptrace.txt
head -30 gpurun_out/r02c_steptrace.txt
rm -rf gpurun_out/r02c_trace
