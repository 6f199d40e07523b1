#!/bin/bash
# GEMM probe: event timings + in-kernel durations (kernel trace) per case
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/probe_kt
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/gpurun_out/probe_kt -o kt -- python3 tools/gemm_probe.py gpurun_out/probe_man.json > gpurun_out/probe.log 2>&1 || { echo PROBEFAIL; tail -20 gpurun_out/probe.log; exit 1; }
python3 tools/gemm_probe.py --trace gpurun_out/probe_kt gpurun_out/probe_man.json > gpurun_out/probe_trace.txt 2>&1
cat gpurun_out/probe_trace.txt
