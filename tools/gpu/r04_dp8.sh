#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
NCCL_GRAPH_MIXING_SUPPORT=0 TAG=trace_dpm BENCH_ARGS=--dp timeout -k 10 400 bash tools/gpu/trace.sh > gpurun_out/r04_trace_dpm.out 2>&1 || { echo TRFAIL; tail -20 gpurun_out/r04_trace_dpm.out; exit 1; }
head -6 gpurun_out/steptrace_trace_dpm.txt
rm -rf gpurun_out/trace_dpm
export NCCL_GRAPH_MIXING_SUPPORT=0
timeout -k 10 900 bash tools/gpu/ab.sh "" "--dp" > gpurun_out/r04_ab_dp8.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/r04_ab_dp8.log; exit 1; }
cat gpurun_out/r04_ab_dp8.log
