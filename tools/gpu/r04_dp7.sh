#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 bash tools/gpu/ab.sh "" "--dp-groups" "--dp" > gpurun_out/r04_ab_dp7.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/r04_ab_dp7.log; exit 1; }
cat gpurun_out/r04_ab_dp7.log
TAG=trace_dp BENCH_ARGS=--dp timeout -k 10 400 bash tools/gpu/trace.sh > gpurun_out/r04_trace_dp.out 2>&1 || { echo TRFAIL; tail -20 gpurun_out/r04_trace_dp.out; exit 1; }
TAG=trace_dpg BENCH_ARGS=--dp-groups timeout -k 10 400 bash tools/gpu/trace.sh > gpurun_out/r04_trace_dpg.out 2>&1 || { echo TRFAIL2; tail -20 gpurun_out/r04_trace_dpg.out; exit 1; }
rm -rf gpurun_out/trace_dp gpurun_out/trace_dpg
head -12 gpurun_out/steptrace_trace_dp.txt; head -12 gpurun_out/steptrace_trace_dpg.txt
