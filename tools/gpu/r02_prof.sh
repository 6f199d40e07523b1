#!/bin/bash
# round-2 baseline: per-call timings (tuned table) + a kernel trace of the benched step
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/callprof.py 64 --autotune > gpurun_out/r02_callprof.log 2>&1 || { echo CPFAIL; tail -30 gpurun_out/r02_callprof.log; exit 1; }
tail -40 gpurun_out/r02_callprof.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02_bench.log 2>&1 || { echo BFAIL; tail -30 gpurun_out/r02_bench.log; exit 1; }
tail -3 gpurun_out/r02_bench.log
find gpurun_out/r02_prof -name "*.csv" | head
