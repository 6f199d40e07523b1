#!/bin/bash
# kernel trace (rocpd sqlite) of the benched step + the per-queue / per-family breakdown of one step
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/trace -o run -- python bench.py ${BENCH_ARGS:-} --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-rooflines > gpurun_out/trace.log 2>&1 || { echo BFAIL; tail -30 gpurun_out/trace.log; exit 1; }
tail -1 gpurun_out/trace.log | cut -c1-200
db=$(find gpurun_out/trace -name "*.db" | head -1)
python tools/steptrace.py $db --list > gpurun_out/steptrace.txt
head -40 gpurun_out/steptrace.txt
