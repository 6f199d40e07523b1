#!/bin/bash
# kernel trace (rocpd sqlite) of the benched step + the per-queue / per-family breakdown of one step
#   BENCH_ARGS: extra bench flags; TAG: output name (default trace); STEPBACK: which step from the
#   end (default 2; 5 for --dp, whose last 3 steps are its timing-report steps)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-trace}
rm -rf gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T -o run -- python bench.py ${BENCH_ARGS:-} --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/$T.log 2>&1 || { echo BFAIL; tail -30 gpurun_out/$T.log; exit 1; }
db=$(find gpurun_out/$T -name "*.db" | head -1)
python tools/steptrace.py $db --list --back ${STEPBACK:-2} > gpurun_out/steptrace_$T.txt
head -30 gpurun_out/steptrace_$T.txt
