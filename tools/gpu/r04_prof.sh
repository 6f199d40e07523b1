#!/bin/bash
# kernel-trace stats of the SGA launch replays (kernel durations vs event-timed launches)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/sga_launches.py 20 > gpurun_out/r04_sga_launches2.txt 2>&1 || { echo SGAFAIL; tail -20 gpurun_out/r04_sga_launches2.txt; exit 1; }
tail -3 gpurun_out/r04_sga_launches2.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_prof -o sga -- python tools/sga_launches.py 20 > gpurun_out/r04_prof.log 2>&1 || { echo PROFFAIL; tail -20 gpurun_out/r04_prof.log; exit 1; }
find gpurun_out/r04_prof -name "*stats*" | head
