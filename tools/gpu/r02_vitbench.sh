#!/bin/bash
# config 4 bench (tile choices saved for the table) + a kernel-trace profile of it
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --model vit --tune-save gpurun_out/tune_vit.json > gpurun_out/r02_vitbench.json 2> gpurun_out/r02_vitbench.err || { echo VBFAIL; tail -20 gpurun_out/r02_vitbench.err; exit 1; }
cat gpurun_out/r02_vitbench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r02_vitkt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --model vit --steps 10 --warmup 3 --no-cpu-baseline --tune-table $GRAFT_REPO_ROOT/gpurun_out/tune_vit.json > $GRAFT_REPO_ROOT/gpurun_out/r02_vitkt.log 2>&1 || { echo KTFAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/r02_vitkt.log; exit 1; }
head -12 $GRAFT_REPO_ROOT/gpurun_out/r02_vitkt/kt_kernel_stats.csv | cut -c1-160
