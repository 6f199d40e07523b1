#!/bin/bash
# graph execution streams / hardware queues vs step time (bench, no CPU baseline); stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-rooflines"
: skip log



for cfg in ${CFGS:-"GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=16" "DEBUG_HIP_FORCE_GRAPH_QUEUES=3" "GPU_MAX_HW_QUEUES=8 DEBUG_HIP_FORCE_GRAPH_QUEUES=6"}; do
  echo "== $cfg"
  env $cfg timeout -k 10 240 $B > gpurun_out/q_bench.txt 2>&1 || { echo BFAIL; tail -5 gpurun_out/q_bench.txt; exit 1; }
  tail -1 gpurun_out/q_bench.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
