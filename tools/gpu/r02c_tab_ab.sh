#!/bin/bash
# same-box A/B: config-2 bench with the table before the config-4 re-time vs the current table
# (first: git show 4929727:t5-resnet-vqa_amd/tuning/gemm_gfx950.json > tools/gpu/_old_table.json)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
i=0
for t in tools/gpu/_old_table.json t5-resnet-vqa_amd/tuning/gemm_gfx950.json tools/gpu/_old_table.json t5-resnet-vqa_amd/tuning/gemm_gfx950.json tools/gpu/_old_table.json t5-resnet-vqa_amd/tuning/gemm_gfx950.json; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --tune-table $t > gpurun_out/tab_$i.json 2> gpurun_out/tab.err || { echo BENCHFAIL; tail -20 gpurun_out/tab.err; exit 1; }
  echo "[$t]" $(python -c "import json;d=json.load(open('gpurun_out/tab_$i.json'));print(d['value'], d['ms_per_step'], d['roofline']['step_gpu_ms'])")
done
