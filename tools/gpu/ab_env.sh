#!/bin/bash
# interleaved same-box A/B of bench.py under environment variants: ab_env.sh "ENV1" "ENV2" ...
# (each variant a space-separated list of VAR=value; "-" = no change); 2 rounds
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    envs=(); [ "$v" != "-" ] && read -ra envs <<< "$v"
    env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines > gpurun_out/ab.json 2> gpurun_out/ab.err \
      || { echo "BENCHFAIL [$v]"; tail -20 gpurun_out/ab.err; exit 1; }
    echo "[$v] $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['roofline']['step_gpu_ms'])")"
  done
done
