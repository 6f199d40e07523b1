#!/bin/bash
# interleaved A/B of bench --model vit under environment variants
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for round in 1 2; do
  for v in "$@"; do
    envs=(); [ "$v" != "-" ] && read -ra envs <<< "$v"
    env "${envs[@]}" timeout -k 10 300 python bench.py --model vit --no-cpu-baseline > gpurun_out/abv.json 2> gpurun_out/abv.err \
      || { echo "BENCHFAIL [$v]"; tail -20 gpurun_out/abv.err; exit 1; }
    echo "[$v] $(python -c "import json;d=json.load(open('gpurun_out/abv.json'));print(d['value'], d['ms_per_step'])")"
  done
done
