#!/bin/bash
# same-box A/B of runtime environment settings: bash tools/gpu/ab_env.sh "<env A>" "<env B>" ...
# (each an env assignment list such as "DEBUG_HIP_FORCE_GRAPH_QUEUES=6", "" = unchanged); every
# set runs twice, interleaved; extra bench flags in BENCH_ARGS
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
i=0
for rep in 1 2; do
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --no-dp-line ${BENCH_ARGS:-} > gpurun_out/abe_$i.json 2> gpurun_out/abe.err || { echo BENCHFAIL; tail -20 gpurun_out/abe.err; exit 1; }
    echo "[$e]" $(python -c "import json;d=json.load(open('gpurun_out/abe_$i.json'));print(d['value'], d['ms_per_step'])")
  done
done
