#!/bin/bash
# config 2 (x2) and config 4 benches with the committed table
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines > gpurun_out/tabc_$i.json 2> gpurun_out/tabc.err || { echo BENCHFAIL; tail -20 gpurun_out/tabc.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/tabc_$i.json'));print('config2', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --model vit --no-cpu-baseline > gpurun_out/tabc_vit.json 2> gpurun_out/tabc_vit.err || { echo BENCHFAIL; tail -20 gpurun_out/tabc_vit.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/tabc_vit.json'));print('vit', d['value'], d['ms_per_step'])"
