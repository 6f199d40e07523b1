#!/bin/bash
# the benched step at 384x384 images (R50 + T5-base + 3xSGA, B = 64; SGA block 0 over 144 keys)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --image-size 384 --no-cpu-baseline --no-kernel-rooflines --tune-save gpurun_out/tune_384.json > gpurun_out/b384.json 2> gpurun_out/b384.err || { echo BENCHFAIL; tail -20 gpurun_out/b384.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b384.json'));print(d['value'], d['ms_per_step'], d['config'], d['roofline']['frac'])"
