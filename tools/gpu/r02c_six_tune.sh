#!/bin/bash
# record the tile choices of the 6-block step (224 and 384) for the committed table
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --blocks 6 --no-cpu-baseline --no-kernel-rooflines --tune-save gpurun_out/tune_six224.json \
  > gpurun_out/r02c_six224b.json 2> gpurun_out/r02c_six224b.err || { echo BENCHFAIL; tail -20 gpurun_out/r02c_six224b.err; exit 1; }
cut -c1-300 gpurun_out/r02c_six224b.json
timeout -k 10 300 python bench.py --blocks 6 --image-size 384 --no-cpu-baseline --no-kernel-rooflines \
  --tune-save gpurun_out/tune_six384.json > gpurun_out/r02c_six384b.json 2> gpurun_out/r02c_six384b.err || { echo BENCHFAIL; tail -20 gpurun_out/r02c_six384b.err; exit 1; }
cut -c1-300 gpurun_out/r02c_six384b.json
