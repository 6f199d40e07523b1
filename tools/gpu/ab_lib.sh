#!/bin/bash
# same-box A/B of two builds of the library: bash tools/gpu/ab_lib.sh <lib A> <lib B> [reps]
# each rep copies A, then B, into t5-resnet-vqa_amd/lib/libvqa_hip.so and runs the bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
A=$1; B=$2; REPS=${3:-3}
L=t5-resnet-vqa_amd/lib/libvqa_hip.so
i=0
for rep in $(seq $REPS); do
  for lib in $A $B; do
    i=$((i+1))
    cp $lib $L
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/abl_$i.json 2> gpurun_out/abl.err || { echo BENCHFAIL; tail -20 gpurun_out/abl.err; exit 1; }
    echo "[$lib]" $(python -c "import json;d=json.load(open('gpurun_out/abl_$i.json'));print(d['value'], d['ms_per_step'])")
  done
done
cp $A $L
