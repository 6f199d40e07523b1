#!/bin/bash
# BASELINE configs[2] code path rehearsed on one GPU: bench.py --gpus 8 --rehearse (8 ranks on cuda:0 over gloo,
# B=64 each, pipelined ResNet, DP T5 weight-gradient groups, captured segment graphs, 16384-token embedding gather)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
(while true; do date > gpurun_out/dp8.heartbeat; sleep 30; done) &
hb=$!
timeout -k 10 900 python bench.py --gpus ${NR:-8} --rehearse --steps 2 --warmup 1 > gpurun_out/dp8.json 2> gpurun_out/dp8.err
rc=$?
kill $hb
cat gpurun_out/dp8.json; grep -v amdgpu.ids gpurun_out/dp8.err | tail -20
exit $rc
