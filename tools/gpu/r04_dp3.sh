#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 bash tools/gpu/ab.sh "" "--dp" "--hw-queues 8" "--dp --hw-queues 8" > gpurun_out/r04_ab_dp3.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/r04_ab_dp3.log; exit 1; }
cat gpurun_out/r04_ab_dp3.log
timeout -k 10 400 python tools/vit_layer_diag.py gpurun_out/r04_vit_layer_diag2.json > gpurun_out/r04_vit_diag2.log 2>&1 || { echo DIAGFAIL; tail -20 gpurun_out/r04_vit_diag2.log; exit 1; }
tail -9 gpurun_out/r04_vit_diag2.log
