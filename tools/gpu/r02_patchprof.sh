#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for p in 1 0; do
VQA_CONV_PATCH=$p timeout -k 10 300 python tools/callprof.py 64 --autotune > gpurun_out/cp_patch$p.log 2>&1 || { echo CPFAIL; tail gpurun_out/cp_patch$p.log; exit 1; }
done
paste <(grep -E "^fwd +[0-9]+ " gpurun_out/cp_patch1.log | head -57 | awk "{print \$2, \$4, \$6, \$7, \$8, \$9, \$10, \$11, \$12}") <(grep -E "^fwd +[0-9]+ " gpurun_out/cp_patch0.log | head -57 | awk '{print $4}')
