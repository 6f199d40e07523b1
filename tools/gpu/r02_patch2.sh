#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider -k "patch" > gpurun_out/r02_patch2.log 2>&1
rc=$?; tail -2 gpurun_out/r02_patch2.log; grep -E "^E |FAILED" gpurun_out/r02_patch2.log | head -12
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/r02_patchprof.sh 2>&1 | grep -E "k= 576|k= 1152|k= 2304|k= 4608" | head -20
bash tools/gpu/ab_env.sh "-" "VQA_CONV_PATCH=0"
