#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_parity_gpu.py tests/test_parity_full_gpu.py tests/test_api_gpu.py -m gpu -q -x --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/r02_patch.log 2>&1
rc=$?; tail -3 gpurun_out/r02_patch.log; grep -E "^E |FAILED" gpurun_out/r02_patch.log | head -12
[ $rc -ne 0 ] && exit $rc
bash tools/gpu/ab_env.sh "-" "VQA_CONV_PATCH=0"
