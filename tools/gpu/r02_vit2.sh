#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_vit_gpu.py tests/test_parity_gpu.py tests/test_api_gpu.py tests/test_dp_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02_vit2.log 2>&1
rc=$?; tail -2 gpurun_out/r02_vit2.log; grep -E "^E |FAILED" gpurun_out/r02_vit2.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --model vit --no-cpu-baseline > gpurun_out/r02_vitbench2.json 2> gpurun_out/r02_vitbench2.err || { echo VBFAIL; tail -20 gpurun_out/r02_vitbench2.err; exit 1; }
cut -c1-400 gpurun_out/r02_vitbench2.json
