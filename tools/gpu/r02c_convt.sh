#!/bin/bash
# GEMM tests (ConvTranspose2d dW among them), the default bench, then the PMC passes of r02_pmc.sh
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02c_gemmtest.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r02c_gemmtest.log; exit 1; }
tail -1 gpurun_out/r02c_gemmtest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r02c_bench.json 2> gpurun_out/r02c_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r02c_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r02c_bench.json'));print(d['value'], d['ms_per_step'], d['roofline_gemm'])"
bash tools/gpu/r02_pmc.sh
