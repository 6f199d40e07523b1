#!/bin/bash
# r04 baseline: GEMM tests touched by the rownorm removal, bench, SGA launch table
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_base_test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r04_base_test.log; exit 1; }
tail -2 gpurun_out/r04_base_test.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines > gpurun_out/r04_base_bench.json 2> gpurun_out/r04_base_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r04_base_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r04_base_bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python tools/sga_launches.py 20 > gpurun_out/r04_sga_launches.txt 2>&1 || { echo SGAFAIL; tail -20 gpurun_out/r04_sga_launches.txt; exit 1; }
cat gpurun_out/r04_sga_launches.txt
