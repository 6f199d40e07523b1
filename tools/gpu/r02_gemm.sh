#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_api_gpu.py tests/test_input_pipeline_gpu.py -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r02_gemmtest.log 2>&1 || { echo GEMMTESTFAIL; grep -E "FAIL|Error|error" gpurun_out/r02_gemmtest.log | head -20; tail -5 gpurun_out/r02_gemmtest.log; exit 1; }
tail -2 gpurun_out/r02_gemmtest.log
timeout -k 10 300 python tools/gemm_lab.py > gpurun_out/gemm_lab2.log 2>&1 || { echo LABFAIL; tail gpurun_out/gemm_lab2.log; exit 1; }
cat gpurun_out/gemm_lab2.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-kernel-rooflines --tune-table none --tune-save gpurun_out/tune_new.json > gpurun_out/b_tune.json 2> gpurun_out/b_tune.err || { echo BENCHFAIL; tail gpurun_out/b_tune.err; exit 1; }
cat gpurun_out/b_tune.json | python -c "import json,sys;d=json.load(sys.stdin);print('fresh-tuned', d['value'], d['ms_per_step'])"
for t in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --tune-table gpurun_out/tune_new.json > gpurun_out/b_new.json 2> gpurun_out/b_new.err || { echo BENCHFAIL; tail gpurun_out/b_new.err; exit 1; }
cat gpurun_out/b_new.json | python -c "import json,sys;d=json.load(sys.stdin);print('new table', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines > gpurun_out/b_old.json 2> gpurun_out/b_old.err || { echo BENCHFAIL; tail gpurun_out/b_old.err; exit 1; }
cat gpurun_out/b_old.json | python -c "import json,sys;d=json.load(sys.stdin);print('old table', d['value'], d['ms_per_step'])"
done
