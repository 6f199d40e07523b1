#!/bin/bash
# round 3: smoke, config-2 bench (kernel rooflines, no CPU baseline), config-5 bench, ResNet per-call times
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r03_bench.err; exit 1; }
cut -c1-400 gpurun_out/r03_bench.json
timeout -k 10 400 python bench.py --config5 --no-cpu-baseline --no-kernel-rooflines --steps 10 --warmup 3 --tune-save gpurun_out/tune_c5.json > gpurun_out/r03_bench_c5.json 2> gpurun_out/r03_bench_c5.err || { echo C5FAIL; tail -20 gpurun_out/r03_bench_c5.err; exit 1; }
cut -c1-600 gpurun_out/r03_bench_c5.json
timeout -k 10 200 python tools/res_micro.py 20 > gpurun_out/r03_res_micro.log 2>&1 || { echo RESFAIL; tail -20 gpurun_out/r03_res_micro.log; exit 1; }
tail -3 gpurun_out/r03_res_micro.log
