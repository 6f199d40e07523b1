set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tg.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/tg.log; exit 1; }
tail -2 gpurun_out/tg.log
timeout -k 10 600 python bench.py --tune-table /nonexistent --tune-save $GRAFT_REPO_ROOT/gpurun_out/tune.json --no-cpu-baseline > gpurun_out/b_tune.json 2> gpurun_out/b_tune.err || { echo BENCHFAIL; tail -20 gpurun_out/b_tune.err; exit 1; }
cat gpurun_out/b_tune.json
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof9 -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --tune-table $R/gpurun_out/tune.json > $R/gpurun_out/p9.log 2>&1 || { echo PROFFAIL; tail -20 $R/gpurun_out/p9.log; exit 1; }
echo done
