set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "attention" > gpurun_out/ta.log 2>&1 || { echo TESTFAIL; tail -60 gpurun_out/ta.log; exit 1; }
tail -3 gpurun_out/ta.log
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/t_a.log 2>&1 || { echo TESTFAIL2; tail -40 gpurun_out/t_a.log; exit 1; }
tail -3 gpurun_out/t_a.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_a.json 2> gpurun_out/b_a.err || { echo BENCHFAIL; tail -20 gpurun_out/b_a.err; exit 1; }
cat gpurun_out/b_a.json
