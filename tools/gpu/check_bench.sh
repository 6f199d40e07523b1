set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/t10.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t10.log; exit 1; }
tail -3 gpurun_out/t10.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b10.json 2> gpurun_out/b10.err || { echo BENCHFAIL; tail -20 gpurun_out/b10.err; exit 1; }
cat gpurun_out/b10.json
timeout -k 10 400 python tools/callprof.py 64 --autotune > gpurun_out/callprof10.log 2>&1 || { echo CPFAIL; tail -30 gpurun_out/callprof10.log; exit 1; }
tail -28 gpurun_out/callprof10.log
