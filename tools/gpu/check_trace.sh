set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/t11.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t11.log; exit 1; }
tail -3 gpurun_out/t11.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b11.json 2> gpurun_out/b11.err || { echo BENCHFAIL; tail -20 gpurun_out/b11.err; exit 1; }
cat gpurun_out/b11.json
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof11 -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/p11.log 2>&1 || { echo PROFFAIL; tail -20 $R/gpurun_out/p11.log; exit 1; }
cd $R && python tools/tracegaps.py gpurun_out/prof11/run_kernel_trace.csv rng_advance
