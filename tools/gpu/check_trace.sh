set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-x}
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/t_$TAG.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -3 gpurun_out/t_$TAG.log
timeout -k 10 300 python bench.py --no-cpu-baseline --tune-save gpurun_out/gemm_gfx950_$TAG.json > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo BENCHFAIL; tail -20 gpurun_out/b_$TAG.err; exit 1; }
cat gpurun_out/b_$TAG.json
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --tune-table $R/gpurun_out/gemm_gfx950_$TAG.json > $R/gpurun_out/p_$TAG.log 2>&1 || { echo PROFFAIL; tail -20 $R/gpurun_out/p_$TAG.log; exit 1; }
cd $R && python tools/tracegaps.py gpurun_out/prof_$TAG/run_kernel_trace.csv rng_advance
