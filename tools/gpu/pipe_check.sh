set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_parity_gpu.py -q -x -k "pipelined" > gpurun_out/tp.log 2>&1 || { echo TESTFAIL; tail -60 gpurun_out/tp.log; exit 1; }
tail -2 gpurun_out/tp.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bp1.json 2> gpurun_out/bp1.err || { echo BENCHFAIL; tail -20 gpurun_out/bp1.err; exit 1; }
cut -c1-200 gpurun_out/bp1.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pipeline > gpurun_out/bp0.json 2> gpurun_out/bp0.err || { echo BENCHFAIL0; tail -20 gpurun_out/bp0.err; exit 1; }
cut -c1-200 gpurun_out/bp0.json
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/profp -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/pp.log 2>&1 || { echo PROFFAIL; tail -20 $R/gpurun_out/pp.log; exit 1; }
echo done
