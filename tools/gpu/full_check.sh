set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/t8.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t8.log; exit 1; }
tail -3 gpurun_out/t8.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s8.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/s8.log; exit 1; }
cat gpurun_out/s8.log
timeout -k 10 300 python bench.py > gpurun_out/b8.json 2> gpurun_out/b8.err || { echo BENCHFAIL; tail -20 gpurun_out/b8.err; exit 1; }
cat gpurun_out/b8.json
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof8 -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/p8.log 2>&1 || { echo PROFFAIL; tail -20 $R/gpurun_out/p8.log; exit 1; }
echo done
