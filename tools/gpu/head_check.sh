set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "head" > gpurun_out/th.log 2>&1 || { echo TESTFAIL; tail -60 gpurun_out/th.log; exit 1; }
tail -2 gpurun_out/th.log
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/t_h.log 2>&1 || { echo TESTFAIL2; tail -40 gpurun_out/t_h.log; exit 1; }
tail -2 gpurun_out/t_h.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/profh -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/ph.log 2>&1 || { echo PROFFAIL; tail -20 $R/gpurun_out/ph.log; exit 1; }
cut -c1-200 $R/gpurun_out/ph.log | grep metric
