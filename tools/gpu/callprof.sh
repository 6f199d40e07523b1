set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "embedding" > gpurun_out/t9.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t9.log; exit 1; }
tail -2 gpurun_out/t9.log
timeout -k 10 500 python tools/callprof.py 64 --configs > gpurun_out/callprof.log 2>&1 || { echo CPFAIL; tail -30 gpurun_out/callprof.log; exit 1; }
tail -40 gpurun_out/callprof.log
