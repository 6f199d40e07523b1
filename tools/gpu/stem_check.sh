set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -q -x > gpurun_out/ts.log 2>&1 || { echo TESTFAIL; tail -60 gpurun_out/ts.log; exit 1; }
tail -2 gpurun_out/ts.log
timeout -k 10 300 python tools/res_micro.py > gpurun_out/resm.log 2>&1 || { echo MICROFAIL; tail -20 gpurun_out/resm.log; exit 1; }
head -8 gpurun_out/resm.log; tail -1 gpurun_out/resm.log
