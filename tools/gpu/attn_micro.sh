set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "attention or attn" > gpurun_out/ta.log 2>&1 || { echo TESTFAIL; tail -60 gpurun_out/ta.log; exit 1; }
tail -3 gpurun_out/ta.log
timeout -k 10 120 ./tools/micro/attn_micro > gpurun_out/am.log 2>&1 || { echo MICROFAIL; tail -20 gpurun_out/am.log; exit 1; }
cat gpurun_out/am.log
