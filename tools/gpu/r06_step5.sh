# r06: persistent-grid ResNet launches (VQA_RES_GRID): bitwise tests, then the step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "persistent" > gpurun_out/t5.log 2>&1; rc=$?; tail -3 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab_env.sh "X=0" "VQA_RES_GRID=512" "VQA_RES_GRID=256" "VQA_RES_GRID=128" "VQA_RES_GRID=64"
