# r06: epilogue operand prefetch: the GEMM kernel tests, the step's bits under both builds, then the A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=t5-resnet-vqa_amd/lib/libvqa_hip.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_gpu.py > gpurun_out/t8.log 2>&1; rc=$?; tail -2 gpurun_out/t8.log; [ $rc -eq 0 ] || exit $rc
for lib in gpurun_ab/lib_r06_base.so gpurun_ab/lib_r06_epi.so; do
  cp $lib $L
  timeout -k 10 300 python tools/lib_bitwise.py > gpurun_out/bits.json 2> gpurun_out/bits.err || { echo BITSFAIL; tail -5 gpurun_out/bits.err; exit 1; }
  echo "[$lib]" $(cat gpurun_out/bits.json)
done
bash tools/gpu/ab_lib.sh gpurun_ab/lib_r06_base.so gpurun_ab/lib_r06_epi.so 2
