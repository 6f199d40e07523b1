# r06: single-pass epilogue (whole tile image at once) vs one pass per wave row
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=t5-resnet-vqa_amd/lib/libvqa_hip.so
cp gpurun_ab/lib_r06_one.so $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py  > gpurun_out/t9.log 2>&1; rc=$?; tail -2 gpurun_out/t9.log; [ $rc -eq 0 ] || exit $rc
for lib in gpurun_ab/lib_r06_epi_keep.so gpurun_ab/lib_r06_one.so; do
  cp $lib $L
  timeout -k 10 300 python tools/lib_bitwise.py > gpurun_out/bits.json 2> gpurun_out/bits.err || { echo BITSFAIL; tail -5 gpurun_out/bits.err; exit 1; }
  echo "[$lib]" $(cat gpurun_out/bits.json)
done
bash tools/gpu/ab_lib.sh gpurun_ab/lib_r06_epi_keep.so gpurun_ab/lib_r06_one.so 3
