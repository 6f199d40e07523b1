# r06: LDS-derived occupancy target on the GEMM kernels -- GEMM/kernel tests, bitwise fingerprint of both builds, same-box bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=t5-resnet-vqa_amd/lib/libvqa_hip.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/s12_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/s12_tests.log; exit 1; }
tail -2 gpurun_out/s12_tests.log
for lib in gpurun_ab/lib_r06_epi_keep.so gpurun_ab/lib_r06_occ.so; do
  cp $lib $L
  timeout -k 10 300 python tools/lib_bitwise.py > gpurun_out/s12_bw.txt 2>&1 || { echo BWFAIL; tail -10 gpurun_out/s12_bw.txt; exit 1; }
  echo "[$lib]" $(tail -1 gpurun_out/s12_bw.txt)
done
bash tools/gpu/ab_lib.sh gpurun_ab/lib_r06_epi_keep.so gpurun_ab/lib_r06_occ.so 3
cp gpurun_ab/lib_r06_occ.so $L
