# r06: GEMM configs 26-28 (one k-tile, single-stage ring) -- tests, re-time the K <= 64 ResNet shapes,
# bitwise fingerprint, same-box A/B of (old lib, committed table) vs (new lib, table with the re-timed shapes)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=t5-resnet-vqa_amd/lib/libvqa_hip.so; T=t5-resnet-vqa_amd/tuning/gemm_gfx950.json
cp $T gpurun_out/tune_committed.json
cp gpurun_ab/lib_r06_k64.so $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py -m gpu > gpurun_out/s13_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/s13_tests.log; exit 1; }
tail -1 gpurun_out/s13_tests.log
timeout -k 10 300 python bench.py --tune-table gpurun_ab/tune_k64_base.json --tune-save gpurun_out/tune_c2_k64.json --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/s13_tc2.json 2> gpurun_out/s13_tc2.err || { echo TUNEFAIL; tail -5 gpurun_out/s13_tc2.err; exit 1; }
grep autotune gpurun_out/s13_tc2.err | cut -c1-200
timeout -k 10 300 python bench.py --config5 --tune-table gpurun_ab/tune_k64_base.json --tune-save gpurun_out/tune_c5_k64.json --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/s13_tc5.json 2> gpurun_out/s13_tc5.err || { echo TUNE5FAIL; tail -5 gpurun_out/s13_tc5.err; exit 1; }
python - <<'PY'
import json
t = json.load(open("gpurun_out/tune_committed.json"))
keys = json.load(open("gpurun_ab/tune_k64_keys.json"))
new = {}
for f in ("gpurun_out/tune_c2_k64.json", "gpurun_out/tune_c5_k64.json"):
    new.update(json.load(open(f)))
for k in keys:
    print(k, t[k], "->", new[k])
    t[k] = new[k]
json.dump(dict(sorted(t.items())), open("gpurun_out/tune_merged.json", "w"), indent=0)
PY
for pair in "gpurun_ab/lib_r06_epi_keep.so gpurun_out/tune_committed.json" "gpurun_ab/lib_r06_k64.so gpurun_out/tune_merged.json"; do
  set -- $pair; cp $1 $L; cp $2 $T
  timeout -k 10 300 python tools/lib_bitwise.py > gpurun_out/s13_bw.txt 2>&1 || { echo BWFAIL; tail -10 gpurun_out/s13_bw.txt; exit 1; }
  echo "[$1]" $(tail -1 gpurun_out/s13_bw.txt)
done
i=0
for rep in 1 2 3; do
  for pair in "gpurun_ab/lib_r06_epi_keep.so gpurun_out/tune_committed.json" "gpurun_ab/lib_r06_k64.so gpurun_out/tune_merged.json"; do
    set -- $pair; cp $1 $L; cp $2 $T; i=$((i+1))
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/s13_ab_$i.json 2> gpurun_out/s13_ab.err || { echo BENCHFAIL; tail -20 gpurun_out/s13_ab.err; exit 1; }
    echo "[$1]" $(python -c "import json;d=json.load(open('gpurun_out/s13_ab_$i.json'));print(d['value'], d['ms_per_step'])")
  done
done
for pair in "gpurun_ab/lib_r06_epi_keep.so gpurun_out/tune_committed.json" "gpurun_ab/lib_r06_k64.so gpurun_out/tune_merged.json"; do
  set -- $pair; cp $1 $L; cp $2 $T
  timeout -k 10 300 python bench.py --config5 --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/s13_c5.json 2> gpurun_out/s13_ab.err || { echo C5FAIL; tail -20 gpurun_out/s13_ab.err; exit 1; }
  echo "c5 [$1]" $(python -c "import json;d=json.load(open('gpurun_out/s13_c5.json'));print(d['value'], d['ms_per_step'])")
done
cp gpurun_out/tune_committed.json $T
