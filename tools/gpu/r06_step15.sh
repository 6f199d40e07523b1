# r06: GEMM config 29 (64x64, one 128-deep k-tile, single-stage ring) -- tests, re-time the K <= 128
# ResNet shapes, bitwise fingerprint, same-box A/B of the committed table vs the re-timed one (same library)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=t5-resnet-vqa_amd/lib/libvqa_hip.so; T=t5-resnet-vqa_amd/tuning/gemm_gfx950.json
cp $T gpurun_out/tune_committed.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -m gpu > gpurun_out/s15_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/s15_tests.log; exit 1; }
tail -1 gpurun_out/s15_tests.log
timeout -k 10 300 python bench.py --tune-table gpurun_ab/tune_k128_base.json --tune-save gpurun_out/tune_c2_k128.json --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/s15_tc2.json 2> gpurun_out/s15_tc2.err || { echo TUNEFAIL; tail -5 gpurun_out/s15_tc2.err; exit 1; }
timeout -k 10 300 python bench.py --config5 --tune-table gpurun_ab/tune_k128_base.json --tune-save gpurun_out/tune_c5_k128.json --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/s15_tc5.json 2> gpurun_out/s15_tc5.err || { echo TUNE5FAIL; tail -5 gpurun_out/s15_tc5.err; exit 1; }
python - <<'PY'
import json
t = json.load(open("gpurun_out/tune_committed.json"))
new = {}
for f in ("gpurun_out/tune_c2_k128.json", "gpurun_out/tune_c5_k128.json"):
    new.update(json.load(open(f)))
for k in json.load(open("gpurun_ab/tune_k128_keys.json")):
    if k in new:
        print(k[:40], t[k], "->", new[k])
        t[k] = new[k]
json.dump(t, open("gpurun_out/tune_k128_merged.json", "w"), indent=0)
PY
A="gpurun_out/tune_committed.json"
B="gpurun_out/tune_k128_merged.json"
for tb in $A $B; do
  cp $tb $T
  timeout -k 10 300 python tools/lib_bitwise.py > gpurun_out/s15_bw.txt 2>&1 || { echo BWFAIL; tail -10 gpurun_out/s15_bw.txt; exit 1; }
  echo "[$tb]" $(tail -1 gpurun_out/s15_bw.txt)
done
n=0
for tb in $A $B; do
  cp $tb $T; n=$((n+1))
  timeout -k 10 300 python tools/res_micro.py > gpurun_out/s15_res_$n.txt 2>&1 || { echo MICROFAIL; tail -5 gpurun_out/s15_res_$n.txt; exit 1; }
  echo "res [$tb]" $(tail -1 gpurun_out/s15_res_$n.txt)
done
i=0
for rep in 1 2 3 4; do
  for tb in $A $B; do
    cp $tb $T; i=$((i+1))
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --no-dp-line > gpurun_out/s15_ab_$i.json 2> gpurun_out/s15_ab.err || { echo BENCHFAIL; tail -20 gpurun_out/s15_ab.err; exit 1; }
    echo "[$tb]" $(python -c "import json;d=json.load(open('gpurun_out/s15_ab_$i.json'));print(d['value'], d['ms_per_step'])")
  done
done
cp $A $T
