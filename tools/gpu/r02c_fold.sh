#!/bin/bash
# GPU suite, then same-box A/B of the folded RMSNorm (VQA_NORM_FOLD) with the tile choices saved
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
rm -f gpurun_out/parity_report.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r02c_gputest.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r02c_gputest.log | tail -1
grep -E "FAILED|ERROR" gpurun_out/r02c_gputest.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --tune-save gpurun_out/tune_fold.json > gpurun_out/fold.json 2> gpurun_out/fold.err || { echo BENCHFAIL; tail -20 gpurun_out/fold.err; exit 1; }
python - <<'PY'
import json
old = json.load(open("t5-resnet-vqa_amd/tuning/gemm_gfx950.json"))
new = json.load(open("gpurun_out/tune_fold.json"))
old.update(new)
json.dump(dict(sorted(old.items())), open("gpurun_out/tune_merged.json", "w"), indent=0)
PY
for round in 1 2; do
  for v in 0 1; do
    VQA_NORM_FOLD=$v timeout -k 10 300 python bench.py --tune-table gpurun_out/tune_merged.json --no-cpu-baseline --no-kernel-rooflines > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo BENCHFAIL; tail -20 gpurun_out/ab.err; exit 1; }
    echo "[VQA_NORM_FOLD=$v] $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'], d['loss'], d['grad_norm'])")"
  done
done
