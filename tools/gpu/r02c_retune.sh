#!/bin/bash
# re-time every GEMM choice of the benched step (no table), merge into the committed table,
# then an interleaved A/B of the committed vs the merged table
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=t5-resnet-vqa_amd/tuning/gemm_gfx950.json
timeout -k 10 400 python bench.py --tune-table /nonexistent.json --tune-save gpurun_out/tune_new.json --no-cpu-baseline --no-kernel-rooflines > gpurun_out/retune.json 2> gpurun_out/retune.err || { echo RETUNEFAIL; tail -20 gpurun_out/retune.err; exit 1; }
python - <<'PY'
import json
old = json.load(open("t5-resnet-vqa_amd/tuning/gemm_gfx950.json"))
new = json.load(open("gpurun_out/tune_new.json"))
ch = {k: (old.get(k), v) for k, v in new.items() if old.get(k) != v}
print("changed", len(ch), "of", len(new))
old.update(new)
json.dump(dict(sorted(old.items())), open("gpurun_out/tune_merged.json", "w"), indent=0)
PY
for round in 1 2; do
  for tab in $T gpurun_out/tune_merged.json; do
    timeout -k 10 300 python bench.py --tune-table $tab --no-cpu-baseline --no-kernel-rooflines > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo BENCHFAIL; tail -20 gpurun_out/ab.err; exit 1; }
    echo "[$tab] $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
  done
done
