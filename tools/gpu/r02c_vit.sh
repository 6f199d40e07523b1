#!/bin/bash
# config 4: bench with the committed table, then re-time every GEMM (no table) and bench with the merged table
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --model vit --no-cpu-baseline > gpurun_out/vit_a.json 2> gpurun_out/vit_a.err || { echo BENCHFAIL; tail -20 gpurun_out/vit_a.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/vit_a.json'));print('committed', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 400 python bench.py --model vit --no-cpu-baseline --tune-table /nonexistent.json --tune-save gpurun_out/tune_vit.json > gpurun_out/vit_b.json 2> gpurun_out/vit_b.err || { echo BENCHFAIL; tail -20 gpurun_out/vit_b.err; exit 1; }
python - <<'PY'
import json
old = json.load(open("t5-resnet-vqa_amd/tuning/gemm_gfx950.json"))
new = json.load(open("gpurun_out/tune_vit.json"))
print("vit shapes changed", sum(old.get(k) != v for k, v in new.items()), "of", len(new))
old.update(new)
json.dump(dict(sorted(old.items())), open("gpurun_out/tune_vit_merged.json", "w"), indent=0)
PY
for r in 1 2; do
  for t in t5-resnet-vqa_amd/tuning/gemm_gfx950.json gpurun_out/tune_vit_merged.json; do
    timeout -k 10 400 python bench.py --model vit --no-cpu-baseline --tune-table $t > gpurun_out/vit_c.json 2> gpurun_out/vit_c.err || { echo BENCHFAIL; tail -20 gpurun_out/vit_c.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/vit_c.json'));print('$t', d['value'], d['ms_per_step'])"
  done
done
