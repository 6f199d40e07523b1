# re-time every GEMM shape of the benched step (no table: every config x split-K candidate),
# save the choices, then interleaved A/B of the committed table against the new one
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu-baseline --no-kernel-rooflines --no-dp-line --tune-table /nonexistent \
  --tune-save gpurun_out/tune_new.json > gpurun_out/retune_bench.json 2> gpurun_out/retune.err || { echo RETUNEFAIL; tail -20 gpurun_out/retune.err; exit 1; }
echo "[retune run]" $(python -c "import json;d=json.load(open('gpurun_out/retune_bench.json'));print(d['value'], d['ms_per_step'])")
bash tools/gpu/ab.sh "" "--tune-table gpurun_out/tune_new.json"
