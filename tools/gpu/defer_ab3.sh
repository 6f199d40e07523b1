set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in "VQA_DEFER_OPT=0" "VQA_OPT_STREAM=0" "VQA_OPT_STREAM=1" "VQA_DEFER_OPT=0" "VQA_OPT_STREAM=0" "VQA_OPT_STREAM=1"; do
  env $cfg timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/ab3.json 2> gpurun_out/ab3.err || { echo BENCHFAIL; tail -20 gpurun_out/ab3.err; exit 1; }
  echo "$cfg" $(python -c "import json;d=json.load(open('gpurun_out/ab3.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])")
done
