set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for cfg in "VQA_DW_STREAM=0 VQA_T5_DW_GROUP=12" "VQA_DW_STREAM=1 VQA_T5_DW_GROUP=6" "VQA_DW_STREAM=1 VQA_T5_DW_GROUP=4" "VQA_DW_STREAM=1 VQA_T5_DW_GROUP=12" "VQA_DW_STREAM=0 VQA_T5_DW_GROUP=12" "VQA_DW_STREAM=1 VQA_T5_DW_GROUP=6"; do
  env $cfg timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/dws.json 2> gpurun_out/dws.err || { echo BENCHFAIL; tail -20 gpurun_out/dws.err; exit 1; }
  echo "$cfg" $(python -c "import json;d=json.load(open('gpurun_out/dws.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])")
done
