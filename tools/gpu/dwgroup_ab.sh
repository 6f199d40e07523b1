# same-box A/B of the T5 weight-gradient group size (VQA_T5_DW_GROUP), after the GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/tdw.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/tdw.log; exit 1; }
tail -1 gpurun_out/tdw.log
for v in ${GROUPS_AB:-4 1 12 4 1 12}; do
  VQA_T5_DW_GROUP=$v timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/dwg_$v.json 2> gpurun_out/dwg.err || { echo BENCHFAIL; tail -20 gpurun_out/dwg.err; exit 1; }
  echo "group=$v" $(python -c "import json;d=json.load(open('gpurun_out/dwg_$v.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])")
done
