set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/ -m gpu -q -x > gpurun_out/tsg.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/tsg.log; exit 1; }
tail -1 gpurun_out/tsg.log
for v in 1 0 1 0; do
  VQA_SGA_DW_BATCH=$v timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/sg_$v.json 2> gpurun_out/sg.err || { echo BENCHFAIL; tail -20 gpurun_out/sg.err; exit 1; }
  echo "sga_batch=$v" $(python -c "import json;d=json.load(open('gpurun_out/sg_$v.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'], d['sga_mfma']['frac'])")
done
