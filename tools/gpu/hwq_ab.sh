set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for q in 4 6 4 6; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/hwq.json 2> gpurun_out/hwq.err || { echo BENCHFAIL; tail -20 gpurun_out/hwq.err; exit 1; }
  echo "queues=$q" $(python -c "import json;d=json.load(open('gpurun_out/hwq.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])")
done
