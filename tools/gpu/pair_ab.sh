set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in 1 0 1 0; do
  VQA_PAIR_BWD=$v timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/pab_$v.json 2> gpurun_out/pab.err || { echo BENCHFAIL; tail -20 gpurun_out/pab.err; exit 1; }
  echo "pair=$v" $(python -c "import json;d=json.load(open('gpurun_out/pab_$v.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])")
done
