# same-box A/B of an engine environment switch: VAR=NAME bash tools/gpu/env_ab.sh "1 0 1 0"
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in $1; do
  env $VAR=$v timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/env_$v.json 2> gpurun_out/env.err || { echo BENCHFAIL; tail -20 gpurun_out/env.err; exit 1; }
  echo "$VAR=$v" $(python -c "import json;d=json.load(open('gpurun_out/env_$v.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_us'])")
done
