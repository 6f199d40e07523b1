# same-box A/B of bench flag sets: bash tools/gpu/ab.sh "<flags A>" "<flags B>" ["<flags C>" ...]
# every set is run twice, the sets interleaved (A B C A B C)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
i=0
for rep in 1 2; do
  for f in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --no-dp-line $f > gpurun_out/ab_$i.json 2> gpurun_out/ab.err || { echo BENCHFAIL; tail -20 gpurun_out/ab.err; exit 1; }
    echo "[$f]" $(python -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));print(d['value'], d['ms_per_step'])")
  done
done
