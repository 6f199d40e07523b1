# r06: DP comm-stream placement A/B: queue traces and bench lines per VQA_DP_COMM
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
for c in own wside side; do
  rm -rf gpurun_out/dpq_$c
  VQA_DP_COMM=$c timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/dpq_$c -o run -- python tools/dp_queue_probe.py 2 > gpurun_out/dpq_$c.log 2>&1 || { echo PROBEFAIL $c; tail -5 gpurun_out/dpq_$c.log; exit 1; }
  db=$(find gpurun_out/dpq_$c -name "*.db" | head -1)
  python tools/dp_queue_probe.py --analyse $db 8 > gpurun_out/dpq_$c.json
  echo "[$c]" $(python -c "import json;d=json.load(open('gpurun_out/dpq_$c.json'));print(d['graph_kernels_per_queue'], d['eager_kernels (name, queue, stream)'][:3], d['comm_queue_carries_graph_kernels'])")
done
for rep in 1 2; do for c in own wside side; do
  VQA_DP_COMM=$c timeout -k 10 300 python bench.py --dp --no-cpu-baseline --no-kernel-rooflines > gpurun_out/bdp_$c.json 2> gpurun_out/bdp.err || { echo BENCHFAIL; tail -20 gpurun_out/bdp.err; exit 1; }
  echo "[$c]" $(python -c "import json;d=json.load(open('gpurun_out/bdp_$c.json'));print(d['value'], d['ms_per_step'])")
done; done
