# r06: DP with the opening id gather, the split embedding update and the early sq-norm partial:
# the DP GPU tests (world-1 RCCL bitwise vs the engine, gloo pairs vs the global batch), then the DP lines
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_dp_gpu.py tests/test_z_dp_bench_step_gpu.py > gpurun_out/t7.log 2>&1; rc=$?; tail -3 gpurun_out/t7.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines > gpurun_out/b7_$rep.json 2> gpurun_out/b7.err || { echo BENCHFAIL; tail -20 gpurun_out/b7.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b7_$rep.json'));w=d['dp_world1'];print(d['value'], d['ms_per_step'], '| dp_world1', w['value'], w['ms_per_step'], w['over_engine_step'])"
done
