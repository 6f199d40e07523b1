# r06: DP with the collectives on the comm stream: world-1 RCCL tests, the queue trace, the bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_dp_gpu.py tests/test_z_dp_bench_step_gpu.py > gpurun_out/t_dp.log 2>&1; rc=$?; tail -3 gpurun_out/t_dp.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/dpq
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/dpq -o run -- python tools/dp_queue_probe.py 6 > gpurun_out/dpq.log 2>&1 || { echo PROBEFAIL; tail -5 gpurun_out/dpq.log; }
grep markers gpurun_out/dpq.log || true
db=$(find gpurun_out/dpq -name "*.db" | head -1)
[ -n "$db" ] && python tools/dp_queue_probe.py --analyse $db
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines > gpurun_out/b_dp.json 2> gpurun_out/b_dp.err || { echo BENCHFAIL; tail -20 gpurun_out/b_dp.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/b_dp.json'));print(d['value'], d['ms_per_step'], d.get('host_issue_ms_per_step'), d.get('dp_world1'))"
