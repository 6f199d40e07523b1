#!/bin/bash
# full GPU suite, smoke, bench (default flags), and a kernel-trace profile of a short bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
rm -f gpurun_out/parity_report.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r02_gputest.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r02_gputest.log | tail -2
grep -E "FAILED|ERROR" gpurun_out/r02_gputest.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r02_smoke.log; exit 1; }
tail -1 gpurun_out/r02_smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --tune-save gpurun_out/tune_r02.json > /dev/null 2> gpurun_out/r02_tune.err || { echo TUNEFAIL; tail -20 gpurun_out/r02_tune.err; exit 1; }
timeout -k 10 300 python bench.py --tune-table gpurun_out/tune_r02.json > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r02_bench.err; exit 1; }
cat gpurun_out/r02_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r02_ktrace -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --tune-table $GRAFT_REPO_ROOT/gpurun_out/tune_r02.json > $GRAFT_REPO_ROOT/gpurun_out/r02_ktrace.log 2>&1 || { echo KTFAIL; tail -5 $GRAFT_REPO_ROOT/gpurun_out/r02_ktrace.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/r02_ktrace.log
