#!/bin/bash
# end-of-session record: GPU suite, smoke, default bench (CPU baseline included), kernel-trace
# stats of the same bench command, PMC passes (tools/gpu/r02_pmc.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
rm -f gpurun_out/parity_report.json
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider \
   > gpurun_out/r02c_gputest.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r02c_gputest.log | tail -1
grep -E "FAILED|ERROR" gpurun_out/r02c_gputest.log | head -20
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02c_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r02c_smoke.log; exit 1; }
tail -1 gpurun_out/r02c_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r02c_bench.json 2> gpurun_out/r02c_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/r02c_bench.err; exit 1; }
cat gpurun_out/r02c_bench.json
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/r02c_ktrace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/r02c_ktrace -o kt -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/r02c_ktrace.log 2>&1 || { echo KTFAIL; tail -5 $R/gpurun_out/r02c_ktrace.log; exit 1; }
tail -1 $R/gpurun_out/r02c_ktrace.log | cut -c1-200
cd $R && bash tools/gpu/r02_pmc.sh > gpurun_out/r02c_pmc.out 2>&1 || { echo PMCFAIL; tail -20 gpurun_out/r02c_pmc.out; exit 1; }
grep -E "pass|FAIL" gpurun_out/r02c_pmc.out
