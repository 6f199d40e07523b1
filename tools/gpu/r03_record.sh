#!/bin/bash
# round 3 record (copied to profiles/ afterwards):
#   GPU suite -> parity report; smoke; config-2 bench with the CPU baseline; kernel-trace stats of
#   the config-2 and config-5 benches; PMC passes (stamped with this tree's digest and PMC_COMMIT);
#   bench.py --gpus 8 --rehearse.  SKIP_SUITE=1 skips the suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "${SKIP_SUITE:-}" ]; then
  rm -f gpurun_out/parity_report.json
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
     > gpurun_out/r03_gputest.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_gputest.log | tail -20; exit 1; }
  grep -E "passed|failed" gpurun_out/r03_gputest.log | tail -1
fi
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r03_smoke.log; exit 1; }
tail -1 gpurun_out/r03_smoke.log
rm -rf gpurun_out/r03_stats gpurun_out/r03_stats_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r03_stats -o run -- python3 bench.py --no-cpu-baseline \
   > gpurun_out/r03_stats_bench.json 2> gpurun_out/r03_stats_bench.err || { echo STATSFAIL; tail -20 gpurun_out/r03_stats_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/r03_stats_c5 -o run -- python3 bench.py --config5 --no-cpu-baseline \
   > gpurun_out/r03_stats_c5.json 2> gpurun_out/r03_stats_c5.err || { echo STATSC5FAIL; tail -20 gpurun_out/r03_stats_c5.err; exit 1; }
cd /tmp
run() {  # tag counters... -- cmd   (each counter group in a run of its own)
  local tag=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
  rm -rf $R/gpurun_out/pmc_$tag
  timeout -k 10 240 rocprofv3 --pmc "${ctrs[@]}" -f csv -d $R/gpurun_out/pmc_$tag -o $tag -- "$@" > $R/gpurun_out/pmc_$tag.log 2>&1 \
    || { echo "PMCFAIL $tag"; tail -20 $R/gpurun_out/pmc_$tag.log; exit 1; }
  echo "pass $tag ok"
}
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-rooflines"
K="python3 $R/tools/kernel_replay.py $R/gpurun_out/replay_manifest.json 5"
run sF FETCH_SIZE -- $B
run sW WRITE_SIZE -- $B
run sM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B
run rF FETCH_SIZE -- $K
run rW WRITE_SIZE -- $K
run rM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- $K
cd $R && python3 tools/pmc_step.py gpurun_out/r03_pmc.json gpurun_out/pmc_sF gpurun_out/pmc_sW gpurun_out/pmc_sM \
   gpurun_out/pmc_rF gpurun_out/pmc_rW gpurun_out/pmc_rM gpurun_out/replay_manifest.json > gpurun_out/r03_pmc.log 2>&1 \
   || { echo SUMFAIL; tail -30 gpurun_out/r03_pmc.log; exit 1; }
echo pmc summary written
# the committed bench with the CPU baseline, quoting the PMC file just written (same tree)
mkdir -p profiles && cp gpurun_out/r03_pmc.json profiles/r03_pmc.json
timeout -k 10 400 python bench.py > gpurun_out/r03_bench_final.json 2> gpurun_out/r03_bench_final.err || { echo BENCHFAIL; tail -20 gpurun_out/r03_bench_final.err; exit 1; }
cut -c1-400 gpurun_out/r03_bench_final.json
if [ -z "${SKIP_DP8:-}" ]; then
  (while true; do date > gpurun_out/dp8.heartbeat; sleep 30; done) &
  hb=$!
  timeout -k 10 900 python bench.py --gpus 8 --rehearse --steps 2 --warmup 1 > gpurun_out/r03_dp8.json 2> gpurun_out/r03_dp8.err
  rc=$?
  kill $hb
  cut -c1-300 gpurun_out/r03_dp8.json; grep -v amdgpu.ids gpurun_out/r03_dp8.err | tail -5
  exit $rc
fi
