#!/bin/bash
# round 6 record, in stages that each fit one gpurun call (STAGE=suite|pmc|bench), copied to profiles/:
#   suite: GPU test suite -> parity report; smoke
#   pmc:   kernel-trace stats of the config-2 and config-5 benches; PMC passes of both steps and of
#          their replayed launches, stamped with this tree's digest and PMC_COMMIT
#   bench: config-2 bench with the CPU baseline (quoting the PMC file), config 5, config 4, --dp,
#          the collate bench, the SGA launch table, bench.py --gpus 8 --rehearse
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
case "${STAGE:-suite}" in
suite)
  rm -f gpurun_out/parity_report.json
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider \
     > gpurun_out/r06_gputest.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06_gputest.log | tail -20; exit 1; }
  grep -E "passed|failed" gpurun_out/r06_gputest.log | tail -1
  timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/r06_smoke.log; exit 1; }
  tail -1 gpurun_out/r06_smoke.log
  ;;
pmc)
  # WS="c2 c5" (default) or one of them per call
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
  for W in ${WS:-c2 c5}; do
    X=""; M=default; ST=r06_stats
    if [ $W = c5 ]; then X="--config5"; M=c5; ST=r06_stats_c5; fi
    rm -rf $R/gpurun_out/$ST
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/$ST -o run -- python3 $R/bench.py $X --no-cpu-baseline --no-dp-line \
       > $R/gpurun_out/${ST}_bench.json 2> $R/gpurun_out/${ST}_bench.err || { echo "STATSFAIL $W"; tail -20 $R/gpurun_out/${ST}_bench.err; exit 1; }
    echo "stats $W ok"
    B="python3 $R/bench.py $X --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-rooflines --no-dp-line"
    K="python3 $R/tools/kernel_replay.py $R/gpurun_out/replay_manifest_$W.json 5 $M"
    run ${W}sF FETCH_SIZE -- $B
    run ${W}sW WRITE_SIZE -- $B
    run ${W}sM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B
    run ${W}rF FETCH_SIZE -- $K
    run ${W}rW WRITE_SIZE -- $K
    run ${W}rM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- $K
    OUT=$R/gpurun_out/r06_pmc.json; [ $W = c5 ] && OUT=$R/gpurun_out/r06_pmc_c5.json
    (cd $R && python3 tools/pmc_step.py $OUT gpurun_out/pmc_${W}sF gpurun_out/pmc_${W}sW gpurun_out/pmc_${W}sM \
       gpurun_out/pmc_${W}rF gpurun_out/pmc_${W}rW gpurun_out/pmc_${W}rM gpurun_out/replay_manifest_$W.json \
       > gpurun_out/r06_pmc_$W.log 2>&1) || { echo "SUMFAIL $W"; tail -30 $R/gpurun_out/r06_pmc_$W.log; exit 1; }
    echo "pmc summary $W written"
  done
  ;;
bench)
  # profiles/r06_pmc*.json must hold this tree's passes (bench.py quotes them only on a digest match)
  timeout -k 10 400 python bench.py > gpurun_out/r06_bench_final.json 2> gpurun_out/r06_bench_final.err || { echo BENCHFAIL; tail -20 gpurun_out/r06_bench_final.err; exit 1; }
  cut -c1-300 gpurun_out/r06_bench_final.json
  timeout -k 10 300 python bench.py --config5 --no-cpu-baseline --no-dp-line > gpurun_out/r06_bench_c5.json 2> gpurun_out/r06_bench_c5.err || { echo C5FAIL; tail -20 gpurun_out/r06_bench_c5.err; exit 1; }
  cut -c1-200 gpurun_out/r06_bench_c5.json
  timeout -k 10 300 python bench.py --model vit > gpurun_out/r06_bench_vit.json 2> gpurun_out/r06_bench_vit.err || { echo VITFAIL; tail -20 gpurun_out/r06_bench_vit.err; exit 1; }
  cut -c1-200 gpurun_out/r06_bench_vit.json
  timeout -k 10 300 python bench.py --dp --no-cpu-baseline --no-kernel-rooflines > gpurun_out/r06_bench_dp.json 2> gpurun_out/r06_bench_dp.err || { echo DPFAIL; tail -20 gpurun_out/r06_bench_dp.err; exit 1; }
  cut -c1-200 gpurun_out/r06_bench_dp.json
  timeout -k 10 300 python tools/collate_bench.py gpurun_out/r06_collate.json --workers 0,4,8,16 > gpurun_out/r06_collate.log 2>&1 || { echo COLFAIL; tail -20 gpurun_out/r06_collate.log; exit 1; }
  tail -4 gpurun_out/r06_collate.log
  timeout -k 10 300 python tools/sga_launches.py 20 > gpurun_out/r06_sga_launches.txt 2>&1 || { echo SGAFAIL; exit 1; }
  tail -1 gpurun_out/r06_sga_launches.txt
  (while true; do date > gpurun_out/dp8.heartbeat; sleep 30; done) &
  hb=$!
  timeout -k 10 600 python bench.py --gpus 8 --rehearse --steps 2 --warmup 1 > gpurun_out/r06_dp8.json 2> gpurun_out/r06_dp8.err
  rc=$?
  kill $hb
  cut -c1-300 gpurun_out/r06_dp8.json; grep -v amdgpu.ids gpurun_out/r06_dp8.err | tail -5
  exit $rc
  ;;
esac
