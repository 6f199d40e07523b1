#!/bin/bash
# PMC passes (each counter group in a run of its own) over the benched step and over
# tools/kernel_replay.py; summary -> gpurun_out/r02_pmc.json (copied to profiles/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {  # tag counters... -- cmd
  local tag=$1; shift
  local ctrs=()
  while [ "$1" != "--" ]; do ctrs+=("$1"); shift; done; shift
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
cd $R && python3 tools/pmc_step.py gpurun_out/r02_pmc.json gpurun_out/pmc_sF gpurun_out/pmc_sW gpurun_out/pmc_sM \
   gpurun_out/pmc_rF gpurun_out/pmc_rW gpurun_out/pmc_rM gpurun_out/replay_manifest.json > gpurun_out/r02_pmc.log 2>&1 \
   || { echo SUMFAIL; tail -30 gpurun_out/r02_pmc.log; exit 1; }
tail -60 gpurun_out/r02_pmc.log
