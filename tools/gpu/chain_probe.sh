#!/bin/bash
# tools/chain_probe.py under HIP runtime knobs, one process each (chained: a failure ends the run)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  echo "== $*" | tee -a gpurun_out/chain_probe.txt
  env "$@" timeout -k 10 240 python -X faulthandler tools/chain_probe.py $VARIANTS >> gpurun_out/chain_probe.txt 2> gpurun_out/chain_probe.err || { echo FAIL $?; tail -20 gpurun_out/chain_probe.err; exit 1; }
  tail -1 gpurun_out/chain_probe.txt
}
rm -f gpurun_out/chain_probe.txt
for e in "$@"; do run $e; done
