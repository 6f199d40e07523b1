# r06: kernel traces of the chain-only graph with and without a CU-masked stream created before capture
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
for pre in none cumask; do
  rm -rf gpurun_out/ct_$pre
  PRE=$pre timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ct_$pre -o run -- python tools/chain_probe.py chain > gpurun_out/ct_$pre.log 2>&1 || { echo FAIL $pre; tail -20 gpurun_out/ct_$pre.log; exit 1; }
  tail -1 gpurun_out/ct_$pre.log
  db=$(find gpurun_out/ct_$pre -name "*.db" | head -1)
  python tools/steptrace.py $db --list --back 2 > gpurun_out/steptrace_ct_$pre.txt
  head -12 gpurun_out/steptrace_ct_$pre.txt
done
