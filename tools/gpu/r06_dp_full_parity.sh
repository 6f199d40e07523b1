# r06: config 2 (world 2) and config 3 (world 8, global batch 512) DP legs at the benched shape vs one
# engine on the global batch (tools/dp_full_parity.py; ranks over gloo on the one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
(while true; do date > gpurun_out/dpfull.heartbeat; sleep 30; done) &
hb=$!
rc=0
for W in 2 8; do
  timeout -k 10 900 python -u tools/dp_full_parity.py gpurun_out/r06_c2_dp${W}_parity.json c2full $W > gpurun_out/r06_c2_dp${W}_parity.log 2>&1
  rc=$?
  grep -v -E "amdgpu.ids|Gloo|socket.cpp|Expected number" gpurun_out/r06_c2_dp${W}_parity.log | tail -3 | cut -c1-700
  [ $rc -eq 0 ] || break
done
kill $hb
exit $rc
