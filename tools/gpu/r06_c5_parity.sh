# r06: config 5's DP leg at the benched shape vs one engine on the global batch (tools/dp_full_parity.py)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
(while true; do date > gpurun_out/c5par.heartbeat; sleep 30; done) &
hb=$!
timeout -k 10 1000 python -u tools/dp_full_parity.py gpurun_out/r06_c5_dp2_parity.json > gpurun_out/r06_c5_dp2_parity.log 2>&1
rc=$?
kill $hb
grep -v -E "amdgpu.ids|Gloo|socket.cpp" gpurun_out/r06_c5_dp2_parity.log | tail -6 | cut -c1-600
exit $rc
