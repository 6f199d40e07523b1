# r06: BASELINE config 5's DP leg at full size on one GPU: two ranks over gloo (bench --rehearse),
# B = 64 per rank, 384^2, T5-large, 6 SGA blocks, e4m3 forward GEMMs; the bench checks lockstep
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
(while true; do date > gpurun_out/c5dp2.heartbeat; sleep 30; done) &
hb=$!
timeout -k 10 900 python bench.py --config5 --gpus 2 --rehearse --steps 2 --warmup 1 > gpurun_out/r06_c5_dp2.json 2> gpurun_out/r06_c5_dp2.err
rc=$?
kill $hb
cut -c1-400 gpurun_out/r06_c5_dp2.json; grep -v -E "amdgpu.ids|Gloo" gpurun_out/r06_c5_dp2.err | tail -5
exit $rc
