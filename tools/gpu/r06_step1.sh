# r06: the chain-only graph beside the next batch's ResNet on a CU-masked stream created AFTER instantiation
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
VARIANTS="full chain" bash tools/gpu/chain_probe.sh POST=plain,all,hi:64,st:4:1,hi:128,st:2:1,hi:32 || { tail -40 gpurun_out/chain_probe.err; exit 1; }
