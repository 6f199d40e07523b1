# r06: the embedding table's update split by rows: grid of the untouched-rows pass beside the backward
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu/ab_env.sh "VQA_EMB_GRID=128" "VQA_EMB_GRID=192" "VQA_EMB_GRID=256" "VQA_EMB_GRID=384" "VQA_EMB_GRID=512" "VQA_EMBED_SPLIT=0"
