set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-x}
timeout -k 10 500 python tools/callprof.py 64 --autotune --configs > gpurun_out/callprof_$TAG.log 2>&1 || { echo CPFAIL; tail -30 gpurun_out/callprof_$TAG.log; exit 1; }
tail -30 gpurun_out/callprof_$TAG.log
