# GPU tests, then a same-box A/B of the grad-norm overlap (VQA_SQ_OVERLAP) and a kernel-stats profile
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t11.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t11.log; exit 1; }
tail -2 gpurun_out/t11.log
VAR=VQA_SQ_OVERLAP bash tools/gpu/env_ab.sh "1 0 1 0 1" || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof11 -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/p11.log 2>&1 || { echo PROFFAIL; tail -20 $R/gpurun_out/p11.log; exit 1; }
echo done
