# L2 hit rate and fill bytes of our GEMM on one shape/config (argument 1: config list, 2: shape)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $R/gpurun_out/gpmc1 -o run -f csv -- python3 $R/tools/gemm_micro.py $1 10 $2 > $R/gpurun_out/gpmc1.log 2>&1 || { echo PMC1FAIL; tail -5 $R/gpurun_out/gpmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $R/gpurun_out/gpmc2 -o run -f csv -- python3 $R/tools/gemm_micro.py $1 10 $2 > $R/gpurun_out/gpmc2.log 2>&1 || { echo PMC2FAIL; tail -5 $R/gpurun_out/gpmc2.log; exit 1; }
echo done
