set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${TAG:-x}
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --no-cpu-baseline --tune-save gpurun_out/gemm_gfx950_$TAG.json > gpurun_out/b_$TAG.json 2> gpurun_out/b_$TAG.err || { echo BENCHFAIL; tail -20 gpurun_out/b_$TAG.err; exit 1; }
cat gpurun_out/b_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $R/gpurun_out/pmcF_$TAG -o fetch -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --tune-table $R/gpurun_out/gemm_gfx950_$TAG.json > $R/gpurun_out/pmcF_$TAG.log 2>&1 || { echo PMCFAIL; tail -20 $R/gpurun_out/pmcF_$TAG.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $R/gpurun_out/pmcW_$TAG -o write -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --tune-table $R/gpurun_out/gemm_gfx950_$TAG.json > $R/gpurun_out/pmcW_$TAG.log 2>&1 || { echo PMCFAIL; tail -20 $R/gpurun_out/pmcW_$TAG.log; exit 1; }
cd $R && python tools/pmc_traffic.py gpurun_out/pmcF_$TAG/*/ gpurun_out/pmcW_$TAG/*/ gpurun_out/pmc_traffic_$TAG.json || python tools/pmc_traffic.py gpurun_out/pmcF_$TAG gpurun_out/pmcW_$TAG gpurun_out/pmc_traffic_$TAG.json
