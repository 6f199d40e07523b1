#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/counters_list.txt 2>&1 || true
grep -E "SQ_WAVE_CYCLES|SQ_WAIT_ANY|SQ_LDS_BANK_CONFLICT|TCC_HIT|TA_BUSY|SQ_INSTS_LDS|TCP_TCC" $R/gpurun_out/counters_list.txt | head -20
K="python3 $R/tools/kernel_replay.py $R/gpurun_out/res_manifest.json 3 res"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $R/gpurun_out/rp1 -o rp1 -- $K > $R/gpurun_out/rp1.log 2>&1 || { echo P1FAIL; tail $R/gpurun_out/rp1.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -f csv -d $R/gpurun_out/rp2 -o rp2 -- $K > $R/gpurun_out/rp2.log 2>&1 || { echo P2FAIL; tail $R/gpurun_out/rp2.log; exit 1; }
cd $R && python3 tools/pmc_kernels.py gpurun_out/res_manifest.json gpurun_out/rp1 gpurun_out/rp2 > gpurun_out/res_pmc.txt 2>&1; cat gpurun_out/res_pmc.txt
