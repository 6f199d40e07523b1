#!/bin/bash
# config-5 depth: the 6-block parity tests, then the B=64 step with 6 SGA blocks at 224 and 384
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -v --timeout 200 --timeout-method thread -p no:cacheprovider \
   -k "six_blocks or 700_answers or at_384" > gpurun_out/r02c_six_test.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/r02c_six_test.log | tail -2
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/r02c_six_test.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --blocks 6 --no-cpu-baseline > gpurun_out/r02c_six224.json 2> gpurun_out/r02c_six224.err || { echo BENCHFAIL; tail -20 gpurun_out/r02c_six224.err; exit 1; }
cut -c1-400 gpurun_out/r02c_six224.json
timeout -k 10 300 python bench.py --blocks 6 --image-size 384 --no-cpu-baseline > gpurun_out/r02c_six384.json 2> gpurun_out/r02c_six384.err || { echo BENCHFAIL; tail -20 gpurun_out/r02c_six384.err; exit 1; }
cut -c1-400 gpurun_out/r02c_six384.json
