#!/bin/bash
# scaler dW as a tap-batched GEMM: parity tests that run the scaler backward, then the
# tile choices of the new shapes (config 2, 384x384 six blocks, config 5) and a bench
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "engine_matches_reference_golden or engine_vs_oracle_multistep or oracle_at_384 or six_blocks or config5 or bench_step or grouped_sga" \
  > gpurun_out/convt_test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/convt_test.log; exit 1; }
tail -2 gpurun_out/convt_test.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --steps 20 --tune-save gpurun_out/tune_c2.json \
  > gpurun_out/convt_bench.json 2> gpurun_out/convt_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/convt_bench.err; exit 1; }
cat gpurun_out/convt_bench.json
timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines --steps 10 --blocks 6 --image-size 384 --tune-save gpurun_out/tune_six384.json \
  > gpurun_out/convt_six384.json 2> gpurun_out/convt_six384.err || { echo SIXFAIL; tail -20 gpurun_out/convt_six384.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline --no-kernel-rooflines --steps 10 --config5 --tune-save gpurun_out/tune_c5.json \
  > gpurun_out/convt_c5.json 2> gpurun_out/convt_c5.err || { echo C5FAIL; tail -20 gpurun_out/convt_c5.err; exit 1; }
grep -h "autotune" gpurun_out/convt_*.err | cut -c1-300
python -c "
import json
for f in ('convt_bench', 'convt_six384', 'convt_c5'):
    d = json.load(open('gpurun_out/%s.json' % f)); print(f, d['value'], d['ms_per_step'])"
