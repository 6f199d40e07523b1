#!/bin/bash
# quick GPU iteration: selected tests (PYTEST_K), then the bench (no CPU baseline) and an optional EXTRA command
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "$PYTEST_K" \
     > gpurun_out/quick_test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/quick_test.log; exit 1; }
  tail -2 gpurun_out/quick_test.log
fi
if [ -z "${NO_BENCH:-}" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernel-rooflines ${BENCH_ARGS:-} > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err || { echo BENCHFAIL; tail -20 gpurun_out/quick_bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/quick_bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
fi
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 600 bash -c "$EXTRA" > gpurun_out/quick_extra.log 2>&1 || { echo EXTRAFAIL; tail -20 gpurun_out/quick_extra.log; exit 1; }
  tail -12 gpurun_out/quick_extra.log
fi
