#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out/dot && cd gpurun_out/dot
DEBUG_HIP_GRAPH_DOT_PRINT=1 timeout -k 10 300 python -u -m pytest "$R/tests/test_dp_gpu.py::test_dp_world1_matches_single_gpu[True-False]" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider --rootdir $R > ../r04_dot.log 2>&1 || { echo FAIL; tail -20 ../r04_dot.log; exit 1; }
ls -la | head -20
for f in *; do echo "== $f"; grep -o 'label="[A-Za-z_]*' "$f" | sort | uniq -c | sort -rn | head -12; done 2>/dev/null | head -80
