#!/bin/bash
# GPU suite + the refine-cost profile (tools/r5_refine.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r05; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_6.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|passed|failed|Error" $OUT/gpu_tests_6.log | tail -12; exit 1; }
tail -1 $OUT/gpu_tests_6.log
bash tools/r5_refine.sh
