#!/bin/bash
# Null-refine tests (list vs per-sample, replay bounds) on the GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r05; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    -k "refine or c4 or bluestein or golden_replay or null" > $OUT/gpu_tests_8.log 2>&1 \
    || { echo "tests failed"; grep -E "^FAILED|passed|failed|Error" $OUT/gpu_tests_8.log | tail -12; exit 1; }
tail -1 $OUT/gpu_tests_8.log
