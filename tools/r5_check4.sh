#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r05; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "golden_replay or observe or utils" > $OUT/gpu_tests_4.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed|Error" $OUT/gpu_tests_4.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/k3_bench.py 512 20 1 8 7.3 4 64 > $OUT/k3_bench4.txt 2>&1 || exit $?
