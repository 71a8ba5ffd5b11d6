#!/bin/bash
# K3 timing + L3 residency with the real kernels + golden replays
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r05; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "golden_replay or observe or utils or smoke" > $OUT/gpu_tests_2.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed|Error" $OUT/gpu_tests_2.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/k3_bench.py 512 20 > $OUT/k3_bench2.txt 2>&1 || exit $?
timeout -k 10 300 python tools/l3_real.py 8 16 32 64 2048 > $OUT/l3_real.txt 2>&1 || exit $?
