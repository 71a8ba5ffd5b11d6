#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r05; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_5.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed|Error" $OUT/gpu_tests_5.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload c5 --no-cpu > $OUT/bench_c5_split.json 2> $OUT/bench_c5_split.err || exit $?
tail -c 700 $OUT/bench_c5_split.json
