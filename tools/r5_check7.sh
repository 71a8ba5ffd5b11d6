#!/bin/bash
# Full GPU suite + smoke on the current library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r05; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_7.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|passed|failed|Error" $OUT/gpu_tests_7.log | tail -12; exit 1; }
tail -1 $OUT/gpu_tests_7.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_7.log 2>&1 || { tail -5 $OUT/smoke_7.log; exit 1; }
tail -1 $OUT/smoke_7.log
