#!/bin/bash
# GPU tests then A/B kernel timings of compile-time variants on the same box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${TAG:-ab}
if [ -n "$TESTS" ]; then
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/gpu_tests_$TAG.log; grep -E "^FAILED|Error:" $OUT/gpu_tests_$TAG.log | head -5
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
VARIANTS="$VARIANTS" LAB_VARIANTS="${LAB_VARIANTS:-full}" bash tools/ablate.sh run $TAG
