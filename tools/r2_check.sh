#!/bin/bash
# GPU tests (all, or $TESTS) + per-kernel timings of the C3 step, pipelined vs not
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${TAG:-chk}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests_$TAG.log; grep -E "FAILED|Error" $OUT/gpu_tests_$TAG.log | head -5
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for f in 0 4; do
  timeout -k 10 300 python tools/kernel_lab.py --no-fill --reps 4 --flags $f full > $OUT/lab_${TAG}_f$f.log 2>&1 || { echo "lab failed"; tail -3 $OUT/lab_${TAG}_f$f.log; exit 1; }
  echo "flags $f"; grep wall $OUT/lab_${TAG}_f$f.log
done
