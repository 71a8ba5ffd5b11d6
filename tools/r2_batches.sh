#!/bin/bash
# wall time of the C3 step vs pair batches on side streams (PSS_BATCHES)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
PSS_BATCHES=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_stats.py -m gpu -x -q -k "bitwise" --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/batch_tests.log 2>&1
rc=$?; echo "bitwise tests (PSS_BATCHES=4) rc=$rc"; tail -2 $OUT/batch_tests.log
[ $rc -ne 0 ] && exit $rc
for b in ${BATCHES:-1 2 4 8}; do
  PSS_BATCHES=$b timeout -k 10 300 python tools/kernel_lab.py --no-fill --reps 4 full > $OUT/batch_$b.log 2>&1 || { echo "lab $b failed"; tail -3 $OUT/batch_$b.log; exit 1; }
  echo "batches $b"; grep wall $OUT/batch_$b.log
done
