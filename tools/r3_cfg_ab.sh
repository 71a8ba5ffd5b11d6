#!/bin/bash
# GPU parity tests, then same-box A/B bench lines of a BASELINE config
# (product library vs an older build, alternating runs).
# usage: tools/r3_cfg_ab.sh TAG OLD_LIB "c4 c5" [skip-tests]
set -o pipefail
TAG=${1:-cfg}
OLD=$2
WLS=${3:-c4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
if [ "$4" != skip-tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > $OUT/gpu_tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/gpu_tests_$TAG.log | tail -8
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
for w in $WLS; do
  steps=10; [ $w = c5 ] && steps=5
  for i in 1 2; do
    for t in new old; do
      if [ $t = old ]; then export PSS_LIB_PATH=$OLD; else unset PSS_LIB_PATH; fi
      timeout -k 10 300 python bench.py --workload $w --steps $steps --warmup 2 --no-cpu \
          > $OUT/ab_${TAG}_${w}_${t}_$i.json 2> $OUT/ab_${TAG}_${w}_${t}_$i.err \
        || { echo "$w $t $i failed"; tail -3 $OUT/ab_${TAG}_${w}_${t}_$i.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/ab_${TAG}_${w}_${t}_$i.json')); print('$w', '$t', $i, d['ms_per_step'], d['step_ms_steady'], round(d['gpu_kernel_ms_per_step'],3), {k: v['avg_ms'] for k, v in d['kernels'].items()})"
    done
  done
  unset PSS_LIB_PATH
done
