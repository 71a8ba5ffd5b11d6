#!/bin/bash
# One GPU-box session of round 3: GPU parity tests, then a same-box A/B of the
# product library against an older build on the C3 bench line (alternating
# runs), then a rocprofv3 kernel-trace summary of the product library.
# usage: tools/r3_round.sh TAG OLD_LIB [skip-tests]
set -o pipefail
TAG=${1:-r3}
OLD=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
if [ "$3" != skip-tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > $OUT/gpu_tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/gpu_tests_$TAG.log | tail -8
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc     # 1 = some tests failed: still measure
fi
if [ -n "$OLD" ]; then
  for i in 1 2; do
    for t in new old; do
      if [ $t = old ]; then export PSS_LIB_PATH=$OLD; else unset PSS_LIB_PATH; fi
      timeout -k 10 300 python bench.py --no-cpu --steps 20 > $OUT/ab_${TAG}_${t}_$i.json 2> $OUT/ab_${TAG}_${t}_$i.err \
        || { echo "$t $i failed"; tail -3 $OUT/ab_${TAG}_${t}_$i.err; exit 1; }
      python -c "import json; d=json.load(open('$OUT/ab_${TAG}_${t}_$i.json')); p=d['gpu_power'] or {}; print('$t', $i, d['ms_per_step'], d['step_ms_steady'], round(d['gpu_kernel_ms_per_step'],2), {k: v['avg_ms'] for k, v in d['kernels'].items()}, p.get('sclk_mhz_median'), p.get('socket_w_median'))"
    done
  done
  unset PSS_LIB_PATH
fi
# strong-scaling per-rank share of C3 on one GPU: 256 ch (N = 8), 512 ch (N = 4)
for nc in 256 512; do
  timeout -k 10 300 python bench.py --no-cpu --steps 30 --nchan $nc > $OUT/bench_${TAG}_n$nc.json 2> $OUT/bench_${TAG}_n$nc.err \
    || { echo "nchan $nc failed"; tail -3 $OUT/bench_${TAG}_n$nc.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_${TAG}_n$nc.json')); print('nchan', $nc, d['ms_per_step'], 'steady', d['step_ms_steady'], 'first', d['step_ms_first'], 'kern', round(d['gpu_kernel_ms_per_step'],3))"
done
timeout -k 10 300 python tools/step_timeline.py 256 > $OUT/timeline_${TAG}_256.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- \
    python $R/bench.py --steps 3 --warmup 1 --no-cpu > $OUT/prof_$TAG.log 2>&1 || exit $?
find $OUT/prof_$TAG -name "*kernel_stats.csv" -exec cp {} $OUT/kstats_$TAG.csv \;
cut -d, -f1-8 $OUT/kstats_$TAG.csv | cut -c1-200 | head -14
