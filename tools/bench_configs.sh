#!/bin/bash
# Bench lines of the other BASELINE configs (C4, C2, C5) on one GPU.
# usage: tools/bench_configs.sh TAG
set -o pipefail
TAG=${1:-cfg}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for w in c4 c2 c5; do
  steps=10; [ $w = c5 ] && steps=5
  timeout -k 10 300 python bench.py --workload $w --steps $steps --warmup 2 --no-cpu --verbose \
      > $OUT/bench_${TAG}_$w.json 2> $OUT/bench_${TAG}_$w.err || { echo "$w failed"; tail -5 $OUT/bench_${TAG}_$w.err; exit 1; }
  cut -c1-400 $OUT/bench_${TAG}_$w.json
done
