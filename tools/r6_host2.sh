#!/bin/bash
# Host planning thread-count sweep (first-step planning of C3 on an idle GPU)
# and the small-workload bench lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r06/${1:-host2}; mkdir -p $OUT
for th in 8 12 16 8; do
  PSS_HOST_THREADS=$th timeout -k 10 200 python tools/host_first.py 2048 > $OUT/host_first_t$th.txt 2>&1 || exit 1
  echo "threads $th: $(grep '^host' $OUT/host_first_t$th.txt | tr '\n' ' ')"
done
for w in t2 t1 c4; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -3 $OUT/bench_$w.err; exit 1; }
  python tools/r6_line.py $OUT/bench_$w.json
done
