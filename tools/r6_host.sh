#!/bin/bash
# Host-side measurements on the GPU box: per-call profiles of the small
# workloads, the C3 first step's host planning, and the bench lines they move.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r06/${1:-host}; mkdir -p $OUT
for w in t2 c4; do
  timeout -k 10 200 python tools/host_prof.py $w > $OUT/host_prof_$w.txt 2>&1 || { tail -5 $OUT/host_prof_$w.txt; exit 1; }
  head -3 $OUT/host_prof_$w.txt
done
timeout -k 10 200 python tools/host_first.py 2048 > $OUT/host_first2048.txt 2>&1 || exit 1
head -2 $OUT/host_first2048.txt
for w in t2 t1 c4 n256 c3; do
  case $w in n256) A="--nchan 256 --no-cpu";; c3) A="--no-cpu";; *) A="--workload $w --no-cpu";; esac
  timeout -k 10 300 python bench.py $A > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -3 $OUT/bench_$w.err; exit 1; }
  python tools/r6_line.py $OUT/bench_$w.json
done
