#!/bin/bash
# Round-5 bench set: the default C3 line, C4, C5, the 256-channel strong-scaling share, s5,
# and the fused-K3 A/B (each step under its own time limit).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r05/${1:-bench}; mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench_c3_default.json 2> $OUT/bench_c3_default.err || exit $?
tail -c 1500 $OUT/bench_c3_default.json
timeout -k 10 200 python bench.py --workload c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit $?
timeout -k 10 200 python bench.py --nchan 256 --no-cpu > $OUT/bench_n256.json 2> $OUT/bench_n256.err || exit $?
timeout -k 10 300 python bench.py --workload c5 --no-cpu > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?
timeout -k 10 200 python bench.py --workload s5 > $OUT/bench_s5.json 2> $OUT/bench_s5.err || exit $?
timeout -k 10 200 python bench.py --workload t1 > $OUT/bench_t1.json 2> $OUT/bench_t1.err || exit $?
timeout -k 10 200 python bench.py --workload t2 > $OUT/bench_t2.json 2> $OUT/bench_t2.err || exit $?
