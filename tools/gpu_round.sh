#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace.
# usage: tools/gpu_round.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/gpu_tests_$TAG.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python bench.py "$@" > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || exit $?
cat $OUT/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o run --output-format csv -- python $R/bench.py --steps 2 --warmup 1 --no-cpu > $OUT/prof_$TAG.log 2>&1 || exit $?
find $OUT/prof_$TAG -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-220 | head -20
