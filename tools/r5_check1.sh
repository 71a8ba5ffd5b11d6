#!/bin/bash
# Round-5 session check: full GPU suite, fused-K3 timing, L3 residency probes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r05; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_1.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed|Error" $OUT/gpu_tests_1.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/k3_bench.py 512 20 8 7.3 > $OUT/k3_bench.txt 2>&1 || exit $?
for n in 8 16 2048; do
  timeout -k 10 180 python bench.py --workload c5 --log2n 22 --nchan $n --steps 10 --no-cpu > $OUT/l3_c5l22_n$n.json 2> $OUT/l3_c5l22_n$n.err || exit $?
done
timeout -k 10 300 ./tools/l3_spill 8 > $OUT/l3_spill_2.txt 2>&1 || exit $?
