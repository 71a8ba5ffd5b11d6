#!/bin/bash
# Round-6 GPU check: full GPU suite, smoke, instruction-rate probe, C3 bench
# line.  usage: tools/r6_check.sh TAG   (outputs under gpurun_out/r06/TAG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r06/${1:-check}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|passed|failed|Error" $OUT/gpu_tests.log | tail -12; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
if [ -x tools/probe_rates ]; then
  timeout -k 10 120 ./tools/probe_rates > $OUT/probe_rates.txt 2>&1 || exit 1
  cat $OUT/probe_rates.txt
fi
timeout -k 10 300 python bench.py --no-cpu > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -5 $OUT/bench_c3.err; exit 1; }
python tools/r6_line.py $OUT/bench_c3.json
