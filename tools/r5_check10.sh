#!/bin/bash
# Full GPU suite + host stalls + n256 / C4 / C3 bench lines (upload stream).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r05; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests_10.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|passed|failed|Error" $OUT/gpu_tests_10.log | tail -12; exit 1; }
tail -1 $OUT/gpu_tests_10.log
timeout -k 10 200 python tools/host_stalls.py 256 40 2>&1 | grep -E "median|step"
for w in n256 n256 c4 c4 c3; do
  case $w in n256) A="--nchan 256 --no-cpu";; c4) A="--workload c4 --no-cpu";; c3) A="--no-cpu";; esac
  timeout -k 10 300 python bench.py $A > $OUT/u10_$w.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$OUT/u10_$w.json').read().strip().splitlines()[-1]); print('$w', d['ms_per_step'], d['step_ms_first'], d['step_ms_steady'])"
done
