#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=gpurun_out/r05/bs2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "bluestein or filter_rows or shift_t or golden_replay or simulate or baseband or observe or shard or fastpath or stats" > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed|Error" $OUT/tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bs_time.py > $OUT/bs_time.txt 2>&1 || exit $?
tail -5 $OUT/bs_time.txt
timeout -k 10 200 python bench.py --workload t1 > $OUT/bench_t1.json 2> $OUT/bench_t1.err || exit $?
python -c "import json; d=json.loads(open('$OUT/bench_t1.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['step_ms_first'], d['step_ms_steady'], d['kernels'], d['published_shape']['gpu_disperse_only'])"
bash tools/r5_bsprof.sh
