#!/bin/bash
# Round-4 quick check: targeted GPU tests (fast == generic bitwise, fast path
# vs oracle, shard invariance, golden replays) then a same-box A/B of the C3
# bench against other builds.
# usage: tools/r4_check.sh TAG "name=lib ..." [test-filter]
set -o pipefail
TAG=${1:-chk}
LIBS=$2
FILT=${3:-"fast_path or shard_invariance or golden_replay or fourstep_pair"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
KARG=(-k "$FILT"); [ "$FILT" = all ] && KARG=()
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    "${KARG[@]}" > $OUT/gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed|Error" $OUT/gpu_tests_$TAG.log | tail -8
[ $rc -ne 0 ] && exit $rc
if [ -n "$LIBS" ]; then bash tools/r3_abn.sh $TAG "$LIBS" skip-tests; fi
