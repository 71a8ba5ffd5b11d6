#!/bin/bash
# Same-box comparison of several builds on the C3 bench line (round-robin,
# 2 rounds), after the GPU parity tests of the product library.
# usage: tools/r3_abn.sh TAG "name=lib[@VAR=val] ..." [skip-tests]   (lib "-" = product)
# The kernels read no environment switch (round 4 removed them all; the
# rejected variants live in the git history): only the variables the Python
# layer reads (PSS_HOST_THREADS, PSS_NO_MALLOPT) may follow "@" -- anything
# else would silently measure the product build twice, so it is refused.
set -o pipefail
TAG=${1:-abn}
LIBS=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
if [ "$3" != skip-tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
      -p no:cacheprovider > $OUT/gpu_tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" $OUT/gpu_tests_$TAG.log | tail -8
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
for i in 1 2; do
  for nl in $LIBS; do
    t=${nl%%=*}; lib=${nl#*=}
    envs=""; case "$lib" in *@*) envs=${lib#*@}; lib=${lib%%@*} ;; esac   # name=lib@VAR=val[,VAR2=val]
    if [ "$lib" = - ]; then unset PSS_LIB_PATH; else export PSS_LIB_PATH=$lib; fi
    unset PSS_HOST_THREADS PSS_NO_MALLOPT
    for e in ${envs//,/ }; do
      case "${e%%=*}" in
        PSS_HOST_THREADS|PSS_NO_MALLOPT) export "$e" ;;
        *) echo "r3_abn.sh: $e is not read by the library or the API layer (no env switches since round 4)"; exit 2 ;;
      esac
    done
    timeout -k 10 300 python bench.py --no-cpu --steps ${AB_STEPS:-20} ${AB_ARGS:-} > $OUT/ab_${TAG}_${t}_$i.json 2> $OUT/ab_${TAG}_${t}_$i.err \
      || { echo "$t $i failed"; tail -3 $OUT/ab_${TAG}_${t}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/ab_${TAG}_${t}_$i.json')); p=d['gpu_power'] or {}; print('$t', $i, d['ms_per_step'], d['step_ms_steady'], round(d['gpu_kernel_ms_per_step'],2), {k: v['avg_ms'] for k, v in d['kernels'].items()}, p.get('sclk_mhz_median'), p.get('socket_w_median'))"
  done
done
unset PSS_LIB_PATH
