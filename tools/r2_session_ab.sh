#!/bin/bash
# Same-box A/B of two library builds on the C3 bench line (alternating runs).
# usage: tools/r2_session_ab.sh OLD_LIB   (the product library is the other)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
OLD=$1
for i in 1 2; do
  for tag in new old; do
    if [ $tag = old ]; then export PSS_LIB_PATH=$OLD; else unset PSS_LIB_PATH; fi
    timeout -k 10 300 python bench.py --no-cpu --steps 20 > $OUT/ab_${tag}_$i.json 2> $OUT/ab_${tag}_$i.err || { echo "$tag $i failed"; tail -3 $OUT/ab_${tag}_$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$OUT/ab_${tag}_$i.json')); p=d['gpu_power'] or {}; print('$tag', $i, d['ms_per_step'], d['step_ms_steady'], round(d['gpu_kernel_ms_per_step'],2), {k: v['avg_ms'] for k, v in d['kernels'].items()}, p.get('sclk_mhz_median'))"
  done
done
