#!/bin/bash
# Round-6 end-of-round measurements, part 2: the default bench line (C3,
# 20 timed steps, CPU baselines; reads profiles/r06/{pmc_traffic,
# kernel_profile}.json from part 1) and the other workloads.
# usage: tools/r5_final2.sh TAG
set -o pipefail
TAG=${1:-fin}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06/$TAG; mkdir -p $OUT; cd $R
timeout -k 10 500 python bench.py > $OUT/bench_c3_default.json 2> $OUT/bench_c3_default.err || { tail -5 $OUT/bench_c3_default.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_c3_default.json').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'], 'first', d['step_ms_first'], 'steady', d['step_ms_steady'], {k: v['avg_ms'] for k, v in d['kernels'].items()}, d['roofline'].get('frac'), d['roofline'].get('frac_profile'))"
for w in c4 c2 c5 s5 t1 t2; do
  nc="--no-cpu"; case $w in t1|t2) nc="";; esac      # (t1 / t2: the oracle on the same shape)
  timeout -k 10 300 python bench.py --workload $w $nc > $OUT/bench_$w.json 2> $OUT/bench_$w.err \
    || { echo "$w failed"; tail -3 $OUT/bench_$w.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1]); print('$w', d['ms_per_step'], 'first', d.get('step_ms_first'), 'steady', d.get('step_ms_steady'), {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
for nc in 256 512; do
  timeout -k 10 300 python bench.py --no-cpu --nchan $nc > $OUT/bench_n$nc.json 2> $OUT/bench_n$nc.err \
    || { echo "nchan $nc failed"; tail -3 $OUT/bench_n$nc.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/bench_n$nc.json').read().strip().splitlines()[-1]); print('n$nc', d['ms_per_step'], 'first', d['step_ms_first'], 'steady', d['step_ms_steady'])"
done
# the first timed step on an idle GPU, decomposed (host planning, the step's
# own kernels against the steady state's, tools/first_step.py)
timeout -k 10 200 python tools/first_step.py 2048 2 > $OUT/first_step.txt 2>&1 || { echo "first_step failed"; exit 1; }
grep "step [01] " $OUT/first_step.txt
