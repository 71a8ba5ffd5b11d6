#!/bin/bash
# End-of-session measurements of the product library on one GPU box:
#   GPU parity suite; PMC passes (traffic + VALU/LDS counters) over the C3 step;
#   the default bench line (C3, CPU baselines) reading this library's traffic;
#   the other BASELINE configs; the strong-scaling per-rank shares; a
#   rocprofv3 kernel-trace summary.
# usage: tools/r4_final.sh TAG
set -o pipefail
TAG=${1:-fin}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|passed|failed" $OUT/gpu_tests.log | tail -8; exit 1; }
tail -1 $OUT/gpu_tests.log
# PMC passes, one counter group per run (kernel trace only)
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc/p$i -o run --output-format csv -- \
      python $R/tools/kernel_lab.py --reps 1 > $OUT/pmc_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc_p$i.log; exit 1; }
done
cd $R
python tools/pmc_traffic.py profiles/r04/pmc_traffic.json $OUT/pmc/p1 $OUT/pmc/p2 > $OUT/pmc_traffic.log 2>&1 || exit 1
cp profiles/r04/pmc_traffic.json $OUT/pmc_traffic.json
python tools/pmc_summary.py $OUT/pmc/p1 $OUT/pmc/p2 $OUT/pmc/p3 $OUT/pmc/p4 > $OUT/pmc_summary.txt 2>&1 || exit 1
# default bench line (no flags: C3, 20 timed steps, CPU baselines)
timeout -k 10 600 python bench.py > $OUT/bench_c3_default.json 2> $OUT/bench_c3_default.err || { tail -5 $OUT/bench_c3_default.err; exit 1; }
cut -c1-600 $OUT/bench_c3_default.json
for w in c4 c2 c5 s5; do
  steps=10; [ $w = c5 ] && steps=5
  timeout -k 10 300 python bench.py --workload $w --steps $steps --warmup 2 --no-cpu > $OUT/bench_$w.json 2> $OUT/bench_$w.err \
    || { echo "$w failed"; tail -3 $OUT/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', d['ms_per_step'], 'steady', d['step_ms_steady'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
for nc in 256 512; do
  timeout -k 10 300 python bench.py --no-cpu --steps 30 --nchan $nc > $OUT/bench_n$nc.json 2> $OUT/bench_n$nc.err \
    || { echo "nchan $nc failed"; tail -3 $OUT/bench_n$nc.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_n$nc.json')); print('nchan', $nc, d['ms_per_step'], 'steady', d['step_ms_steady'], 'kern', round(d['gpu_kernel_ms_per_step'],3))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python $R/bench.py --steps 3 --warmup 1 --no-cpu > $OUT/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
cut -d, -f1-4 $OUT/kernel_stats.csv | cut -c1-160 | head -8
