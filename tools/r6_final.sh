#!/bin/bash
# Round-6 end-of-round measurements, part 1 (one GPU box): the GPU parity
# suite, PMC passes over the C3 step (one counter group per rocprofv3 run,
# kernel trace only), and the rocprofv3 kernel trace of a short C3 bench run.
# Writes profiles/r06/{pmc_traffic,kernel_profile}.json on the box (read by
# bench.py in part 2) and copies everything under gpurun_out/r06/$TAG.
# usage: tools/r5_final.sh TAG
set -o pipefail
TAG=${1:-fin}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06/$TAG; mkdir -p $OUT; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $OUT/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|passed|failed" $OUT/gpu_tests.log | tail -8; exit 1; }
tail -1 $OUT/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc/p$i -o run --output-format csv -- \
      python3 $R/tools/kernel_lab.py --reps 1 > $OUT/pmc_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc_p$i.log; exit 1; }
done
echo "pmc passes ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu > $OUT/prof_bench.json 2> $OUT/prof.log || { echo "rocprof failed"; tail -5 $OUT/prof.log; exit 1; }
cd $R
mkdir -p profiles/r06
python tools/pmc_traffic.py profiles/r06/pmc_traffic.json $OUT/pmc/p1 $OUT/pmc/p2 > $OUT/pmc_traffic.log 2>&1 || exit 1
cp profiles/r06/pmc_traffic.json $OUT/pmc_traffic.json
python tools/pmc_summary.py $OUT/pmc/p1 $OUT/pmc/p2 $OUT/pmc/p3 $OUT/pmc/p4 > $OUT/pmc_summary.txt 2>&1 || exit 1
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
tr=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py $tr --json profiles/r06/kernel_profile.json > $OUT/kernel_summary.md || exit 1
cp profiles/r06/kernel_profile.json $OUT/kernel_profile.json
rm -rf $OUT/prof $OUT/pmc            # raw CSVs: the summaries above carry what is kept
cat $OUT/kernel_profile.json; head -12 $OUT/pmc_summary.txt
