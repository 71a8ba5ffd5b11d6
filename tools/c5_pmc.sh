#!/bin/bash
# Two PMC passes (issue / wait and LDS / instruction counters) over one C5 step (bench.py --workload c5, one warm-up); summary under gpurun_out/r06/c5pmc.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r06/c5pmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc/p$i -o run --output-format csv -- \
      python3 $R/bench.py --workload c5 --steps 1 --warmup 1 --no-cpu > $OUT/pmc_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc_p$i.log; exit 1; }
done
cd $R
python tools/pmc_summary.py $OUT/pmc/p1 $OUT/pmc/p2 > $OUT/pmc_summary.txt 2>&1 || exit 1
rm -rf $OUT/pmc
head -80 $OUT/pmc_summary.txt
