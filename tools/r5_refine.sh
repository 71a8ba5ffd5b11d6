#!/bin/bash
# rocprofv3 kernel stats of tools/refine_cost.py (the float64 null refine's launches).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/refine; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/raw -o k -- \
    python3 $R/tools/refine_cost.py > $OUT/log.txt 2>&1 || { tail -5 $OUT/log.txt; exit 1; }
grep "per run" $OUT/log.txt
f=$(find $OUT/raw -name "*kernel_trace.csv" | head -1)
python3 $R/tools/prof_summary.py $f > $OUT/summary.md
head -24 $OUT/summary.md | cut -c1-170
