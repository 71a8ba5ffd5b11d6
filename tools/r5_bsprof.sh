#!/bin/bash
# Kernel stats of the Bluestein headline case (tools/bs_one.py) under rocprofv3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/bsprof; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/raw -o bs -- \
    python3 $R/tools/bs_one.py ${1:-512} ${2:-1048574} > $OUT/log.txt 2>&1 || exit $?
f=$(find $OUT/raw -name "*kernel_stats.csv" | head -1)
cp $f $OUT/kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print("%-90s %6s %10.4f %8.2f" % (r["Name"][:90], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["Percentage"])))
PY
