#!/bin/bash
# HIP API trace of the steady-state n256 steps (tools/host_stalls.py): the
# API calls that block the host for > 1 ms.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/hiptrace; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --output-format csv -d $OUT/raw -o h -- \
    python3 $R/tools/host_stalls.py 256 60 > $OUT/log.txt 2>&1 || { tail -5 $OUT/log.txt; exit 1; }
grep -E "median|step" $OUT/log.txt
f=$(find $OUT/raw -name "*hip_api_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
agg = defaultdict(list)
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    agg[r["Function"]].append(d)
print("calls > 1 ms:")
for f, v in sorted(agg.items(), key=lambda kv: -max(kv[1])):
    big = [x for x in v if x > 1.0]
    if big:
        print("  %-40s n=%d  >1ms: %d  max %.2f  sum>1ms %.1f" % (f, len(v), len(big), max(big), sum(big)))
PY
