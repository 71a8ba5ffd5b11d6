#!/bin/bash
# Kernel-trace summary of a short bench run (rocprofv3 --kernel-trace
# --stats, CSV) and the per-kernel table; usage: tools/r4_prof.sh TAG [bench args]
set -o pipefail
TAG=${1:-prof}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
    python bench.py --no-cpu --steps 5 --warmup 2 "$@" > $OUT/prof_$TAG.json 2> $OUT/prof_$TAG.err || exit $?
f=$(find $OUT/prof_$TAG -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print("%-70s %6s %10.4f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
