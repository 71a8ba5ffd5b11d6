#!/bin/bash
# Kernel stats (rocprofv3) of the 256-channel strong-scaling share and of C4,
# to see the fixed per-run kernels next to the per-channel passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r05/small; rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for w in n256 c4; do
  if [ $w = n256 ]; then A="--nchan 256"; else A="--workload c4"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/raw_$w -o k -- \
      python3 $R/bench.py $A --steps 10 --warmup 2 --no-cpu > $OUT/bench_$w.json 2> $OUT/bench_$w.err || exit $?
  f=$(find $OUT/raw_$w -name "*kernel_stats.csv" | head -1)
  cp $f $OUT/kernel_stats_$w.csv
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:22]:
    print("%-80s %6s %9.4f %9.4f %6.2f" % (r["Name"][:80], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6, float(r["Percentage"])))
PY
done
