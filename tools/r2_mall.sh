#!/bin/bash
# round-2 diagnostics: VALU rates (wall x in-kernel clock) + per-kernel time vs channel batch size
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 180 $R/tools/probe_rates > $R/gpurun_out/probe_rates2.txt 2>&1 || { echo "probe failed"; exit 1; }
cat $R/gpurun_out/probe_rates2.txt
for n in 16 32 64 256 2048; do
  timeout -k 10 300 python $R/tools/kernel_lab.py --no-fill --reps 4 --nchan $n full nonull > $R/gpurun_out/mall_$n.log 2>&1 || { echo "lab $n failed"; tail -5 $R/gpurun_out/mall_$n.log; exit 1; }
  echo "nchan $n"; grep wall $R/gpurun_out/mall_$n.log
done
