#!/bin/bash
# round-2 diagnostic call: VALU issue rates at the in-kernel clock + ablations
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 120 $R/tools/probe_rates > $R/gpurun_out/probe_rates.txt 2>&1 || { echo "probe failed"; exit 1; }
cat $R/gpurun_out/probe_rates.txt
VARIANTS="${VARIANTS}" LAB_VARIANTS="${LAB_VARIANTS:-full}" bash $R/tools/ablate.sh run ${TAG:-abl}
