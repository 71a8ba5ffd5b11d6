#!/bin/bash
# C3 wall time with pair batches whose pass A runs next to the previous
# batch's pass C (PSS_BATCH_AFTER=row), for the product pass C (16 columns)
# and an 8-column pass C that leaves LDS for a pass-A workgroup per CU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
for lib in libpss_hip libpss_hip_ablbc8; do
  for cfg in "1 a" "2 row" "4 row" "8 row" "4 a"; do
    set -- $cfg
    PSS_LIB_PATH=$R/psrsigsim_amd/$lib.so PSS_BATCHES=$1 PSS_BATCH_AFTER=$2 timeout -k 10 300 \
      python tools/kernel_lab.py --no-fill --reps 3 full > $OUT/ov_${lib}_$1_$2.log 2>&1 || { echo "$lib $cfg failed"; tail -3 $OUT/ov_${lib}_$1_$2.log; exit 1; }
    echo "$lib batches=$1 after=$2: $(grep wall $OUT/ov_${lib}_$1_$2.log)"
  done
done
