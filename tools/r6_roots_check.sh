#!/bin/bash
# Round 6: the lockstep root bisections against the previous build
# (psrsigsim_amd/libpss_hip_rootsold.so): the C3 geometry's root records and
# output rows bit for bit, then the 256-channel kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/mc; mkdir -p $O
timeout -k 10 200 python tools/mask_count.py 22 2 $O/new > $O/new.txt 2>&1 || { tail -5 $O/new.txt; exit 1; }
PSS_LIB_PATH=psrsigsim_amd/libpss_hip_rootsold.so timeout -k 10 200 python tools/mask_count.py 22 2 $O/old > $O/old.txt 2>&1 || { tail -5 $O/old.txt; exit 1; }
python - > $O/cmp.txt <<'PY' || exit 1
import numpy as np
# (the records' list order follows k_mask_table's per-wave atomics, so the
# records are compared as a multiset of 64-B rows; the rows carry their roots)
for k in ("rec", "data"):
    a = np.load("gpurun_out/mc/new_%s.npy" % k); b = np.load("gpurun_out/mc/old_%s.npy" % k)
    if k == "rec":
        a = np.sort(a.reshape(-1, 64).view("V64").ravel()); b = np.sort(b.reshape(-1, 64).view("V64").ravel())
    print(k, a.shape, b.shape, "bitwise equal" if a.shape == b.shape and a.tobytes() == b.tobytes() else "DIFFER")
PY
cat $O/cmp.txt; rm -f $O/*_data.npy $O/*_rec.npy
[ "$1" = cmp-only ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --nchan 256 > $R/$O/b256p.json 2> $R/$O/b256p.err || exit 1
find $R/$O/prof -name "*kernel_stats.csv" -exec cp {} $R/$O/kstats256.csv \;
rm -rf $R/$O/prof
