#!/bin/bash
# Compile one launch unit for gfx950 and list VGPRs / occupancy / scratch per kernel.
# usage: tools/vgprs.sh [UNIT] [extra hipcc flags]   (UNIT default pss_fourstep.hip: the C3 kernels)
U=${1:-pss_fourstep.hip}; shift
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -ffp-contract=on -c \
  -I/root/repo/include /root/repo/psrsigsim_amd/csrc/$U -o /tmp/vg.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | \
python3 -c '
import sys, re
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1); info = {}; continue
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        info[m.group(1).split()[0]] = m.group(2)
        if m.group(1).startswith("LDS"):
            n = re.sub(r"I\d+(Pair|Rows|Cols|SinglePass)", r"<\1", cur)
            n = re.sub(r"EN3pss5RList.*", "", n)
            print("%-60s vgpr %4s occ %s scratch %s lds %s" % (n[:60], info.get("VGPRs"), info.get("Occupancy"), info.get("ScratchSize"), info.get("LDS")))
'
