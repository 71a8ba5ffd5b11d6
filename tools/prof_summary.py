#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace (csv): per kernel name and grid shape,
launch count and average/min/max duration.  Separates the full-size launches
(grid rows = channels) from the 1-row probe / shadow launches.

usage: tools/prof_summary.py run_kernel_trace.csv [> summary.md]"""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(list)
    meta = {}
    for r in rows:
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "")
        if "<" in short:
            short = short.split("<")[0] + "<" + short.split("<", 1)[1][:60]
        gy = int(r["Grid_Size_Y"])
        key = (short, gy, int(r["Grid_Size_X"]))
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        meta[key] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Workgroup_Size_X"])
    print("| kernel | grid (x, y) | launches | avg ms | min ms | max ms | VGPR | SGPR | LDS B | WG |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for key in sorted(agg, key=lambda k: -sum(agg[k])):
        d = agg[key]
        v, s, l, w = meta[key]
        print("| %s | (%d, %d) | %d | %.4f | %.4f | %.4f | %s | %s | %s | %s |"
              % (key[0], key[2], key[1], len(d), sum(d) / len(d), min(d), max(d), v, s, l, w))


if __name__ == "__main__":
    main(sys.argv[1])
