#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace (csv): per kernel name and grid shape,
launch count and average/min/max duration.  Separates the full-size launches
(grid rows = channels) from the 1-row probe / shadow launches.

With --json OUT it also writes, per C3 kernel kind (bench.py's names), the
average duration of its full-size launches (the largest grid of that kernel
in the trace: the band's run, not the channel-0 probe) -- the per-launch
figure bench.py reports as roofline.frac_profile next to its own HIP-event
timing.

usage: tools/prof_summary.py run_kernel_trace.csv [--json OUT] [> summary.md]"""
import csv
import json
import sys
from collections import defaultdict

KIND = {"k_pairA_fast": "fourstep_colA", "k_pair_row": "fourstep_row",
        "k_pairC_fast": "fourstep_colC", "k_null_fix_list": "null_fix"}


def full_launches(rows):
    """kind -> (avg ms, launches, grid) over the largest-grid launches."""
    by = defaultdict(list)
    for r in rows:
        base = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        k = KIND.get(base)
        if k is None:
            continue
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r.get("Grid_Size_Z", 1) or 1)
        by[k].append((g, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    out = {}
    for k, v in by.items():
        gmax = max(g for g, _ in v)
        d = [ms for g, ms in v if g == gmax]
        out[k] = {"avg_ms": round(sum(d) / len(d), 4), "launches": len(d), "grid_size": gmax}
    return out


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
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(full_launches(list(csv.DictReader(open(sys.argv[1])))), f, indent=1)
