#!/usr/bin/env python
"""Summarise rocprofv3 --pmc counter_collection CSVs (one or more passes):
per kernel (short name, grid size), the average of every counter.

usage: tools/pmc_summary.py DIR [DIR...]   (each DIR holds run_counter_collection.csv)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    s = name.split("(")[0].replace("void ", "")
    return s.split("<")[0]


def main(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                key = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
                acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta[key] = (r["VGPR_Count"], r["LDS_Block_Size"], r["Workgroup_Size"])
    for key in sorted(acc, key=lambda k: -k[1]):
        c = acc[key]
        v = {n: sum(x) / len(x) for n, x in c.items()}
        print("%s grid=%d VGPR=%s LDS=%s WG=%s" % (key + meta[key]))
        for n in sorted(v):
            print("    %-24s %.4g" % (n, v[n]))


if __name__ == "__main__":
    main(sys.argv[1:])
