"""Same-process A/B of engine variants selectable through pss_set_flags
(placement choices that must stay bitwise neutral), on the C3 step of
bench.py: the variants alternate step by step so clock and power drift hit
them alike.  Prints per variant the median step span (HIP events on the
launch stream), the mean kernel ms per kind and the wall time per step.
GPU box.  usage: tools/ab_flags.py FLAGS_A FLAGS_B [...] [--steps K] [--nchan C]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import psrsigsim_amd as pss
from psrsigsim_amd import _lib
import bench

ap = argparse.ArgumentParser()
ap.add_argument("flags", nargs="+", type=lambda s: int(s, 0))
ap.add_argument("--steps", type=int, default=12)
ap.add_argument("--nchan", type=int, default=2048)
ap.add_argument("--workload", default="c3", choices=("c3", "c5"))
a = ap.parse_args()
L = _lib.lib()
pss.seed(1776)
step = (lambda: bench.c3_step(pss, a.nchan, (0, a.nchan), 22)) if a.workload == "c3" else \
    (lambda: bench.c5_step(pss, a.nchan, (0, a.nchan), 24))
res = {f: {"span": [], "k": {}, "wall": []} for f in a.flags}
for f in a.flags:                          # warm-up of every variant
    L.pss_set_flags(f)
    for _ in range(2):
        s = step()
        del s
torch.cuda.synchronize()
L.pss_timing_enable(1)
for i in range(a.steps):
    for f in a.flags:
        L.pss_set_flags(f)
        _lib.timing_collect()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        s = step()
        del s
        e1.record()
        torch.cuda.synchronize()
        res[f]["wall"].append(time.perf_counter() - t0)
        res[f]["span"].append(e0.elapsed_time(e1))
        for k, ms, u in _lib.timing_collect():
            if u == a.nchan * (1 << (22 if a.workload == "c3" else 24)):
                res[f]["k"].setdefault(k, []).append(ms)
L.pss_timing_enable(0)
L.pss_set_flags(0)
for f in a.flags:
    r = res[f]
    ks = {k: round(float(np.mean(v)), 3) for k, v in r["k"].items()}
    print("flags 0x%x: span median %.3f ms (min %.3f)  wall %.3f ms  kernels %s  sum %.3f" % (
        f, float(np.median(r["span"])), float(np.min(r["span"])), float(np.median(r["wall"])) * 1e3, ks,
        sum(ks.values())), flush=True)
