"""The first step after an idle GPU vs the steady steps: per-kernel HIP-event
durations (pss_timing) and the step span, to separate host planning from
slower first kernels.  GPU box.  usage: tools/first_step.py [c4|c3|n256]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import psrsigsim_amd as pss
from psrsigsim_amd import _lib
import bench

w = sys.argv[1] if len(sys.argv) > 1 else "c4"
if w == "c4":
    step = lambda: bench.c4_step(pss, 2048, None, False)
elif w == "n256":
    step = lambda: bench.c3_step(pss, 256, None, 22)
else:
    step = lambda: bench.c3_step(pss, 2048, None, 22)
L = _lib.load()
for _ in range(3):
    s = step()
    del s
torch.cuda.synchronize()
L.pss_timing_enable(1)
_lib.timing_collect()
for rep in range(3):
    torch.cuda.synchronize()
    time.sleep(0.05)                       # the GPU idles, as between the warm-up and the timed region
    e = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    t0 = time.perf_counter()
    e[0].record()
    for i in range(5):
        s = step()
        e[i + 1].record()
        del s
    torch.cuda.synchronize()
    spans = [e[i].elapsed_time(e[i + 1]) for i in range(5)]
    ks = {}
    for kind, ms, u in _lib.timing_collect():
        ks.setdefault(kind, []).append(round(ms, 3))
    print("rep %d step spans %s" % (rep, [round(x, 3) for x in spans]), flush=True)
    for kind, v in ks.items():
        print("   %-16s %s" % (kind, v[:12]), flush=True)
L.pss_timing_enable(0)
