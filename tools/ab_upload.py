"""Same-process A/B of _engine.UPLOAD_MODE (table uploads on the launch
stream, on an upload stream, or direct when the launch stream is idle) on
bench-style timed regions (barrier, 20 steps, sync), alternating modes.
GPU box.  usage: tools/ab_upload.py [c4|n256] [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import psrsigsim_amd as pss
from psrsigsim_amd import _engine
import bench

w = sys.argv[1] if len(sys.argv) > 1 else "c4"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
step = (lambda: bench.c4_step(pss, 2048, None, False)) if w == "c4" else (lambda: bench.c3_step(pss, 256, None, 22))
res = {}
for r in range(rounds):
    for mode in ("direct", "stream", "auto"):
        _engine.UPLOAD_MODE = mode
        for _ in range(2):
            s = step()
            del s
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            s = step()
            if w == "c4":
                _ = s.data
            del s
        torch.cuda.synchronize()
        res.setdefault(mode, []).append((time.perf_counter() - t0) / 20 * 1e3)
for mode, v in res.items():
    print("%s %-6s ms/step %s  median %.3f" % (w, mode, [round(x, 3) for x in v], float(np.median(v))), flush=True)
