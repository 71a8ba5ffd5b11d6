"""Where the first timed step's extra time goes: for a step issued on an idle
GPU and for the steady steps after it, the stream span (HIP events), the host
return time and the sum of the step's own kernel durations (pss timing
events).  GPU box only.  usage: tools/first_step.py [nchan] [reps] [heat]
heat: none | sleep (a one-wave spin kernel on a side stream while the first
step's host planning runs) | copy (16-GB device copies on a side stream):
tells a clock / power-state ramp from other first-step costs."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import psrsigsim_amd as pss
from psrsigsim_amd import _lib
import bench

NCH = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 3
STEPS = 5
HEAT = sys.argv[3] if len(sys.argv) > 3 else "none"
side = torch.cuda.Stream()
if HEAT == "copy":
    buf_a = torch.empty(1 << 31, dtype=torch.float32, device="cuda")
    buf_b = torch.empty_like(buf_a)
for _ in range(2):
    s = bench.c3_step(pss, NCH, None, 22)
    del s
torch.cuda.synchronize()
L = _lib.load()
for rep in range(REPS):
    L.pss_timing_enable(1)
    _lib.timing_collect()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(STEPS + 1)]
    for e in evs:
        e.record()
    torch.cuda.synchronize()
    time.sleep(0.05)
    t0 = time.perf_counter()
    evs[0].record()
    if HEAT == "sleep":
        with torch.cuda.stream(side):
            torch.cuda._sleep(20_000_000)
    elif HEAT == "copy":
        with torch.cuda.stream(side):
            for _ in range(4):
                buf_b.copy_(buf_a)
    host = []
    for i in range(STEPS):
        t = time.perf_counter()
        s = bench.c3_step(pss, NCH, None, 22)
        del s
        evs[i + 1].record()
        host.append((time.perf_counter() - t) * 1e3)
    torch.cuda.synchronize()
    L.pss_timing_enable(0)
    launches = _lib.timing_collect()
    per = len(launches) // STEPS
    spans = [a.elapsed_time(b) for a, b in zip(evs, evs[1:])]
    for i in range(STEPS):
        ks = launches[i * per:(i + 1) * per]
        ksum = sum(ms for _, ms, _ in ks)
        big = " ".join("%s %.2f" % (k, ms) for k, ms, _ in ks if ms > 0.5)
        print("%s rep %d step %d span %.2f host %.2f kernels %.2f gap %.2f | %s"
              % (HEAT, rep, i, spans[i], host[i], ksum, spans[i] - ksum, big))
