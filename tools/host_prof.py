"""Host-side profile (cProfile) of a bench workload step on the GPU box:
where the non-kernel time of a step goes.  usage: tools/host_prof.py c4|c3|t1|t2 [steps]"""
import cProfile
import pstats
import sys
import time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch
import psrsigsim_amd as pss
import bench

wl = sys.argv[1] if len(sys.argv) > 1 else "c4"
step = {"c4": lambda: bench.c4_step(pss, 2048, None, False),
        "c3": lambda: bench.c3_step(pss, 2048, None, 22),
        "t1": lambda: bench.tutorial_step(pss, "t1", 128, None),
        "t2": lambda: bench.tutorial_step(pss, "t2", 64, None)}[wl]
for _ in range(2):
    s = step()
    s.data
torch.cuda.synchronize()
pr = cProfile.Profile()
t = time.perf_counter()
pr.enable()
N = int(sys.argv[2]) if len(sys.argv) > 2 else 5
for _ in range(N):
    s = step()
    if wl != "c3":
        s.data
torch.cuda.synchronize()
pr.disable()
print("ms/step %.2f (under cProfile)" % ((time.perf_counter() - t) / N * 1e3))
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
pstats.Stats(pr).sort_stats("cumtime").print_stats(30)
