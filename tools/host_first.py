"""Host work of one C3 step issued on an idle GPU (the first timed step's
critical path): wall time and cProfile of the API calls.  GPU box only.
usage: tools/host_first.py [nchan]"""
import cProfile
import os
import pstats
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import psrsigsim_amd as pss
import bench

NCH = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
for _ in range(2):
    s = bench.c3_step(pss, NCH, None, 22)
    s.data
    del s
torch.cuda.synchronize()
for _ in range(2):
    t = time.perf_counter()
    s = bench.c3_step(pss, NCH, None, 22)
    print("host %.2f ms" % ((time.perf_counter() - t) * 1e3))
    torch.cuda.synchronize()
    del s
pr = cProfile.Profile()
pr.enable()
s = bench.c3_step(pss, NCH, None, 22)
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("cumtime").print_stats(30)
pstats.Stats(pr).sort_stats("tottime").print_stats(40)
