"""Host time of each API call of the C3 step (bench.c3_step's sequence) on
an idle GPU -- the first timed step's exposed planning, call by call.
GPU box.  usage: tools/host_calls.py [c4] [nchan ...]   (c4: bench.c4_step's sequence)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import psrsigsim_amd as pss
import bench
from psrsigsim_amd.signal import FilterBankSignal
from psrsigsim_amd.pulsar import Pulsar, GaussProfile
from psrsigsim_amd.ism import ISM
from psrsigsim_amd.telescope import telescope as T


def step(nch, t):
    t.append(time.perf_counter())
    sig = FilterBankSignal(1400, 400, Nsubband=nch, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    ism = ISM()
    t.append(time.perf_counter())
    ism.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    t.append(time.perf_counter())
    psr.make_pulses(sig, tobs=(1 << 22) * bench.TOBS_PER_SAMPLE)
    t.append(time.perf_counter())
    ism.disperse(sig, 100)
    t.append(time.perf_counter())
    psr.null(sig, 0.1)
    t.append(time.perf_counter())
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True, ret_resampsig=False)
    t.append(time.perf_counter())
    return sig


def step_c4(nch, t):
    from psrsigsim_amd.pulsar import DataProfile
    t.append(time.perf_counter())
    sig = FilterBankSignal(1400, 400, Nsubband=nch, sample_rate=bench.F0_B1855 * 1024 * 1e-6, sublen=60.0,
                           fold=True)
    psr = Pulsar(1.0 / bench.F0_B1855, 0.005, profiles=DataProfile(bench.b1855_profile(), Nchan=nch))
    t.append(time.perf_counter())
    t.append(time.perf_counter())
    psr.make_pulses(sig, tobs=1800.0)
    t.append(time.perf_counter())
    ISM().disperse(sig, 13.299393)
    t.append(time.perf_counter())
    t.append(time.perf_counter())
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
    t.append(time.perf_counter())
    return sig


names = ["construct", "scatter_broaden", "make_pulses", "disperse", "null", "observe(launch)"]
args = sys.argv[1:]
if args and args[0] == "c4":
    step = step_c4
    args = args[1:]
for nch in [int(a) for a in args] or [256, 2048]:
    for _ in range(2):
        step(nch, [])
    torch.cuda.synchronize()
    rows = []
    for _ in range(5):
        t = []
        s = step(nch, t)
        rows.append(np.diff(t) * 1e3)
        torch.cuda.synchronize()
        del s
    m = np.median(np.array(rows), axis=0)
    print("nchan %5d host %.2f ms: %s" % (nch, m.sum(), ", ".join("%s %.2f" % (n, v) for n, v in zip(names, m))),
          flush=True)
