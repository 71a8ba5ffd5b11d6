"""Host time of each API call of the C3 step (bench.c3_step's sequence) on
an idle GPU -- the first timed step's exposed planning, call by call.
GPU box.  usage: tools/host_calls.py [nchan ...]"""
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


names = ["construct", "scatter_broaden", "make_pulses", "disperse", "null", "observe(launch)"]
for nch in [int(a) for a in sys.argv[1:]] or [256, 2048]:
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
