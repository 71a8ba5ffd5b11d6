"""Where the host blocks in the steady state (no sync between steps): per
API call of the C3 step, the time of each call over consecutive steps, the
calls whose time exceeds their median by > 2 ms listed.  GPU box.
usage: tools/host_stalls.py [nchan] [steps]"""
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

NCH = int(sys.argv[1]) if len(sys.argv) > 1 else 256
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 40
names = ["construct", "scatter", "make_pulses", "disperse", "null", "observe", "del"]


def step(t):
    t.append(time.perf_counter())
    sig = FilterBankSignal(1400, 400, Nsubband=NCH, fold=False)
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
    del sig
    t.append(time.perf_counter())


for _ in range(3):
    step([])
torch.cuda.synchronize()
rows = []
for _ in range(STEPS):
    t = []
    step(t)
    rows.append(np.diff(t) * 1e3)
torch.cuda.synchronize()
a = np.array(rows)
med = np.median(a, axis=0)
print("median ms per call:", ", ".join("%s %.2f" % (n, v) for n, v in zip(names, med)))
for i, r in enumerate(a):
    slow = [(names[j], round(float(r[j]), 2)) for j in range(len(names)) if r[j] > med[j] + 2.0]
    if slow:
        print("step %2d: %s" % (i, slow))
