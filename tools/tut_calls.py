"""Host time per API call of the tutorial-shape steps (bench --workload t1 /
t2) in the steady state, no sync between steps: a call whose time tracks the
kernels' is blocking on the GPU.  GPU box.  usage: tools/tut_calls.py t1|t2 [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import psrsigsim_amd as pss  # noqa: F401
from psrsigsim_amd.signal import FilterBankSignal
from psrsigsim_amd.pulsar import Pulsar, GaussProfile
from psrsigsim_amd.ism import ISM
from psrsigsim_amd.telescope import telescope as T

WL = sys.argv[1] if len(sys.argv) > 1 else "t1"
STEPS = int(sys.argv[2]) if len(sys.argv) > 2 else 40
names = ["signal", "pulsar", "make_pulses", "disperse", "telescope", "observe", "del"]


def step(t):
    t.append(time.perf_counter())
    prof = GaussProfile(peak=0.5, width=0.05, amp=1.0)
    if WL == "t1":
        sig = FilterBankSignal(820, 200.0, Nsubband=128, fold=False)
        t.append(time.perf_counter())
        psr = Pulsar(1.0, 10.0, profiles=prof, name="J0000+0000")
        t.append(time.perf_counter())
        psr.make_pulses(sig, tobs=2.0)
        sysname = "820_GUPPI"
    else:
        sig = FilterBankSignal(1500, 800.0, Nsubband=64, sample_rate=(1.0 / 0.010) * 2048 * 10 ** -6,
                               sublen=60.0, fold=True)
        t.append(time.perf_counter())
        psr = Pulsar(0.010, 0.005, profiles=prof, name="J0000+0000", specidx=-1.6, ref_freq=1400.0)
        t.append(time.perf_counter())
        psr.make_pulses(sig, tobs=60.0 * 20)
        sysname = "Lband_GUPPI"
    t.append(time.perf_counter())
    ISM().disperse(sig, 40.0)
    t.append(time.perf_counter())
    tel = T.GBT()
    t.append(time.perf_counter())
    tel.observe(sig, psr, system=sysname, noise=True)
    t.append(time.perf_counter())
    del sig
    t.append(time.perf_counter())


for _ in range(3):
    step([])
torch.cuda.synchronize()
rows = []
ev0 = torch.cuda.Event(enable_timing=True)
ev1 = torch.cuda.Event(enable_timing=True)
ev0.record()
t0 = time.perf_counter()
for _ in range(STEPS):
    t = []
    step(t)
    rows.append(np.diff(t) * 1e3)
t_host = time.perf_counter() - t0
ev1.record()
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
rows = np.array(rows)
print("%s: host loop %.3f ms/step, with final sync %.3f ms/step, GPU span %.3f ms/step"
      % (WL, t_host / STEPS * 1e3, t_all / STEPS * 1e3, ev0.elapsed_time(ev1) / STEPS))
for i, n in enumerate(names):
    print("  %-12s median %.3f  max %.3f ms" % (n, np.median(rows[:, i]), rows[:, i].max()))
