"""Infinity-Cache residency with the real kernels: the
C3 pipeline without its null (pulses, disperse(100), Arecibo noise; the
four-step pass A -> row -> pass C at 1024 x 4096) run on `nchan`-channel
signals, so one run's pair spill is nchan/2 x 32 MiB -- 128 MiB at 8
channels, L3-resident, against 32 GiB at 2048.  Prints per-kernel ms scaled
to 2048 channels (HIP events on the launch stream).  GPU box.
usage: tools/l3_real.py nchan [nchan ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import psrsigsim_amd as pss
from psrsigsim_amd import _lib
from psrsigsim_amd.signal import FilterBankSignal
from psrsigsim_amd.pulsar import Pulsar, GaussProfile
from psrsigsim_amd.ism import ISM
from psrsigsim_amd.telescope import telescope as T

N = 1 << 22


def step(nch):
    sig = FilterBankSignal(1400, 400, Nsubband=2048, fold=False, shard=(0, nch))
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, tobs=N * 20.48e-6)
    ISM().disperse(sig, 100)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
    return sig


pss.seed(3)
for nch in [int(a) for a in sys.argv[1:]] or [8, 16, 32, 2048]:
    reps = max(3, min(200, 4096 // nch))
    for _ in range(2):
        s = step(nch)
        del s
    torch.cuda.synchronize()
    _lib.load().pss_timing_enable(1)
    _lib.timing_collect()
    t0 = time.perf_counter()
    for _ in range(reps):
        s = step(nch)
        del s
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    _lib.load().pss_timing_enable(0)
    agg = {}
    for k, ms, u in _lib.timing_collect():
        if u == nch * N:
            agg[k] = agg.get(k, 0.0) + ms / reps
    sc = 2048.0 / nch
    print("nchan %5d spill %7.0f MiB  reps %3d  wall %.3f ms  kernels x%.0f: %s  sum %.2f" % (
        nch, nch / 2 * 32, reps, dt * 1e3, sc, {k: round(v * sc, 2) for k, v in agg.items()},
        sum(agg.values()) * sc), flush=True)
