"""Cost of the float64 null-decision refine (k_box_row,
k_tw64, k_null_bspec, k_row_absmax, k_null_refine) on the packed fallback
paths with a delayed null: C4's fold-mode geometry (2048 x 30720, DM 13.3,
null 0.1 -> Bluestein) and a search-mode length at the refine limit
(64 x (2^17 - 2)).  Run under rocprofv3 --kernel-trace --stats
(tools/r5_refine.sh); prints the wall time per run.  GPU box."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import psrsigsim_amd as pss
import bench
from psrsigsim_amd.signal import FilterBankSignal
from psrsigsim_amd.pulsar import Pulsar, GaussProfile, DataProfile
from psrsigsim_amd.ism import ISM
from psrsigsim_amd.telescope import telescope as T


def c4_null():
    sig = FilterBankSignal(1400, 400, Nsubband=2048, sample_rate=bench.F0_B1855 * 1024 * 1e-6, sublen=60.0,
                           fold=True)
    psr = Pulsar(1.0 / bench.F0_B1855, 0.005, profiles=DataProfile(bench.b1855_profile(), Nchan=2048))
    psr.make_pulses(sig, tobs=1800.0)
    ISM().disperse(sig, 13.299393)
    psr.null(sig, 0.1)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
    return sig


def search_null(n=(1 << 17) - 2, nch=64):
    sig = FilterBankSignal(1400, 400, Nsubband=nch, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, tobs=(n + 0.5) * bench.TOBS_PER_SAMPLE)
    ISM().disperse(sig, 30)
    psr.null(sig, 0.1)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
    return sig


pss.seed(3)
for name, fn in (("c4_null 2048 x 30720", c4_null), ("search_null 64 x 131070", search_null)):
    for _ in range(2):
        fn().data
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        s = fn()
        s.data
    torch.cuda.synchronize()
    print("%s: %.3f ms per run (5 runs after 2 warm-up; n = %d)" % (name, (time.perf_counter() - t) / 5 * 1e3,
                                                                     s._ncols), flush=True)
