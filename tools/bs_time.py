"""Timing of the fallback transforms: shift_t (one fused FFT-delay run) on
device-resident rows at lengths that take the Bluestein path, next to the
power-of-two four-step and the O(N^2) direct DFT where it finishes."""
import sys
import time
import numpy as np
import torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from psrsigsim_amd import _lib
from psrsigsim_amd.utils import shift_t


def run(R, N, reps=3, direct=False):
    x = torch.rand((R, N), device="cuda")
    s = np.linspace(0.3, 1234.5, R)
    L = _lib.load()
    old = L.pss_set_flags(_lib.FLAG_DIRECT_DFT if direct else 0)
    try:
        shift_t(x, s, dt=1.0)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            shift_t(x, s, dt=1.0)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / reps
    finally:
        L.pss_set_flags(old)
    print("R=%5d N=%9d %-9s %8.3f ms  %.3g ch-samp/s" % (R, N, "direct" if direct else "", dt * 1e3, R * N / dt),
          flush=True)


run(64, 3125000)              # reference simulate fixture geometry (Bluestein, M = 2^23)
run(2048, 30720)              # C4 length (Bluestein when a delayed null forces the fallback)
run(512, 1 << 20)             # power-of-two four-step, for scale
run(512, (1 << 20) - 2)       # Bluestein at the same size
run(16, 30720, reps=1, direct=True)   # O(N^2) direct DFT at the C4 length
