"""Diagnostic: Bluestein fallback error per M1 (shift_t vs the float64 oracle)."""
import sys
import numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from oracle import pss_cpu as O
from psrsigsim_amd.utils import shift_t

for N in [int(a) for a in sys.argv[1:]]:
    x = np.random.default_rng(N).random((1, N)).astype(np.float32)
    got = shift_t(x, np.array([0.37]), dt=1.0)
    ref = O.shift_t(x[0].astype(np.float64), 0.37, dt=1.0)
    M = 1
    while M < 2 * N - 1:
        M <<= 1
    print(N, "M=2^%d" % (M.bit_length() - 1), "err %.3g" % (np.max(np.abs(got[0] - ref)) / np.max(np.abs(ref))), flush=True)
