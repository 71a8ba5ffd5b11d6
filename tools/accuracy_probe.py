#!/usr/bin/env python
"""Accuracy diagnostic: fp32 device shift_t vs float64 oracle on pulsar-like
(profile x chi2) rows and on uniform rows, several N; prints normwise max
error and relative RMS error.  PSS_LIB_PATH selects the library build."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import pss_cpu as O  # noqa: E402
from psrsigsim_amd.utils import shift_t  # noqa: E402


def rows(kind, N, R, rng):
    if kind == "uniform":
        return rng.random((R, N))
    ph = (np.arange(N) / 244.140625) % 1
    prof = np.exp(-0.5 * ((ph - 0.5) / 0.05) ** 2)
    return prof[None, :] * rng.chisquare(1, (R, N))


rng = np.random.default_rng(0)
for N in [1 << 13, 1 << 16, 1 << 17, 1 << 20, 1 << 22]:
    for kind in ("uniform", "pulsar"):
        R = 2
        x = rows(kind, N, R, rng).astype(np.float32)
        s = np.array([13567.3, -2345.77])
        g = shift_t(x, s, dt=1.0)
        errs = []
        for r in range(R):
            ref = O.shift_t(x[r].astype(np.float64), float(s[r]), dt=1.0)
            d = g[r] - ref
            errs.append((np.max(np.abs(d)) / np.max(np.abs(ref)), np.sqrt(np.mean(d * d) / np.mean(ref * ref))))
        print("N=2^%d %-8s normwise %.2e  rms %.2e" % (int(np.log2(N)), kind, max(e[0] for e in errs),
                                                      max(e[1] for e in errs)))
