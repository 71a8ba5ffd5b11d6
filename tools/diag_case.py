#!/usr/bin/env python
"""Diagnostic: run a C3-like case staged through the GPU and the oracle and
print, per stage, the normwise error, the location of the max error and the
reference value there."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import replay  # noqa: E402
from tests.test_gpu_parity import _big_case  # noqa: E402

rec = []
orig = replay._err


def err(gpu, ref, exclude=None):
    e = orig(gpu, ref, exclude)
    g = np.asarray(gpu, dtype=np.float64)
    r = np.asarray(ref, dtype=np.float64)
    if g.shape == r.shape:
        d = np.abs(g - r)
        i = np.unravel_index(np.argmax(d), d.shape)
        rec.append((e, i, float(r[i]), float(g[i]), float(np.max(np.abs(r))),
                    float(np.sqrt(np.mean(d ** 2)) / np.sqrt(np.mean(r ** 2)))))
    return e


replay._err = err
log2n, nchan = int(sys.argv[1]), int(sys.argv[2])
null = len(sys.argv) < 4 or sys.argv[3] != "nonull"
out = replay.run_case(None, fused=False, case=_big_case(log2n, nchan, null=null), seed=log2n)
for (k, v), r in zip(out.items(), rec):
    print("%-9s err %.3e  at %s ref %.5g gpu %.5g  max|ref| %.4g  rel-rms %.2e" % (k, v, r[1], r[2], r[3], r[4], r[5]))
