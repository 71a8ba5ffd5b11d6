"""Diagnostic: fast vs generic kernels (and run-to-run determinism) per row
for a few search-mode configurations.  GPU only; prints one line per case."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def run(nchan, log2n, null, dm, prof_kind, flags=None):
    import psrsigsim_amd as pss
    from psrsigsim_amd import _lib
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile, DataProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    L = _lib.lib()
    old = L.pss_set_flags(flags) if flags is not None else None
    try:
        pss.seed(11)
        sig = FilterBankSignal(1400, 400, Nsubband=nchan, fold=False)
        if prof_kind == "gauss":
            prof = GaussProfile(0.5, 0.05, 1)
        else:
            x = np.linspace(0, 1, 256)
            prof = DataProfile(np.exp(-0.5 * ((x - 0.5) / 0.05) ** 2), Nchan=nchan)
        psr = Pulsar(0.005, 1.0, profiles=prof)
        psr.make_pulses(sig, tobs=(1 << log2n) * 20.48e-6)
        if dm:
            ISM().disperse(sig, dm)
        if null:
            psr.null(sig, 0.2)
        T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
        return sig.data.cpu().numpy()
    finally:
        if old is not None:
            L.pss_set_flags(old)


def rows(a, b):
    return " ".join("%.3f" % np.mean(a[r] != b[r]) for r in range(a.shape[0]))


def main():
    from psrsigsim_amd import _lib
    cases = [(3, 22, True, 100, "gauss"), (3, 22, False, 100, "gauss"), (2, 22, True, 100, "gauss"),
             (4, 22, True, 100, "gauss"), (3, 22, True, 100, "data"), (3, 22, True, 0, "gauss"),
             (3, 20, True, 100, "gauss"), (3, 18, True, 100, "gauss")]
    for c in cases:
        f1 = run(*c)
        f2 = run(*c)
        g1 = run(*c, flags=_lib.FLAG_NO_FAST)
        g2 = run(*c, flags=_lib.FLAG_NO_FAST)
        print(c, "fast-fast", rows(f1, f2), "| gen-gen", rows(g1, g2), "| fast-gen", rows(f1, g1), flush=True)


if __name__ == "__main__":
    sys.exit(main())
