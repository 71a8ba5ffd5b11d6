"""Fast-vs-generic bitwise check over a small grid of options (diagnostic:
which stage makes the two paths differ).  Usage: python tools/diag_fast.py"""
import sys
import numpy as np


def run(nchan, log2n, null, noise, dm, scatter=False):
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    pss.seed(11)
    sig = FilterBankSignal(1400, 400, Nsubband=nchan, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, tobs=(1 << log2n) * 20.48e-6)
    ISM().disperse(sig, dm)
    if null:
        psr.null(sig, 0.2)
    if noise:
        T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
    return sig.data.cpu().numpy()


def main():
    from psrsigsim_amd import _lib
    L = _lib.lib()
    cases = [(3, 16, True, True), (3, 16, True, False), (3, 16, False, True), (3, 16, False, False),
             (2, 16, True, True), (4, 16, True, True), (3, 15, True, True), (3, 17, True, True),
             (3, 14, True, True)]
    for nchan, log2n, null, noise in cases:
        fast = run(nchan, log2n, null, noise, 100)
        fast2 = run(nchan, log2n, null, noise, 100)
        old = L.pss_set_flags(_lib.FLAG_NO_FAST)
        try:
            gen = run(nchan, log2n, null, noise, 100)
            gen2 = run(nchan, log2n, null, noise, 100)
        finally:
            L.pss_set_flags(old)
        d = fast != gen
        rows = [int(x) for x in d.sum(axis=1)]
        first = np.argwhere(d)[:3].tolist()
        print("nchan=%d log2n=%d null=%d noise=%d: fast/fast %d gen/gen %d fast/gen %d rows %s first %s maxabs %.3g"
              % (nchan, log2n, null, noise, int((fast != fast2).sum()), int((gen != gen2).sum()), int(d.sum()),
                 rows, first, float(np.abs(fast - gen).max())), flush=True)


if __name__ == "__main__":
    sys.exit(main())
