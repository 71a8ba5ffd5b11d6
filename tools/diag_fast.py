"""Diagnostic: where do the fast-path kernels differ from the generic ones?"""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(nchan, log2n, null, noise=True):
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    pss.seed(11)
    sig = FilterBankSignal(1400, 400, Nsubband=nchan, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, tobs=(1 << log2n) * 20.48e-6)
    ISM().disperse(sig, 100)
    if null:
        psr.null(sig, 0.2)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=noise)
    return sig.data.cpu().numpy()


def main():
    from psrsigsim_amd import _lib
    L = _lib.lib()
    for (nchan, log2n, null, noise) in [(3, 16, False, False), (3, 16, False, True), (3, 16, True, True)]:
        fast = run(nchan, log2n, null, noise)
        old = L.pss_set_flags(_lib.FLAG_NO_FAST)
        gen = run(nchan, log2n, null, noise)
        L.pss_set_flags(old)
        bad = np.argwhere(fast != gen)
        print("case", nchan, log2n, null, noise, "mismatch", len(bad), "of", fast.size)
        if len(bad):
            N = fast.shape[1]
            N2 = 4096 if log2n == 16 else 8192
            ch, n = bad[:, 0], bad[:, 1]
            print("  channels", np.unique(ch), "n2 blocks(512)", np.unique((n % N2) // 512)[:20],
                  "n1", np.unique(n // N2)[:20])
            i = bad[0]
            print("  first", i, fast[tuple(i)], gen[tuple(i)], "rel", np.max(np.abs(fast - gen)) / np.max(np.abs(gen)))


if __name__ == "__main__":
    main()
