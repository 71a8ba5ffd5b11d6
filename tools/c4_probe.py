"""C4-shaped fold-mode run (2048 ch x 30 subints x 1024 bins = 30720 samples
per channel, DM 13.3, radiometer noise) with a Gaussian portrait: timing of
the non-power-of-two path."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(nchan):
    import torch
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    F0 = 186.4940812499314404
    sig = FilterBankSignal(1400, 400, Nsubband=nchan, sample_rate=F0 * 1024 * 1e-6, sublen=60.0, fold=True)
    psr = Pulsar(1.0 / F0, 0.005, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, tobs=1800.0)
    ISM().disperse(sig, 13.299393)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
    d = sig.data
    torch.cuda.synchronize()
    return d.shape


def main():
    import torch
    nchan = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    print("shape", run(nchan))
    for _ in range(2):
        t = time.perf_counter()
        run(nchan)
        print("nchan %d: %.1f ms" % (nchan, (time.perf_counter() - t) * 1e3), flush=True)


if __name__ == "__main__":
    main()
