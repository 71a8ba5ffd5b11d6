"""Diagnostic: host-side timeline of the C3 step (which API call blocks)."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import psrsigsim_amd as pss
    from psrsigsim_amd import _engine
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    nchan = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    pss.seed(1)
    orig = _engine.null_shift_device

    def probe(*a, **k):
        t = time.perf_counter()
        r = orig(*a, **k)
        print("    probe %.2f ms" % ((time.perf_counter() - t) * 1e3))
        return r
    _engine.null_shift_device = probe
    import psrsigsim_amd.pulsar.pulsar as PP
    PP._engine.null_shift_device = probe
    ms = torch.cuda.Stream() if os.environ.get("MAIN_STREAM") else None
    if ms is not None:
        torch.cuda.set_stream(ms)
    for step in range(5):
        t = [time.perf_counter()]
        sig = FilterBankSignal(1400, 400, Nsubband=nchan, fold=False)
        psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
        ism = ISM()
        ism.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
        t.append(time.perf_counter())
        psr.make_pulses(sig, tobs=(1 << 22) * 20.48e-6)
        t.append(time.perf_counter())
        ism.disperse(sig, 100)
        t.append(time.perf_counter())
        psr.null(sig, 0.1)
        t.append(time.perf_counter())
        T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
        t.append(time.perf_counter())
        del sig
        names = ["setup+scatter", "make_pulses", "disperse", "null", "observe"]
        print("step", step, " ".join("%s %.2f" % (n, (b - a) * 1e3) for n, a, b in zip(names, t, t[1:])))
    torch.cuda.synchronize()




def profile_step():
    """cProfile of one steady-state step (after two warm-up steps)."""
    import cProfile
    import pstats
    import torch
    sys.argv = sys.argv[:1]
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T

    def step():
        sig = FilterBankSignal(1400, 400, Nsubband=2048, fold=False)
        psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
        ism = ISM()
        ism.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
        psr.make_pulses(sig, tobs=(1 << 22) * 20.48e-6)
        ism.disperse(sig, 100)
        psr.null(sig, 0.1)
        T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
        del sig
    pss.seed(1)
    step()
    step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "prof":
        profile_step()
    else:
        main()
