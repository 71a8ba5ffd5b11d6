"""observe()'s resampling branches (telescope.py:108-125) with the fused K3
epilogue: the run's epilogue sums the pre-noise samples into float64 window
sums and one small kernel divides, clips and casts (PssPipeline.out_len).
Times a search-mode signal (GaussProfile, disperse) observed with a backend
sampling `factor` times slower than the signal -- the down_sample branch for
an integer factor, rebin otherwise -- against the same run with no returned
copy (ret_resampsig=False), and prints the kernel trace of one run.  GPU box.
usage: tools/k3_bench.py [nchan] [log2n] [factor ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import psrsigsim_amd as pss
from psrsigsim_amd import _lib
from psrsigsim_amd.signal import FilterBankSignal
from psrsigsim_amd.pulsar import Pulsar, GaussProfile
from psrsigsim_amd.ism import ISM
from psrsigsim_amd.telescope import Telescope, Receiver, Backend
from psrsigsim_amd._units import Quantity

NCH = int(sys.argv[1]) if len(sys.argv) > 1 else 512
LOG2N = int(sys.argv[2]) if len(sys.argv) > 2 else 20
FACTORS = [float(a) for a in sys.argv[3:]] or [1.0, 8.0, 7.3]
DT = 20.48e-6


def staged_observe(tel, sig, psr, system):
    """The round-4 staged form of the same branch, for the A/B: the run
    writes a full-resolution fp32 pre-noise copy, then pss_down_sample /
    pss_rebin and pss_clip_cast run as separate kernels."""
    from psrsigsim_amd import _engine
    from psrsigsim_amd.utils.utils import rebin_edges
    rcvr, bak = tel.systems[system]
    kind, arg = tel.resample_branch(sig, bak)
    pend = sig._pend()
    rows, ncols = sig._c1 - sig._c0, sig._ncols
    dev = _engine.device()
    pre = torch.empty((rows, ncols), dtype=torch.float32, device=dev)
    pend.out = {"kind": _lib.OUT_F32, "tensor": pre, "clip": float("inf")}
    rcvr.radiometer_noise(sig, psr, gain=tel.gain, Tsys=tel.Tsys)
    sig._flush()
    if kind == "down":
        new_nt = ncols // arg
        res = torch.empty((rows, new_nt), dtype=torch.float32, device=dev)
        _lib.check(_lib.lib().pss_down_sample(_engine.ptr(pre), _engine.ptr(res), rows, ncols, pre.stride(0),
                                              int(arg), _engine.stream_ptr()))
    else:
        new_nt = int(arg)
        lo, hi = rebin_edges(ncols, new_nt)
        dlo, dhi = _engine.to_dev(lo), _engine.to_dev(hi)
        res = torch.empty((rows, new_nt), dtype=torch.float32, device=dev)
        _lib.check(_lib.lib().pss_rebin(_engine.ptr(pre), _engine.ptr(res), rows, ncols, pre.stride(0), new_nt,
                                        _engine.ptr(dlo), _engine.ptr(dhi), _engine.stream_ptr()))
    out = torch.empty((rows, new_nt), dtype=torch.float32, device=dev)
    _lib.check(_lib.lib().pss_clip_cast(_engine.ptr(res), _engine.ptr(out), res.numel(), float(sig._draw_max),
                                        _lib.OUT_F32, _engine.stream_ptr()))
    return out


def step(factor, ret):
    sig = FilterBankSignal(1400, 400, Nsubband=NCH, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, tobs=(1 << LOG2N) * DT)
    ISM().disperse(sig, 100)
    tel = Telescope(20.0, area=None, Tsys=25.0, name="T")
    # backend rate 1 / (2 dt_tel): dt_tel = factor * dt_sig
    tel.add_system(name="S", receiver=Receiver(fcent=1400, bandwidth=400, name="L"),
                   backend=Backend(samprate=1.0 / (2 * Quantity(factor * DT, "s")), name="B"))
    kind = tel.resample_branch(sig, tel.systems["S"][1])
    if ret == "staged":
        return sig, staged_observe(tel, sig, psr, "S"), kind
    out = tel.observe(sig, psr, system="S", noise=True, ret_resampsig=ret)
    return sig, out, kind


pss.seed(5)
for factor in FACTORS:
    for ret in (True, "staged", False):
        if ret == "staged" and factor == 1.0:
            continue
        for _ in range(2):
            s, o, kind = step(factor, ret)
            del s, o
        torch.cuda.synchronize()
        _lib.load().pss_timing_enable(1)
        _lib.timing_collect()
        t0 = time.perf_counter()
        n = 10
        for _ in range(n):
            s, o, kind = step(factor, ret)
            del s, o
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        _lib.load().pss_timing_enable(0)
        launches = _lib.timing_collect()
        agg = {}
        for k, ms, u in launches:
            agg[k] = agg.get(k, 0.0) + ms / n
        print("factor %.2f branch %-5s ret_resampsig=%-6s  %.3f ms/step  kernels %s" % (
            factor, kind[0], ret, dt * 1e3, {k: round(v, 3) for k, v in agg.items()}), flush=True)
