#!/usr/bin/env python
"""Per-kernel timing of C3 pipeline variants (GPU; diagnostic only).

Runs the C3 step with stages switched off one at a time and prints the average
per-kernel duration (HIP events, pss_timing_*), to attribute the cost of each
kernel to generation / null / noise / FFT work.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def step(variant, nchan, log2n):
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    sig = FilterBankSignal(1400, 400, Nsubband=nchan, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    ism = ISM()
    ism.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    psr.make_pulses(sig, tobs=(1 << log2n) * 20.48e-6)
    ism.disperse(sig, 100)
    if "nonull" not in variant:
        psr.null(sig, 0.1)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise="nonoise" not in variant)
    return sig


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nchan", type=int, default=2048)
    ap.add_argument("--log2n", type=int, default=22)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-fill", action="store_true")
    ap.add_argument("--flags", type=int, default=0, help="pss_set_flags value (e.g. 4 = no pipelined kernels)")
    ap.add_argument("variants", nargs="*", default=["full", "nonoise", "nonull", "nonull_nonoise"])
    a = ap.parse_args()
    import torch
    import psrsigsim_amd as pss
    from psrsigsim_amd import _lib
    L = _lib.lib()
    L.pss_set_flags(a.flags)
    pss.seed(1)
    res = {}
    for v in a.variants:
        s = step(v, a.nchan, a.log2n)
        _ = s.data
        del s
        torch.cuda.synchronize()
        L.pss_timing_enable(1)
        _lib.timing_collect()
        t0 = time.perf_counter()
        spans = []
        launches = []
        for _ in range(a.reps):
            s = step(v, a.nchan, a.log2n)
            _ = s.data
            del s
            torch.cuda.synchronize()
            spans.append(L.pss_timing_span_ms())      # device span of this step's runs
            launches += _lib.timing_collect()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.reps * 1e3
        L.pss_timing_enable(0)
        agg = {}
        full = a.nchan * (1 << a.log2n)
        for kind, ms, u in launches:
            if u != full:
                continue
            x = agg.setdefault(kind, [0.0, 0])
            x[0] += ms
            x[1] += 1
        res[v] = {"wall_ms": round(wall, 2), "span_ms": round(sum(spans) / len(spans), 3),
                  **{k: round(x[0] / x[1], 3) for k, x in agg.items()}}
        print(v, json.dumps(res[v]), flush=True)

    if a.no_fill:
        return
    # raw RNG cost: pss_chi2_fill over the same number of samples
    n = a.nchan * (1 << a.log2n)
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for df in (1.0, 100.0, 11190.0):
        L.pss_chi2_fill(out.data_ptr(), a.nchan, 0, 1 << a.log2n, df, 7, 3, 4, st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            L.pss_chi2_fill(out.data_ptr(), a.nchan, 0, 1 << a.log2n, df, 7, 3, 4, st)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        print("chi2_fill df=%g: %.3f ms (%.1f Gsamples/s)" % (df, ms, n / ms / 1e6), flush=True)


if __name__ == "__main__":
    main()
