#!/usr/bin/env python
"""NumPy model of the device's chi2(1) draws (diagnostic / statistics study).

Philox4x32-R (Salmon et al. 2011; the device's pss::philox, R = 7) with the
pipeline's keying -- counter (block, tag 0, channel, call << 4 | purpose),
key = seed; block n >> 2 holds samples 4 (n >> 2) .. + 3 (the noise and
replacement draws; the search pulses' draws of an N-sample row, N % 4 == 0,
take block n mod N/4, element n div N/4 for N >= 2^24: pss::pulse_draw, `layout="quarter"`
below) -- and the Box-Muller chi2(1) of pss::chi2_1x4.  It reproduces
the device stream bit for bit (a GPU test's KS statistic on device draws
equals the model's to all printed digits), so the quality of the generator
can be studied on the CPU at sample sizes no GPU test would use:

  tools/philox_model.py study     -> profiles/r03/philox_quality.txt

compares R = 7 (both Box-Muller forms) and R = 10 on (a) KS p-values of the on-pulse selection of
tests/test_gpu_stats.py::test_search_pulse_draws_are_chi2_1 over 400 seeds
(their distribution must be uniform), (b) lag correlations over 6.7e7
draws, (c) mean / second moment over 6.7e7 draws."""
import os
import sys

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
MASK = np.uint64(0xFFFFFFFF)


def philox(c0, c1, c2, c3, k0, k1, rounds):
    c0, c1, c2, c3 = [np.asarray(x, dtype=np.uint64) & MASK for x in (c0, c1, c2, c3)]
    k0, k1 = np.uint64(k0), np.uint64(k1)
    for _ in range(rounds):
        p0, p1 = c0 * M0, c2 * M1
        c0, c1, c2, c3 = (((p1 >> np.uint64(32)) ^ c1 ^ k0) & MASK, p1 & MASK,
                          ((p0 >> np.uint64(32)) ^ c3 ^ k1) & MASK, p0 & MASK)
        k0 = (k0 + np.uint64(0x9E3779B9)) & MASK
        k1 = (k1 + np.uint64(0xBB67AE85)) & MASK
    return c0, c1, c2, c3


def chi2_1(n, chan, seed, call, purpose, rounds=7, form="cos2", layout="consecutive"):
    """Draws n = 0 .. n-1 of global channel `chan`.  form "cos2" (the device's
    sampler): h (1 +- cos 4 pi v), h = -ln u, with the
    fp32 roundings of the device's last three operations (so the cancellation
    of the small member of a pair is modelled); "two-trig": the previous
    -2 ln u cos^2 / sin^2 form, float64."""
    blocks = np.arange((n + 3) // 4, dtype=np.uint64)
    r = philox(blocks, 0, chan, (call << 4) | purpose, seed & 0xFFFFFFFF, seed >> 32, rounds)
    u01 = lambda x: x.astype(np.float64) * 2.0 ** -32 + 2.0 ** -33
    fr = lambda x: (x >> np.uint64(9)).astype(np.float64) * 2.0 ** -23
    if form == "cos2":
        f32 = np.float32
        fr2 = lambda x: ((x << np.uint64(1)) & MASK).astype(np.uint64)
        h0, h1 = f32(-np.log(u01(r[0]))), f32(-np.log(u01(r[2])))
        c0, c1 = f32(np.cos(2 * np.pi * fr(fr2(r[1])))), f32(np.cos(2 * np.pi * fr(fr2(r[3]))))
        # fused h (1 +- c): the product exact in float64, one fp32 rounding
        d0, d1 = h0.astype(np.float64) * c0, h1.astype(np.float64) * c1
        out = np.stack([f32(h0 + d0), f32(h0 - d0), f32(h1 + d1), f32(h1 - d1)], 1).astype(np.float64)
        return _arrange(out, n, layout)
    l0, l1 = -2 * np.log(u01(r[0])), -2 * np.log(u01(r[2]))
    v0, v1 = 2 * np.pi * fr(r[1]), 2 * np.pi * fr(r[3])
    out = np.stack([l0 * np.cos(v0) ** 2, l0 * np.sin(v0) ** 2, l1 * np.cos(v1) ** 2, l1 * np.sin(v1) ** 2], 1)
    return _arrange(out, n, layout)


def _arrange(out, n, layout):
    """Samples from the [block][4] draws: consecutive (sample 4 m + e) or
    the search pulses' quarter layout (sample m + e n/4, n % 4 == 0, n >= 2^24)."""
    if layout == "quarter" and n % 4 == 0 and n >= (1 << 24):
        return out[:n // 4].T.ravel()
    return out.ravel()[:n]


def study(out):
    from scipy import stats
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    sig = FilterBankSignal(1400, 400, Nsubband=2, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.1, 1))
    psr.make_pulses(sig, tobs=(1 << 18) * 20.48e-6)
    n = sig._ncols
    spp = (sig._samprate_MHz() * 0.005) * 1e6
    sel = psr.Profiles.calc_profiles((np.arange(n) / spp) % 1)[0] > 0.5
    lines = []
    for R, form in ((7, "cos2"), (7, "two-trig"), (10, "two-trig")):
        ps = np.array([stats.kstest(chi2_1(n, 0, s, 1, 1, R, form, layout="quarter")[sel], stats.chi2(1).cdf).pvalue
                       for s in range(1, 401)])
        lag = {}
        m1 = m2 = 0.0
        small = 0
        for ch in range(8):
            x = chi2_1(1 << 23, 10 + ch, 4242, 1, 1, R, form)
            small += int((x < 1e-4).sum())
            m1 += x.mean() / 8
            m2 += (x * x).mean() / 8
            x = x - 1.0
            for l in (1, 2, 3, 4, 5, 8):
                lag[l] = lag.get(l, 0.0) + np.mean(x[:-l] * x[l:]) / 2.0 / 8
        se = 1.0 / np.sqrt(8 * (1 << 23))
        lines.append("Philox4x32-%d, %s sampler: on-pulse KS over 400 seeds: frac p<0.01 %.4f, p<0.05 %.4f, "
                     "uniformity of the p-values (KS) %.3f; P(x < 1e-4) = %.3e (chi2(1): %.3e)"
                     % (R, form, (ps < .01).mean(), (ps < .05).mean(), stats.kstest(ps, "uniform").pvalue,
                        small / (8.0 * (1 << 23)), stats.chi2(1).cdf(1e-4)))
        lines.append("  6.7e7 draws: mean-1 %.2e (SE %.1e), E[x^2]/3-1 %.2e (SE %.1e); lag correlations in SE units %s"
                     % (m1 - 1, np.sqrt(2 / 6.7e7), m2 / 3 - 1, np.sqrt(96 / 6.7e7) / 3,
                        {l: round(v / se, 2) for l, v in lag.items()}))
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "study":
        study(sys.argv[2] if len(sys.argv) > 2 else "profiles/r03/philox_quality.txt")
