#!/usr/bin/env python
"""Certification rate of the delayed-null mask table's root records (diagnostic).

Restates k_mask_table on the CPU for a C3-like mask row (2^22 samples, 1718
nulled periods of 244 chi2(100) box values): the KCH = 12 node shifts of the
box row (float64 FFT, the reference's Nyquist rule), their Chebyshev
coefficients per position (fp32, as on the device), the classification
(always / never / f-dependent), and for the f-dependent positions the scan
certification of root_hit (pss_pipeline.hip) at several grid sizes NG:

  * a cell whose ends share a sign holds no root when
    min(|g(t_j)|, |g(t_j+1)|) - err > D2 h^2 / 8   (chord-interpolation bound),
  * a cell with a sign change holds exactly one when
    |g(t_j+1) - g(t_j)| - 2 err > D2 h^2           (g' keeps its sign),

g = value - 1, D2 = sum_n |c_n| n^2 (n^2 - 1) / 3 (Markov's bound on T_n''),
err the fp32 Clenshaw error bound.  Positions that fail keep coefficient
records (evaluated directly by the null fix-up): the printed fraction is what
that costs.  The first bound tried in round 3, a derivative bound
|g(t_j)| + |g(t_j+1)| > h sum_n n^2 |c_n|, left ~90 % of the positions
uncertified at any NG (the Markov derivative bound is far above the actual
slopes) and cost the fix-up +0.5 ms on the GPU.

usage: python tools/mask_cert.py
"""
import numpy as np

N, NPH, NSUB, KCH = 1 << 22, 244, 17180, 12


def main():
    rng = np.random.default_rng(1)
    pulses = rng.choice(NSUB, NSUB // 10, replace=False)
    box = np.zeros(N)
    for p in pulses:
        b = np.arange(NPH * p, NPH * (p + 1)) + 2
        b = b[b < N]
        box[b] = rng.chisquare(100, b.size)
    t = np.cos(np.pi * (np.arange(KCH) + 0.5) / KCH)
    f = 0.5 * (t + 1)
    X = np.fft.rfft(box)
    k = np.arange(X.size)
    nodes = np.empty((KCH, N), np.float32)
    for j in range(KCH):
        Y = X * np.exp(-2j * np.pi * k * f[j] / N)
        Y[-1] = X[-1] * np.cos(np.pi * f[j])
        nodes[j] = np.fft.irfft(Y, n=N)
    T = np.array([[np.cos(np.pi * n * (j + 0.5) / KCH) * (2.0 if n else 1.0) / KCH for j in range(KCH)]
                  for n in range(KCH)], np.float32)
    C = (T @ nodes).astype(np.float32)
    S = np.abs(C[1:]).sum(0)
    eps = 1e-3 + 4e-6 * (np.abs(C[0]) + S)
    hi = C[0] - S > 1 + eps
    amb = ~hi & ~(C[0] + S < 1 - eps)
    c = C[:, np.where(amb)[0]].astype(np.float64)
    print("f-dependent positions: %d (%.4f of N)" % (c.shape[1], c.shape[1] / N))
    n = np.arange(1, KCH)[:, None]
    D2 = ((n ** 2 * (n ** 2 - 1) / 3) * np.abs(c[1:])).sum(0)
    err = 4e-6 * (np.abs(c[0]) + np.abs(c[1:]).sum(0))
    for NG in (32, 64, 128, 256, 512):
        H = 2.0 / NG
        g = np.stack([np.polynomial.chebyshev.chebval(-1 + i * H, c) - 1 for i in range(NG + 1)])
        flip = (g[1:] > 0) != (g[:-1] > 0)
        ok_flip = np.abs(g[1:] - g[:-1]) - 2 * err > D2 * H * H
        ok_same = np.minimum(np.abs(g[1:]), np.abs(g[:-1])) - err > D2 * H * H / 8
        cert = np.where(flip, ok_flip, ok_same).all(0)
        print("NG %4d: uncertified %.4f of the f-dependent positions (%d), max flips %d"
              % (NG, 1 - cert.mean(), (~cert).sum(), flip.sum(0).max()))


if __name__ == "__main__":
    main()
