"""Diagnostic: Bluestein chirp / Bhat tables in the workspace vs numpy."""
import sys
import numpy as np
import torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from psrsigsim_amd import _engine
from psrsigsim_amd.utils import shift_t

a256 = lambda b: ((b + 255) // 256) * 256
for N in [int(a) for a in sys.argv[1:]]:
    x = np.random.default_rng(N).random((1, N)).astype(np.float32)
    shift_t(x, np.array([0.37]), dt=1.0)
    torch.cuda.synchronize()
    ws = _engine._ws[(_engine.device().index, "main")]
    M = 1
    while M < 2 * N - 1:
        M <<= 1
    M2 = 8192 if M >= 2 ** 25 else 4096
    M1 = M // M2
    o = a256(2 * N * 8 + N * 8)
    ch = ws[o:o + N * 8].view(torch.complex64).cpu().numpy()
    n = np.arange(N, dtype=np.uint64)
    w = np.exp(-1j * np.pi * ((n * n) % np.uint64(2 * N)).astype(np.float64) / N)
    bad = np.nonzero(np.abs(ch - w) > 1e-5)[0]
    print(N, "chirp maxerr %.3g" % np.max(np.abs(ch - w)), "nbad", bad.size, bad[:5], flush=True)
    o2 = o + a256(N * 8)
    bh = ws[o2:o2 + M * 8].view(torch.complex64).cpu().numpy().reshape(M1, M2)
    b = np.zeros(M, complex)
    b[:N] = np.conj(w)
    j = np.arange(1, N)
    b[M - j] = np.conj(w[j])
    Y = np.fft.fft(b.reshape(M1, M2), axis=0) * np.exp(-2j * np.pi * np.arange(M1)[:, None] * np.arange(M2)[None, :] / M)
    ref = np.fft.fft(Y, axis=1) / M
    e = np.abs(bh - ref)
    print("  bhat maxerr %.3g (ref max %.3g)" % (e.max(), np.abs(ref).max()), "worst at", np.unravel_index(e.argmax(), e.shape), flush=True)
    # hypotheses: which b would give the device table?
    def four(bb):
        Y = np.fft.fft(bb.reshape(M1, M2), axis=0) * np.exp(-2j * np.pi * np.arange(M1)[:, None] * np.arange(M2)[None, :] / M)
        return np.fft.fft(Y, axis=1) / M
    rowe = e.max(axis=1)
    cole = e.max(axis=0)
    print("  rows bad:", np.sum(rowe > 1e-6), "cols bad:", np.sum(cole > 1e-6))
    # recover the device's b by inverting the four-step
    Q = np.fft.ifft(bh * M, axis=1)
    Q = Q * np.exp(2j * np.pi * np.arange(M1)[:, None] * np.arange(M2)[None, :] / M)
    bdev = np.fft.ifft(Q, axis=0).reshape(M)
    d = np.abs(bdev - b)
    badn = np.nonzero(d > 1e-4)[0]
    print("  recovered b: nbad", badn.size, "first", badn[:8], "last", badn[-8:] if badn.size else None, flush=True)
    if badn.size:
        i = badn[0]
        print("  b[%d] dev" % i, bdev[i], "ref", b[i], flush=True)
