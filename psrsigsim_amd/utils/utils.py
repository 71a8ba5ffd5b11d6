"""utils -- mirrors the synthesis-path helpers of ``psrsigsim/utils/utils.py``.

``shift_t``, ``down_sample`` and ``rebin`` run on the GPU (pss_shift_rows,
pss_down_sample, pss_rebin).  They accept NumPy arrays (returned as NumPy, like
the reference) or torch tensors (kept on the device), 1-D like the reference
or 2-D as a batch of rows.
"""
import numpy as np
import torch

from .._units import make_quant  # noqa: F401  (re-exported, utils.py:310)
from .. import _engine, _lib

__all__ = ["shift_t", "down_sample", "rebin", "make_quant", "top_hat_width", "make_par"]


def _as_rows(y):
    """(device float32 rows tensor, was_numpy, was_1d)."""
    was_np = not isinstance(y, torch.Tensor)
    t = torch.as_tensor(np.asarray(y, dtype=np.float32)) if was_np else y
    was_1d = t.dim() == 1
    if was_1d:
        t = t.reshape(1, -1)
    t = t.to(device=_engine.device(), dtype=torch.float32).contiguous()
    return t, was_np, was_1d


def _ret(t, was_np, was_1d):
    if was_1d:
        t = t.reshape(-1)
    return t.cpu().numpy().astype(np.float64) if was_np else t


def shift_t(y, shift, dt=1):
    """utils.py:17-59: delay y by ``shift`` (same units as ``dt``).  Integer
    shift with dt == 1 -> circular roll; otherwise the Fourier shift theorem:
    rfft -> exp(-2 pi i f shift) -> irfft (Nyquist bin keeps cos(pi s)).
    For odd N the result has N - 1 samples, as the reference's irfft (no n=)
    returns.  ``shift`` may be one value per row for a 2-D batch."""
    if isinstance(shift, int) and dt == 1:
        if isinstance(y, torch.Tensor):
            return torch.roll(y, shift, dims=-1)
        return np.roll(y, shift)
    t, was_np, was_1d = _as_rows(y)
    if not was_np and t.data_ptr() == y.data_ptr():
        t = t.clone()          # the reference returns a new array; y stays as it was
    R, N = t.shape
    s = np.broadcast_to(np.asarray(shift, dtype=np.float64) / float(dt), (R,))
    ramp = _engine.u64_to_i64_tensor(_engine.ramp_words(s, N))
    nyq = _engine.to_dev(np.cos(np.pi * s).astype(np.float32))
    ws = _engine.workspace(_lib.load().pss_workspace_bytes(R, N))
    rc = _lib.lib().pss_shift_rows(_engine.ptr(t), R, N, t.stride(0), _engine.ptr(ramp),
                                   _engine.ptr(nyq), _engine.ptr(ws), _engine.stream_ptr())
    _lib.check(rc, "shift_t")
    if N % 2:
        # odd N: np.fft.irfft without n= returns N - 1 samples (utils.py:57);
        # the library wrote them into the first N - 1 columns
        t = t[:, :N - 1]
    return _ret(t, was_np, was_1d)


def down_sample(ar, fact):
    """utils.py:62-68: mean over consecutive groups of ``fact`` samples."""
    t, was_np, was_1d = _as_rows(ar)
    R, N = t.shape
    if N % fact:
        raise ValueError("cannot reshape array of size %d into shape (%d)" % (N, fact))
    out = torch.empty((R, N // fact), dtype=torch.float32, device=t.device)
    rc = _lib.lib().pss_down_sample(_engine.ptr(t), _engine.ptr(out), R, N, t.stride(0), int(fact),
                                    _engine.stream_ptr())
    _lib.check(rc, "down_sample")
    return _ret(out, was_np, was_1d)


def rebin_edges(size, newlen):
    """Integer windows [lo_i, hi_i) of utils.py:77-89 -- the same float64
    operations as the reference's per-bin loop (ceil(lbin), ceil(lbin +
    stride) clipped to the size), elementwise over the bins."""
    newBins = np.linspace(0, size, newlen, endpoint=False)
    stride = newBins[1] - newBins[0]
    hi = np.minimum(np.ceil(newBins + stride), size).astype(np.int64)
    lo = np.ceil(newBins).astype(np.int64)
    return lo, hi


def rebin(ar, newlen):
    """utils.py:71-91: general downsampler (ceil-edged windows, mean)."""
    t, was_np, was_1d = _as_rows(ar)
    R, N = t.shape
    lo, hi = rebin_edges(N, newlen)
    dlo, dhi = _engine.to_dev(lo), _engine.to_dev(hi)
    out = torch.empty((R, newlen), dtype=torch.float32, device=t.device)
    rc = _lib.lib().pss_rebin(_engine.ptr(t), _engine.ptr(out), R, N, t.stride(0), int(newlen),
                              _engine.ptr(dlo), _engine.ptr(dhi), _engine.stream_ptr())
    _lib.check(rc, "rebin")
    return _ret(out, was_np, was_1d)


def top_hat_width(subband_df, subband_f0, DM):
    """utils.py:94-105 (scalar helper, off the synthesis path): intra-channel
    dispersion smearing 2 D DM df / f0^3 in ms, D = 4.148808e3 s MHz^2 cm^3/pc."""
    D = 4.148808e3
    return 2 * D * DM * subband_df / subband_f0 ** 3 * 1.0e+3


# par-file lines of make_par after PSR / F0 / DM (utils.py:366-391)
_PAR_DEFAULTS = [("LAMBDA", "            10.0"), ("BETA", "           10.0"), ("PMLAMBDA", "            0.0"),
                 ("PMBETA", "            0.0"), ("PX", "            0.0"), ("POSEPOCH", "            56000.0")]
_PAR_TAIL = [("PEPOCH", "            56000.0"), ("START", "            50000.0"), ("FINISH", "            60000.0")]
_PAR_END = [("EPHEM", "               DE436"), ("SOLARN0", "               0.00"), ("ECL", "                 IERS2010"),
            ("CLK", "                 TT(BIPM2015) "), ("UNITS", "               TDB"),
            ("TIMEEPH", "             FB90"), ("T2CMETHOD", "           TEMPO"),
            ("CORRECT_TROPOSPHERE", " N"), ("PLANET_SHAPIRO", "      N"), ("DILATEFREQ", "          N"),
            ("TZRMJD", "        56000.0"), ("TZRFRQ", "            1500.0"), ("TZRSITE", "                  @"),
            ("MODE", "                     1")]


def make_par(signal, pulsar, outpar="simpar.par"):
    """utils.py:350-395: a par file for the simulated pulsar (called by the
    PSRFITS save path when no par file is given): PSR name, F0 = 1/period,
    DM, and the reference's fixed defaults, one line each."""
    period = float(getattr(pulsar.period, "value", pulsar.period))
    dm = float(getattr(signal.dm, "value", signal.dm))
    lines = ["PSR            %s\n" % (pulsar.name)]
    lines += ["%s%s\n" % kv for kv in _PAR_DEFAULTS]
    lines.append("F0           %s\n" % (1.0 / period))
    lines += ["%s%s\n" % kv for kv in _PAR_TAIL]
    lines.append("DM                %s\n" % (dm))
    lines += ["%s%s\n" % kv for kv in _PAR_END]
    with open(outpar, "w") as op:
        op.writelines(lines)
