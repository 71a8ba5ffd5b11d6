"""Pulse portraits (host plan layer).

Mirrors ``psrsigsim/pulsar/portraits.py`` (class names, methods, the Amax /
_max_profile state machine, errors).  Portraits are small (Nchan x Nph) float64
tables built on the host; the per-sample evaluation over the whole
(Nchan, nsamp) signal happens on the GPU (k_* source stage, ``pchip_eval``)
from the PCHIP coefficient table exported by :meth:`DataPortrait.device_table`.

The PCHIP construction follows the published Fritsch-Butland/Fritsch-Carlson
monotone cubic (as in scipy.interpolate.PchipInterpolator, which the
reference uses at portraits.py:252): weighted-harmonic-mean interior slopes,
one-sided three-point end slopes with the shape-preserving clamps, cubic
Hermite pieces, extrapolation with the end pieces.
"""
import logging

import numpy as np

from .. import _lib

log = logging.getLogger("psrsigsim_amd")

__all__ = ["PulsePortrait", "GaussPortrait", "DataPortrait", "UserPortrait", "is_uniform", "rows_of",
           "pchip_slopes", "pchip_coefficients", "pchip_coefficients_np", "ppoly_eval", "ppoly_eval_np"]


# ---------------------------------------------------------------------------
# row-uniform tables
#
# A 1-D profile tiled over the channels (GaussProfile, DataProfile of a 1-D
# template -- BASELINE configs C2-C5) gives an (Nchan, Nph) table whose rows
# are all the same.  Such tables are kept as read-only broadcast views of
# their one row (row stride 0) and every table operation below runs on that
# row: the values are exactly those of the full table (each row is computed
# by the same float64 operations), at 1/Nchan of the host time and memory.
# ---------------------------------------------------------------------------
def is_uniform(a):
    """True for a broadcast table: 2-D, several rows, row stride 0."""
    return isinstance(a, np.ndarray) and a.ndim >= 2 and a.shape[0] > 1 and a.strides[0] == 0


def rows_of(a):
    """The distinct rows to compute on: row 0 of a uniform table, else all."""
    return a[:1] if is_uniform(a) else a


def like_rows(res, a):
    """``res`` (computed on rows_of(a)) with ``a``'s row count restored."""
    if is_uniform(a) and res.shape[0] == 1:
        return np.broadcast_to(res, (a.shape[0],) + res.shape[1:])
    return res


def tile_rows(row, nrows):
    """np.tile(row, (nrows, 1)) as a uniform (broadcast) table."""
    row = np.asarray(row)
    return np.broadcast_to(row[None] if row.ndim == 1 else row[:1], (nrows,) + row.shape[-1:])


def table_max(a):
    return rows_of(a).max()


# ---------------------------------------------------------------------------
# PCHIP (float64, host)
# ---------------------------------------------------------------------------
def _edge_slope(h0, h1, m0, m1):
    d = ((2 * h0 + h1) * m0 - h0 * m1) / (h0 + h1)
    flip = np.sign(d) != np.sign(m0)
    big = (np.sign(m0) != np.sign(m1)) & (np.abs(d) > 3 * np.abs(m0))
    d = np.where(flip, 0.0, d)
    return np.where((~flip) & big, 3 * m0, d)


def pchip_slopes(x, y, h=None, m=None):
    """Knot derivatives for rows of ``y`` (shape [rows, K]) at knots ``x``."""
    x = np.asarray(x, dtype=float)
    y = np.asarray(y, dtype=float)
    if h is None:
        h = np.diff(x)
    if m is None:
        m = np.diff(y, axis=1) / h
    K = x.size
    if K == 2:
        return np.repeat(m, 2, axis=1)
    d = np.empty_like(y)
    m0, m1 = m[:, :-1], m[:, 1:]
    w1 = 2 * h[1:] + h[:-1]
    w2 = h[1:] + 2 * h[:-1]
    with np.errstate(divide="ignore", invalid="ignore"):
        inner = 1.0 / ((w1 / m0 + w2 / m1) / (w1 + w2))
    flat = (np.signbit(m0) != np.signbit(m1)) | (m1 == 0) | (m0 == 0)
    inner[flat] = 0.0
    d[:, 1:-1] = inner
    d[:, 0] = _edge_slope(h[0], h[1], m[:, 0], m[:, 1])
    d[:, -1] = _edge_slope(h[-1], h[-2], m[:, -1], m[:, -2])
    return d


def pchip_coefficients(x, y):
    """Piecewise-cubic coefficients [rows, K-1, 4] in powers (t - x_i)^(3..0).
    Computed natively (pss_host_pchip_coef, one pass per row, host threads);
    bitwise equal to :func:`pchip_coefficients_np`.  A uniform table's
    coefficients are computed once and broadcast."""
    y = np.atleast_2d(np.asarray(y, dtype=float))
    return like_rows(_lib.host_pchip_coef(x, np.ascontiguousarray(rows_of(y))), y)


def pchip_coefficients_np(x, y):
    """NumPy statement of :func:`pchip_coefficients` (the tested reference)."""
    x = np.asarray(x, dtype=float)
    y = np.asarray(y, dtype=float)
    h = np.diff(x)
    m = np.diff(y, axis=1) / h
    d = pchip_slopes(x, y, h, m)
    d0, d1 = d[:, :-1], d[:, 1:]
    t = (d0 + d1 - 2 * m) / h
    c = np.empty((y.shape[0], x.size - 1, 4))
    c[:, :, 0] = t / h
    c[:, :, 1] = (m - d0) / h - t
    c[:, :, 2] = d0
    c[:, :, 3] = y[:, :-1]
    return c


def ppoly_eval(x, c, ph, y=None):
    """Evaluate the piecewise cubic at phases ``ph`` (extrapolating with the
    end pieces); returns [rows, len(ph)].

    The arithmetic replicates the published PPoly evaluation scipy performs for
    the reference (power accumulation res += c_k * s^k, s^k by repeated
    multiplication, lowest power first; interval = last breakpoint <= x,
    clipped to the end pieces) bit for bit, because the reference makes exact
    float decisions on these values (the periodic-closure test at
    portraits.py:234 compares generator(0) with generator(1))."""
    ph = np.asarray(ph, dtype=float)
    if y is not None and ph.size <= x.size and np.array_equal(ph, x[:ph.size]):
        return like_rows(np.array(rows_of(y)[:, :ph.size]), y)
    return like_rows(_lib.host_ppoly_eval(x, np.ascontiguousarray(rows_of(c)), ph), c)


def ppoly_eval_np(x, c, ph):
    """NumPy statement of :func:`ppoly_eval` (the tested reference)."""
    ph = np.asarray(ph, dtype=float)
    i = np.clip(np.searchsorted(x, ph, side="right") - 1, 0, x.size - 2)
    s = (ph - x[i])[None, :]
    ci = c[:, i, :]
    res = ci[:, :, 3] * 1.0
    z = s
    res = res + ci[:, :, 2] * z
    z = z * s
    res = res + ci[:, :, 1] * z
    z = z * s
    res = res + ci[:, :, 0] * z
    return res


# ---------------------------------------------------------------------------
# portraits
# ---------------------------------------------------------------------------
def _first_max_row(profiles, rowset=None):
    """``[pr for pr in profiles if pr.max() == 1.0][0]`` (portraits.py:45),
    vectorised; IndexError when no row peaks at exactly 1.0, as there.  With
    a ``rowset`` (shard-local planning) ``profiles`` holds this rank's rows
    and the first such row of the whole band comes from the rank holding it."""
    if rowset is not None:
        row = rowset.first_row(np.max(profiles, axis=1) == 1.0, profiles)
        if row is None:
            raise IndexError("list index out of range")
        return row
    hit = np.flatnonzero(np.max(rows_of(profiles), axis=1) == 1.0)
    if hit.size == 0:
        raise IndexError("list index out of range")
    return rows_of(profiles)[hit[0]]


def _band_max(profiles, rowset=None):
    """table_max over the whole band (a reduction over the plan group when
    ``profiles`` holds only this rank's rows)."""
    m = table_max(profiles)
    return m if rowset is None else rowset.max(m)


class PulsePortrait(object):
    """portraits.py:9-91."""
    _profiles = None

    def __call__(self, phases=None):
        if phases is None:
            if self._profiles is None:
                print("Warning: base profiles not generated, returning `None`")
            return self._profiles
        return self.calc_profiles(phases)

    _rowset = None      # shard.RowSet: this portrait holds only the rank's rows

    def init_profiles(self, Nphase, Nchan=None):
        """portraits.py:32-45: sample at arange(N)/N, renormalise to max 1."""
        ph = np.arange(Nphase) / Nphase
        self._profiles = self.calc_profiles(ph, Nchan=Nchan)
        self._Amax = _band_max(self._profiles, self._rowset)
        # (x / 1.0 is x: calc_profiles already divided by the band max, so the
        # renormalisation is the identity unless a rank's rows differ)
        if self.Amax != 1.0:
            self._profiles = like_rows(rows_of(self._profiles) / self.Amax, self._profiles)
        self._max_profile = _first_max_row(self._profiles, self._rowset)

    def calc_profiles(self, phases, Nchan=None):
        raise NotImplementedError()

    def _calcOffpulseWindow(self, Nphase=None):
        """portraits.py:62-82: argmin over a sliding trapezoid of width Nph/8
        (circular), window returned as float indices mod Nph."""
        ws = (2048 / 8) if Nphase is None else Nphase / 8
        half = ws // 2
        prof = np.asarray(self._max_profile, dtype=float)
        n = len(prof)
        integral = np.zeros_like(prof)
        lo = int(-half)
        width = int(2 * half)
        # trapezoid over `width` consecutive (circular) samples starting at i-half
        idx = (np.arange(n)[:, None] + lo + np.arange(width)[None, :]) % Nphase
        w = prof[idx]
        integral[:] = w.sum(axis=1) - 0.5 * (w[:, 0] + w[:, -1]) if width > 1 else 0.0
        minind = np.argmin(integral)
        return np.arange(minind - half, minind + half + 1) % Nphase

    @property
    def profiles(self):
        return self._profiles

    @property
    def Amax(self):
        return self._Amax


def _gauss_single(ph, peak, width, amp):
    ph = np.asarray(ph)
    if ph.size and (ph.max() > 1 or ph.min() < 0):      # (np.any(ph > 1) or np.any(ph < 0): NaN passes both)
        raise ValueError('Phase values must all lie within [0,1].')
    t = (ph - peak) / width
    if t.dtype != np.float64 or np.ndim(amp) or np.ndim(t) == 0:
        return amp * np.exp(-0.5 * t ** 2)
    # amp * exp(-0.5 * t ** 2) in place (t ** 2 is np.square; the same
    # operations and bits, two temporaries fewer on a 48 828-phase profile)
    np.square(t, out=t)
    t *= -0.5
    np.exp(t, out=t)
    t *= amp
    return t


def _gauss_sum(ph, peaks, widths, amps):
    if np.any(ph > 1) or np.any(ph < 0):
        raise ValueError('Phase values must all lie within [0,1].')
    return np.sum(amps[:, None] * np.exp(-0.5 * ((ph[None, :] - peaks[:, None]) / widths[:, None]) ** 2),
                  axis=0)


class GaussPortrait(PulsePortrait):
    """portraits.py:94-198: sum of Gaussian components; 1-D parameters are
    tiled over channels, 2-D parameters give one row per channel."""

    def __init__(self, peak=0.5, width=0.05, amp=1):
        self._peak = peak
        self._width = width
        self._amp = amp
        self._profiles = None

    def init_profiles(self, Nphase, Nchan=None):
        """portraits.py:131-140 (no renormalisation)."""
        ph = np.arange(Nphase) / Nphase
        self._profiles = self.calc_profiles(ph, Nchan=Nchan)
        self._max_profile = _first_max_row(self._profiles)

    def calc_profiles(self, phases, Nchan=None):
        ph = np.array(phases)
        if hasattr(self.peak, 'ndim') and self.peak.ndim == 2:
            profiles = np.array([_gauss_sum(ph, self.peak[:], self.width[:], self.amp[:])
                                 for _ in range(self.peak.shape[0])])
        else:
            if Nchan is None:
                raise ValueError('Nchan must be provided if only 1-dim profile information provided.')
            if hasattr(self.peak, 'ndim') and self.peak.ndim == 1:
                one = _gauss_sum(ph, self.peak, self.width, self.amp)
            else:
                one = _gauss_single(ph, self.peak, self.width, self.amp)
            profiles = tile_rows(one, Nchan)
        self._Amax = self.Amax if hasattr(self, '_Amax') else table_max(profiles)
        return like_rows(rows_of(profiles) / self._Amax, profiles)

    @property
    def peak(self):
        return self._peak

    @property
    def width(self):
        return self._width

    @property
    def amp(self):
        return self._amp

    @property
    def Amax(self):
        return self._Amax


class DataPortrait(PulsePortrait):
    """portraits.py:200-267: PCHIP through the sampled profiles; periodicity is
    enforced by appending the first column (phases arange(N+1)/N) when the
    first and last columns differ."""

    def __init__(self, profiles, phases=None, *, rowset=None):
        """``rowset`` (keyword-only, shard-local planning): ``profiles`` holds
        the rows of ``rowset.gids`` only; the portrait-wide decisions (the
        periodic closure here, Amax and the max row later) are reductions over
        its group."""
        self._rowset = rowset
        profiles = np.asarray(profiles)
        uni = is_uniform(profiles)
        work = rows_of(profiles)            # a uniform table is processed as its one row
        neg = work < 0.0
        if np.any(neg):
            log.warning("Some phase bins of input profile are negative, replacing them with zeros...")
            if uni:
                work = np.where(neg, 0.0, work)
            else:
                work[neg] = 0.0            # in place on the caller's array, as there
        def band_any(flags):
            f = bool(np.any(flags))
            return f if rowset is None else rowset.any(f)
        self._geo = None
        if phases is None:
            N = work.shape[1]
            if band_any(work[:, 0] != work[:, -1]):
                work = np.append(work, work[:, 0][:, np.newaxis], axis=1)
                phases = np.arange(N + 1) / N
            else:
                phases = np.arange(N) / N
            if phases.size >= 2:
                self._geo = (N, phases.size - 1)   # knots k / N: uniform_knots' answer
        else:
            phases = np.asarray(phases, dtype=float)
            if phases[-1] != 1:
                phases = np.append(phases, 1)
                work = np.append(work, work[:, 0][:, np.newaxis], axis=1)
            elif band_any(work[:, 0] != work[:, -1]):
                if uni:
                    work = np.array(work)
                work[:, -1] = work[:, 0]
        self._knots = np.asarray(phases, dtype=float)
        kv = np.asarray(work, dtype=float)
        self._kvals = np.broadcast_to(kv, (profiles.shape[0],) + kv.shape[1:]) if uni else kv
        self._coef_cache = None

    @property
    def _coef(self):
        # built on first use: a fold-mode signal only ever evaluates the
        # portrait AT its knots (the reference's linspace resampling hits them
        # exactly), which needs no coefficients
        if self._coef_cache is None:
            self._coef_cache = pchip_coefficients(self._knots, self._kvals)
        return self._coef_cache

    def _knot_hit(self, ph):
        return ph.size <= self._knots.size and np.array_equal(ph, self._knots[:ph.size])

    def _generator(self, phases):
        ph = np.asarray(phases, dtype=float)
        if self._knot_hit(ph):
            return like_rows(np.array(rows_of(self._kvals)[:, :ph.size]), self._kvals)
        if self._coef_cache is None:
            # no coefficient table needed: PCHIP built and evaluated per row
            return like_rows(_lib.host_pchip_eval(self._knots, rows_of(self._kvals), ph), self._kvals)
        return ppoly_eval(self._knots, self._coef, phases, self._kvals)

    def calc_profiles(self, phases, Nchan=None):
        ph = np.asarray(phases, dtype=float)
        if hasattr(self, '_Amax'):
            # the division by Amax fused into the one pass that makes the rows
            # (the same IEEE operations as generator-then-divide)
            if self._knot_hit(ph):
                return like_rows(rows_of(self._kvals)[:, :ph.size] / self.Amax, self._kvals)
            if self._coef_cache is None:
                return like_rows(_lib.host_pchip_eval(self._knots, rows_of(self._kvals), ph, self.Amax),
                                 self._kvals)
        if self._knot_hit(ph):
            # the knot values themselves: the band max over the view, one
            # division pass (no copy first)
            kv = rows_of(self._kvals)[:, :ph.size]
            return like_rows(kv / _band_max(kv, self._rowset), self._kvals)
        profiles = self._generator(phases)
        Amax = self.Amax if hasattr(self, '_Amax') else _band_max(profiles, self._rowset)
        return like_rows(rows_of(profiles) / Amax, profiles)

    def row_ids(self):
        """Global channel of each row of this portrait's tables (None: row c is
        channel c, or one shared row)."""
        return None if self._rowset is None else self._rowset.gids

    # -- device export --------------------------------------------------
    def uniform_knots(self):
        """(M, nint) when the knots are k/M (k = 0..nint), else None."""
        if getattr(self, "_geo", None) is not None:
            return self._geo
        x = self._knots
        nint = x.size - 1
        M = int(round(1.0 / (x[1] - x[0]))) if nint >= 1 else 0
        # (allclose(x, arange / M, rtol=0, atol=1e-15), without its temporaries)
        if M < 1 or not np.max(np.abs(x - np.arange(x.size) / M)) <= 1e-15:
            return None
        return M, nint

    def device_table(self, room=False):
        """float32 [rows, nint, 4] coefficients in the local coordinate
        u = (phase - k/M) * M, ordered (u^3, u^2, u^1, u^0), divided by Amax
        so the device evaluates calc_profiles directly; plus (M, nint).  On
        non-uniform knots see :meth:`split_table` (the third element is then
        the [M] split points instead of nint, and the table is [rows, M, 8]).
        ``room``: a one-row table whose knots stop short of the period may come
        back M intervals wide, the last M - nint left for the caller
        (pulsar._device_table's extrapolated pieces)."""
        geo = self.uniform_knots()
        if geo is None:
            return self.split_table()
        M, nint = geo
        h = 1.0 / M
        amax = self.Amax if hasattr(self, '_Amax') else 1.0
        # = (self._coef * [h**3, h**2, h, 1] / amax).astype(float32), natively
        # (one row for a uniform table: the device then shares it); straight
        # from the knot values when no coefficient table exists yet
        if self._coef_cache is None:
            return _lib.host_pchip_table(self._knots, rows_of(self._kvals), h, amax,
                                         width=M if room else None), M, nint
        return _lib.host_device_table(np.ascontiguousarray(rows_of(self._coef)), h, amax), M, nint


    def split_table(self, max_cells=1 << 16):
        """Device form of a portrait on NON-uniform phases: M = 2^m uniform
        cells over [0, 1), each holding at most one interior breakpoint; per
        cell and row the cubic in force at the cell's start and the one after
        its breakpoint, both re-expanded in the cell coordinate u = phase M - c
        (float64, then /Amax to float32), and the breakpoint's u (2 when the
        cell has none).  Evaluating the cubic on the breakpoint's side is the
        piecewise polynomial the reference evaluates (interval = last
        breakpoint <= phase, end pieces extrapolated; portraits.py:252).
        Returns (table [rows, M, 8] float32, M, split [M] float32)."""
        x = self._knots
        K = x.size - 1
        c = np.asarray(rows_of(self._coef), dtype=np.float64)          # [rows, K, 4], powers 3..0
        inner = x[1:K]                       # breakpoints where the piece changes
        M = 1
        while M < 2 * K:
            M *= 2
        while True:
            pos = inner * M
            cell = np.floor(pos).astype(np.int64)
            strict = pos != cell            # on a cell boundary: no split needed
            if cell[strict].size == np.unique(cell[strict]).size:
                break
            M *= 2
            if M > max_cells:
                raise NotImplementedError("portrait breakpoints closer than 1/%d of a period" % max_cells)
        starts = np.arange(M, dtype=np.float64) / M
        iL = np.clip(np.searchsorted(x, starts, side="right") - 1, 0, K - 1)
        split = np.full(M, 2.0)
        iR = iL.copy()
        sc = cell[strict]
        split[sc] = pos[strict] - sc
        iR[sc] = np.clip(np.searchsorted(x, inner[strict], side="right") - 1, 0, K - 1)
        h = 1.0 / M

        def expand(idx):
            d = starts - x[idx]                                       # [M]
            ci = c[:, idx, :]                                         # [rows, M, 4]
            c3, c2, c1, c0 = ci[..., 0], ci[..., 1], ci[..., 2], ci[..., 3]
            return np.stack([c3 * h ** 3, (3 * c3 * d + c2) * h ** 2, ((3 * c3 * d + 2 * c2) * d + c1) * h,
                             ((c3 * d + c2) * d + c1) * d + c0], axis=-1)
        amax = self.Amax if hasattr(self, '_Amax') else 1.0
        tab = np.concatenate([expand(iL), expand(iR)], axis=-1) / amax
        tab = like_rows(tab, self._coef) if tab.shape[0] == 1 else tab
        return np.ascontiguousarray(rows_of(tab)).astype(np.float32), M, split.astype(np.float32)


class UserPortrait(PulsePortrait):
    """portraits.py:270-275."""

    def __init__(self):
        raise NotImplementedError()
