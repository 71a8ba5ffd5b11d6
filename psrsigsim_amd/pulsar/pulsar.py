"""Pulsar -- mirrors ``psrsigsim/pulsar/pulsar.py``.

make_pulses builds the host plan (Nph, nsamp, nsub, Nfold, draw_norm, the
spectral-index-scaled PCHIP portrait) exactly as the reference does
(pulsar.py:86-151) and records a *source* stage; the (Nchan, nsamp)
intensities -- profile x chi2 draws x draw_norm -- are generated on the GPU
inside the fused run.  null() derives the pulse choice and the off-pulse
level on the host, shift_val on the device (no host round trip), and records
a null stage (pulsar.py:246-333).
"""
import math

import numpy as np

from .profiles import GaussProfile, DataPortrait
from .portraits import GaussPortrait, is_uniform, rows_of
from .._units import make_quant, Quantity, to_value
from .. import _engine

__all__ = ["Pulsar"]


class Pulsar(object):
    """pulsar.py:11-84."""

    def __init__(self, period, Smean, profiles=None, name=None, specidx=0.0, ref_freq=None):
        self._period = make_quant(period, 's')
        self._Smean = make_quant(Smean, 'Jy')
        self._name = name
        self._specidx = specidx
        if ref_freq is not None:
            self._ref_freq = make_quant(ref_freq, "MHz")
        else:
            self._ref_freq = ref_freq
        self._Profiles = GaussProfile() if profiles is None else profiles

    def __repr__(self):
        namestr = "" if self.name is None else self.name + ", "
        return "Pulsar(" + namestr + "{})".format(self.period.to('ms'))

    @property
    def Profiles(self):
        return self._Profiles

    @property
    def name(self):
        return self._name

    @property
    def period(self):
        return self._period

    @property
    def Smean(self):
        return self._Smean

    @property
    def specidx(self):
        return self._specidx

    @property
    def ref_freq(self):
        return self._ref_freq

    # -- helpers -------------------------------------------------------------
    def _P(self):
        return float(to_value(self._period, 's'))

    def _nph(self, signal):
        """int((samprate * period).decompose()) (pulsar.py:96, 124)."""
        return int((signal._samprate_MHz() * self._P()) * 1e6)

    def _add_spec_idx(self, signal):
        """pulsar.py:86-105: resample the profile to Nph phases, scale by
        (f/ref)^specidx, wrap it as a DataPortrait (PCHIP)."""
        C = (np.asarray(signal._freqs_MHz()) / float(to_value(self.ref_freq, 'MHz'))) ** self.specidx
        C = np.reshape(C, (signal.Nchan, 1))
        Nph = self._nph(signal)
        self.Profiles.init_profiles(Nph, Nchan=signal.Nchan)
        full_profs = self.Profiles.calc_profiles(np.linspace(0.0, 1.0, Nph), Nchan=signal.Nchan)
        rs = getattr(signal, "_rowset", None)
        if is_uniform(full_profs) and np.all(C == 1.0):
            rs = None     # x 1.0 is the identity: the uniform table stays one row
        else:
            if rs is not None:
                # shard-local planning: this rank's rows (and their factors)
                if getattr(self.Profiles, "_rowset", None) is None and full_profs.shape[0] == signal.Nchan:
                    full_profs = np.array(full_profs[rs.gids])
                if full_profs.shape[0] == rs.gids.size:
                    C = C[rs.gids]
                else:
                    rs = None
            if is_uniform(full_profs) and C.shape[0] == full_profs.shape[0]:
                # the tiled row times C in one pass (the values of the
                # reference's copy-then-scale-in-place: x * C either way)
                full_profs = rows_of(full_profs) * C
            else:
                if is_uniform(full_profs):
                    full_profs = np.array(full_profs)
                full_profs *= C   # in place: a 1-row portrait with Nchan > 1 raises, as there
        self._Profiles = DataPortrait(full_profs, rowset=rs)

    def make_pulses(self, signal, tobs):
        """pulsar.py:107-151 (filterbank signals)."""
        signal._tobs = make_quant(tobs, 's')
        if self.ref_freq is None:
            self._ref_freq = signal.fcent
        if signal.sigtype == "FilterBankSignal":
            self._add_spec_idx(signal)
        Nph = self._nph(signal)
        self.Profiles.init_profiles(Nph, signal.Nchan)
        if signal.sigtype in ["RFSignal", "BasebandSignal"]:
            self._make_amp_pulses(signal)
        elif signal.sigtype == "FilterBankSignal":
            self._make_pow_pulses(signal)
        else:
            raise NotImplementedError("no pulse method for signal: {}".format(signal.sigtype))
        pr = self.Profiles._max_profile
        signal._Smax = self.Smean * len(pr) / np.sum(pr)

    def _make_amp_pulses(self, signal):
        """pulsar.py:153-183: data = sqrt(calc_profiles(phase(n))) x N(0, 1),
        phase(n) = n / (samprate P) mod 1, on the device: the profile's PCHIP
        table (DataProfile / DataPortrait, as in the reference's own baseband
        tests) evaluated per sample, Philox Box-Muller normals."""
        if signal.sigtype != "BasebandSignal":
            raise NotImplementedError("RFSignal is not built (baseband and filterbank only)")
        P = self._P()
        sr = signal._samprate_MHz()
        tobs = float(to_value(signal.tobs, 's'))
        call = _engine.next_call()
        inj = _engine.take_injection("gen")
        signal._nsamp = int((tobs * sr) * 1e6)
        spp = (sr * P) * 1e6
        inv = 1.0 / spp
        step = int(round(math.ldexp(inv - math.floor(inv), 64)))
        prof = self.Profiles
        if isinstance(prof, GaussPortrait) and np.ndim(prof.peak) <= 1:
            # analytic: the device sums the components at each sample's phase
            pk = np.atleast_1d(np.asarray(prof.peak, dtype=np.float64))
            wd = np.broadcast_to(np.asarray(prof.width, dtype=np.float64), pk.shape)
            am = np.broadcast_to(np.asarray(prof.amp, dtype=np.float64), pk.shape)
            comps = np.stack([pk, 1.0 / wd, am / float(prof.Amax), np.zeros_like(pk)], axis=1)
            src = _engine.Source("search", comps.astype(np.float32)[None], 1.0, 1.0, call, M=1,
                                 nint=len(pk), phase_step=step % (1 << 64), inj=inj)
            src.amp = "gauss"
        elif hasattr(prof, "device_table"):
            tab, M, nint, split = _device_table(prof)
            src = _engine.Source("search", _dedupe(tab), 1.0, 1.0, call, M=M, nint=nint,
                                 phase_step=step % (1 << 64), inj=inj, split=split)
            src.amp = "pchip"
        else:
            raise NotImplementedError("amplitude pulses from a %s" % type(prof).__name__)
        signal._ncols = int(signal._nsamp)
        signal._pending = _engine.Pending(src)
        signal._row0 = None
        # new data: an earlier null()'s tie error / pending checks no longer apply
        signal._null_error = None
        signal._null_checks = []

    def _make_pow_pulses(self, signal):
        """pulsar.py:185-244: fold -> tile(profiles, nsub) x chi2(Nfold);
        search -> PCHIP(phase(n)) x chi2(1).  Recorded as the source stage."""
        P = self._P()
        sr = signal._samprate_MHz()
        tobs = float(to_value(signal.tobs, 's'))
        call = _engine.next_call()
        inj = _engine.take_injection("gen")
        if signal.fold:
            if signal.sublen is None:
                signal._sublen = signal.tobs
                signal._nsub = 1
            else:
                signal._nsub = int(np.round(tobs / float(to_value(signal.sublen, 's'))))
            signal._nsamp = int((signal._nsub * (P * sr)) * 1e6)
            table = np.asarray(self.Profiles(), dtype=np.float64)
            Nph = table.shape[1]
            nfold = float(to_value(signal.sublen, 's')) / P
            signal._Nfold = Quantity(nfold, '')
            signal._set_draw_norm(df=nfold)
            ncols = Nph * signal._nsub
            src = _engine.Source("fold", _dedupe(table).astype(np.float32), nfold,
                                 signal._draw_norm, call, nph=Nph, inj=inj, row_ids=_row_ids(self.Profiles))
        else:
            signal._sublen = self.period
            signal._nsub = int(np.round(tobs / P))
            signal._set_draw_norm(df=1)
            signal._nsamp = int((tobs * sr) * 1e6)
            ncols = signal._nsamp
            tab, M, nint, split = _device_table(self.Profiles)
            tab = _dedupe(tab)
            spp = (sr * P) * 1e6                      # samples per period
            inv = 1.0 / spp                           # cycles per sample
            step = int(round(math.ldexp(inv - math.floor(inv), 64)))
            src = _engine.Source("search", tab, 1.0, signal._draw_norm, call, M=M, nint=nint,
                                 phase_step=step % (1 << 64), inj=inj, row_ids=_row_ids(self.Profiles),
                                 split=split)
        signal._ncols = int(ncols)
        signal._pending = _engine.Pending(src)
        signal._row0 = None
        # new data: an earlier null()'s tie error / pending checks no longer apply
        signal._null_error = None
        signal._null_checks = []

    def null(self, signal, null_frac, length=None, frequency=None):
        """pulsar.py:246-333."""
        null_pulses = int(np.round(signal.nsub * null_frac))
        Nph = self._nph(signal)
        opw = self.Profiles._calcOffpulseWindow(Nphase=Nph)
        if signal.fold:
            df = float(signal.Nfold)
        else:
            df = 1.0
        if not signal.fold or float(signal.Nfold) < 100:
            check_df = 100.0
        else:
            check_df = float(signal.Nfold)
        pend = signal._pending if signal._pending is not None else _engine.Pending(None)
        if pend.null is not None or pend.noise is not None:
            signal._flush()
            pend = _engine.Pending(None)
        # shift_val = Nph//2 - argmax(channel 0, first Nph samples), on the
        # device: no host round trip (a non-unique maximum raises on the
        # first read of the data, see _engine.check_null_status)
        shift_dev = _engine.null_shift_device(signal, pend, Nph)
        if length is not None or frequency is not None:
            raise NotImplementedError("Length and Frequency not been implimented yet")
        signal._null_checks = getattr(signal, "_null_checks", []) + [(shift_dev, Nph)]
        call = _engine.next_call()
        rand_pulses = _engine.take_injection("null_pulses")
        if rand_pulses is None:
            rand_pulses = _engine.host_rng(call).choice(signal.nsub, null_pulses, replace=False)
        rand_pulses = np.asarray(rand_pulses, dtype=np.int64)
        rank = np.full(max(int(signal.nsub), 1), -1, dtype=np.int32)
        if np.unique(rand_pulses).size == rand_pulses.size:
            rank[rand_pulses] = np.arange(rand_pulses.size, dtype=np.int32)
        else:
            for r, p in enumerate(rand_pulses):      # repeats: the later entry wins, as there
                rank[p] = r
        opm = float(np.mean(self.Profiles._max_profile[opw.astype(int)]))
        dn = float(signal._draw_norm)
        st = {"rank": rank, "shift_dev": shift_dev, "nph": Nph, "call_id": call,
              "inj_box": _engine.take_injection("box"), "inj_rep": _engine.take_injection("rep")}
        if null_pulses == 0 or rand_pulses.size == 0:
            return
        if signal.delay is None:
            st.update(mode="undelayed", box_df=df, box_scale=dn * opm)
            if signal._pending is None:
                signal._pending = _engine.Pending(None)
            signal._pending.null = st
            return
        total_ms = np.asarray(to_value(signal.delay, 'ms'), dtype=np.float64)
        mask_samples = total_ms / signal._dt_ms()
        st.update(mode="delayed", box_df=check_df, box_scale=dn, rep_df=df, rep_scale=dn * opm,
                  mask_samples=mask_samples)
        pend = signal._pending
        if pend is not None and pend.shifts:
            fused = np.sum(pend.shifts, axis=0)
            if np.allclose(fused, mask_samples, rtol=1e-12, atol=1e-9):
                pend.null = st
                return
        # the data already carries (part of) the delay: shift only the mask
        signal._flush()
        signal._pending = _engine.Pending(None)
        signal._pending.null = st


def _device_table(portrait):
    """(table, M, nint, split): uniform knots -> split None; non-uniform
    knots -> the split-cell table (DataPortrait.split_table), nint = M.

    The device table always covers the whole period (nint == M): when the
    knots stop short of phase 1 (arange(N)/N, portraits.py:231-240) the
    reference extrapolates with the last piece (scipy's default), so the
    intervals k = nint .. M-1 get that cubic re-expanded in their own local
    coordinate, c(u + m) with m = k - nint + 1, in float64.  The kernels then
    need no extrapolation branch per sample."""
    tab, M, third = portrait.device_table(room=True)
    if np.ndim(third) == 1:
        return tab, M, M, np.asarray(third, dtype=np.float32)
    nint = int(third)
    if nint < M:
        from .portraits import rows_of
        h = 1.0 / M
        amax = portrait.Amax if hasattr(portrait, '_Amax') else 1.0
        x = portrait._knots
        if getattr(portrait, "_coef_cache", None) is None and x.size >= 4:
            # the last piece only: its slopes come from the last four knots
            # (an interior slope and the end slope), so the PCHIP through
            # those gives that piece bit for bit without fitting every interval
            from .portraits import pchip_coefficients
            c = np.asarray(pchip_coefficients(x[-4:], rows_of(portrait._kvals)[:, -4:]), dtype=np.float64)[:, -1, :]
        else:
            c = np.asarray(rows_of(portrait._coef), dtype=np.float64)[:, nint - 1, :]
        d3, d2, d1, d0 = (c[:, 0] * h ** 3 / amax, c[:, 1] * h ** 2 / amax, c[:, 2] * h / amax, c[:, 3] / amax)
        ext = []
        for m in range(1, M - nint + 1):
            ext.append(np.stack([d3, 3 * d3 * m + d2, (3 * d3 * m + 2 * d2) * m + d1,
                                 ((d3 * m + d2) * m + d1) * m + d0], axis=-1))
        ext = np.stack(ext, axis=1).astype(np.float32)
        if np.shape(tab)[1] == M:
            tab[:, nint:, :] = ext         # (the table came with room for them)
        else:
            tab = np.concatenate([np.asarray(tab, dtype=np.float32), ext], axis=1)
    return tab, M, M, None


def _row_ids(portrait):
    """Global channels of a shard-local portrait's rows (None: band-wide)."""
    f = getattr(portrait, "row_ids", None)
    return f() if f is not None else None


def _dedupe(tab):
    """One shared row when every channel's table is identical."""
    if is_uniform(tab):
        return np.ascontiguousarray(tab[0:1])
    # (row 1 against row 0 first: per-channel tables differ there already)
    if tab.shape[0] > 1 and np.array_equal(tab[1], tab[0]) and np.all(tab == tab[0:1]):
        return np.ascontiguousarray(tab[0:1])
    return np.ascontiguousarray(tab)
