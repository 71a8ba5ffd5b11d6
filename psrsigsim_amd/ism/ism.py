"""ISM -- mirrors ``psrsigsim/ism/ism.py``.

Every delay method computes its per-channel delays on the host (float64, the
reference's formulas), accumulates ``signal._delay`` exactly as the reference
does, and appends a delay stage to the signal's pending pipeline.  Consecutive
delay stages run as ONE forward/inverse FFT pass on the GPU (the reference runs
one rfft/irfft pair per channel per call: ism.py:57-60, 136-139, 203-206).
"""
import numpy as np
import scipy.fft as _sp_fft

from ..utils.constants import DM_K_VALUE, KOLMOGOROV_BETA
from ..utils.utils import make_quant
from .._units import Quantity, to_value
from .. import _lib
from ..pulsar.portraits import DataPortrait, is_uniform
from .. import _engine

__all__ = ["ISM"]


def push_delay(signal, delays_ms):
    """Accumulate ``signal._delay`` (ms, ism.py:44-47) and append a delay
    stage of delays_ms / dt samples per channel."""
    delays_ms = np.asarray(delays_ms, dtype=np.float64)
    if signal.delay is None:
        signal._delay = Quantity(delays_ms.copy(), 'ms')
    else:
        signal._delay = Quantity(np.asarray(to_value(signal.delay, 'ms')) + delays_ms, 'ms')
    if signal._ncols % 2:
        # shift_t's irfft (no n=) returns N-1 samples; the row assignment fails
        raise ValueError("could not broadcast input array from shape (%d,) into shape (%d,)"
                         % (signal._ncols - 1, signal._ncols))
    pend = signal._pending
    if pend is not None and (pend.null is not None or pend.noise is not None):
        signal._flush()
        pend = None
    if pend is None:
        pend = signal._pend()
    pend.shifts.append(delays_ms / signal._dt_ms())


def push_tail(signal, a):
    """Append a scattering-tail filter stage (ISM.scatter_broaden(tail=True)):
    per channel decay factor a = exp(-dt/tau) of h[n] = (1 - a) a^n."""
    if signal._ncols % 2:
        raise ValueError("could not broadcast input array from shape (%d,) into shape (%d,)"
                         % (signal._ncols - 1, signal._ncols))
    pend = signal._pending
    if pend is not None and (pend.null is not None or pend.noise is not None or pend.tail is not None):
        signal._flush()
        pend = None
    if pend is None:
        pend = signal._pend()
    pend.tail = np.broadcast_to(np.asarray(a, dtype=np.float64), (signal.Nchan,)).copy()


class ISM(object):
    """ism.py:12-358 (filterbank path)."""

    def __init__(self):
        pass

    def disperse(self, signal, dm):
        """ism.py:20-38: cold-plasma delay DM_K * DM / f^2 per channel (f =
        channel lower edge), relative to infinite frequency."""
        signal._dm = make_quant(dm, 'pc/cm^3')
        if hasattr(signal, '_dispersed'):
            raise ValueError('Signal has already been dispersed!')
        if signal.sigtype == 'FilterBankSignal':
            self._disperse_filterbank(signal, signal._dm)
        elif signal.sigtype == 'BasebandSignal':
            self._disperse_baseband(signal, signal._dm)
        signal._dispersed = True

    def _disperse_filterbank(self, signal, dm):
        """ism.py:40-74; delays in ms."""
        f = signal._freqs_MHz()
        delays_ms = (DM_K_VALUE * float(to_value(dm, 'pc/cm^3')) * np.power(f, -2.0)) * 1e3
        push_delay(signal, delays_ms)

    def _disperse_baseband(self, signal, dm):
        """ism.py:76-98: per channel irfft(rfft(x) * H), Lorimer & Kramer
        (2006) eq. 5.21, H = exp(2 pi i DM_K dm f^2 / ((f + f0) f0^2)), with
        the reference's frequency grid kept exactly: u = rfftfreq(N + 1, dt)
        (2 len(rfft) - 1 points) in Hz, labelled MHz by make_quant, f = u -
        bw/2.  H (N/2 + 1 bins, the same for every channel) is planned on the
        host in float64; the transforms run on the device."""
        N = signal._ncols
        if N % 2:
            raise ValueError("could not broadcast input array from shape (%d,) into shape (%d,)"
                             % (N - 1, N))
        f0 = float(to_value(signal.fcent, 'MHz'))
        bw = float(to_value(signal.bw, 'MHz'))
        u = np.fft.rfftfreq(2 * (N // 2 + 1) - 1, d=signal._dt_s())
        f = u - bw / 2.0
        # DM_K [MHz^2 s cm^3/pc] dm [pc/cm^3] f^2/((f+f0) f0^2) [1/MHz] -> MHz s = 1e6
        ph = DM_K_VALUE / ((f + f0) * f0 ** 2) * float(to_value(dm, 'pc/cm^3')) * f ** 2 * 1e6
        H = np.exp(1j * 2 * np.pi * ph)
        _engine.filter_rows(signal, H)

    def FD_shift(self, signal, FD_params):
        """ism.py:100-156: sum_i FD_i * ln(f / 1 GHz)^(i+1)."""
        f = signal._freqs_MHz()
        delays = np.zeros(len(f))
        for ii in range(len(FD_params)):
            c_ms = float(to_value(make_quant(FD_params[ii], 's'), 's')) * 1e3
            delays += c_ms * np.power(np.log(f / 1000.0), ii + 1)
        push_delay(signal, delays)
        signal._FDshifted = True

    def scatter_broaden(self, signal, tau_d, ref_freq, beta=KOLMOGOROV_BETA, convolve=False,
                        pulsar=None, *, tail=False):
        """ism.py:158-240.  convolve=False: a pure extra delay
        tau_d (f/f_ref)^(-2 beta/(beta-2)); convolve=True: linear convolution
        of each channel's profile with a normalised exp(-t/tau) tail (before
        make_pulses), replacing the pulsar's profile by a DataPortrait.

        ``tail=True`` (keyword-only EXTENSION, no reference counterpart --
        SURVEY.md App. A.11): scatter-broaden the time series itself -- every
        channel's samples circularly convolved with the normalised exponential
        (1 - a) a^n, a = exp(-dt / tau_c), tau_c scaled as above -- as the
        transfer function H(k) = (1 - a)/(1 - a e^{-2 pi i k/N}) applied in the
        same forward/inverse FFT pass as the delays (no extra HBM pass).  No
        delay is added to ``signal.delay`` (the tail is a filter)."""
        f = signal._freqs_MHz()
        ref = float(to_value(make_quant(ref_freq, 'MHz'), 'MHz'))
        tau_ms = float(to_value(make_quant(tau_d, 's'), 's')) * 1e3
        tau_scaled = self.scale_tau_d(tau_ms, ref, f, beta=beta)
        if tail:
            push_tail(signal, np.exp(-signal._dt_ms() / np.asarray(tau_scaled, dtype=np.float64)))
            return
        if not convolve:
            push_delay(signal, tau_scaled)
            return
        Nph = pulsar._nph(signal)
        pulsar.Profiles.init_profiles(Nph, signal.Nchan)
        full_profs = pulsar.Profiles.calc_profiles(np.linspace(0.0, 1.0, Nph), signal.Nchan)
        t = np.linspace(0, pulsar._P(), Nph)
        tau = np.atleast_1d(tau_scaled)
        rs = getattr(signal, "_rowset", None)
        if (rs is not None and tau.size == signal.Nchan and
                (getattr(pulsar.Profiles, "_rowset", None) is rs or full_profs.shape[0] == signal.Nchan)):
            # shard-local planning: convolve this rank's channels (+ the
            # channel-0 pair) only; the portrait's band-wide max and max row
            # are reductions over the plan group (shard.RowSet)
            if getattr(pulsar.Profiles, "_rowset", None) is not rs:
                full_profs = full_profs[rs.gids]
            full_profs = np.array(full_profs)
            taur = tau[rs.gids]
            pulsar._Profiles = DataPortrait(self._convolve_rows(
                full_profs, lambda a, b: np.exp(-(t[None, :] * 1e3) / taur[a:b, None]), Nph), rowset=rs)
            return
        # (a uniform table -- one profile tiled over the channels -- stays one
        # row through the convolution's profile side: _convolve_rows)

        def tails(a, b):
            # rows [a, b) of the exponential tails, t [s] / tau [ms]; rows past
            # tau.size zero (the reference's tails[:tau.size]); computed on
            # the convolution's row-block threads, elementwise as one array
            k = np.zeros((b - a, Nph))
            e = min(b, tau.size)
            if e > a:
                k[:e - a, :] = np.exp(-(t[None, :] * 1e3) / tau[a:e, None])
            return k

        pulsar._Profiles = DataPortrait(self._convolve_rows(full_profs, tails, Nph))

    def convolve_profile(self, profiles, convolve_array, width=2048):
        """ism.py:243-288: per row, linear convolution of the sum-normalised
        profile with the sum-normalised kernel, first `width` samples,
        rescaled by the profile sum.  Row blocks run on host threads (every
        step is row-wise: numpy and pocketfft release the GIL), so the
        per-signal planning of a 2048-channel band is not one core's work."""
        kern = np.asarray(convolve_array, dtype=float)
        return self._convolve_rows(profiles, lambda a, b: kern[a:b], width, rows=kern.shape[0])

    def _convolve_rows(self, profiles, kern_rows, width, rows=None):
        """convolve_profile with the kernel rows [a, b) from ``kern_rows(a,
        b)``, so scatter_broaden's tails are computed on the row-block
        threads too (bit for bit the same values)."""
        prof = np.asarray(profiles, dtype=float)
        rows = prof.shape[0] if rows is None else rows
        uni = is_uniform(prof)
        # scipy.signal.fftconvolve(pn, kn, mode='full', axes=1) stated through
        # its own transforms (signal/_signaltools.py _freq_domain_conv: real
        # FFTs of the next fast length >= the full length, product, inverse,
        # the leading columns): the same pocketfft calls and bits, without
        # fftconvolve's per-call argument handling, which holds the GIL the
        # row-block threads share (2048-channel convolution 8.0-8.7 -> 6.6-6.9
        # ms on this container)
        klen = np.shape(kern_rows(0, 1))[1] if rows > 0 else prof.shape[1]
        nfft = _sp_fft.next_fast_len(prof.shape[1] + klen - 1, True)
        if uni:
            # one profile for every channel (a tiled GaussProfile, C3): its
            # sum, normalisation and spectrum are computed once -- fftconvolve
            # broadcasts a 1-row operand over the rows, and every row's
            # arithmetic is the per-row arithmetic of the full table (the same
            # bits; tests/test_host_plan.py)
            prof = prof[:1]
            ps1 = np.sum(prof, axis=1, keepdims=True)
            pn1 = np.where(ps1 != 0.0, prof / np.where(ps1 != 0.0, ps1, 1.0), prof)
            sp1 = _sp_fft.rfftn(pn1, [nfft], axes=[1])
            out = np.empty((rows, width))
        else:
            out = profiles

        def block(a, b):
            kb = kern_rows(a, b)
            if uni:
                ps, sp = ps1, sp1
            else:
                ps = np.sum(prof[a:b], axis=1, keepdims=True)
                pn = np.where(ps != 0.0, prof[a:b] / np.where(ps != 0.0, ps, 1.0), prof[a:b])
                sp = _sp_fft.rfftn(pn, [nfft], axes=[1])
            ks = np.sum(kb, axis=1, keepdims=True)
            kn = np.where(ks != 0.0, kb / np.where(ks != 0.0, ks, 1.0), kb)
            # the reference's per-row scipy.signal.convolve(..., method='fft')
            # (it later makes exact float decisions on these values)
            conv = _sp_fft.irfftn(sp * _sp_fft.rfftn(kn, [nfft], axes=[1]), [nfft], axes=[1])
            out[a:b, :] = ps * conv[:, :width]

        _lib.host_rows(rows, block)
        return out

    def scale_dnu_d(self, dnu_d, nu_i, nu_f, beta=KOLMOGOROV_BETA):
        """ism.py:300-318."""
        if beta < 4:
            exp = 2.0 * beta / (beta - 2)
        elif beta > 4:
            exp = 8.0 / (6 - beta)
        return dnu_d * (nu_f / nu_i) ** exp

    def scale_dt_d(self, dt_d, nu_i, nu_f, beta=KOLMOGOROV_BETA):
        """ism.py:320-338."""
        if beta < 4:
            exp = 2.0 / (beta - 2)
        elif beta > 4:
            exp = float(beta - 2) / (6 - beta)
        return dt_d * (nu_f / nu_i) ** exp

    def scale_tau_d(self, tau_d, nu_i, nu_f, beta=KOLMOGOROV_BETA):
        """ism.py:340-358."""
        if beta < 4:
            exp = -2.0 * beta / (beta - 2)
        elif beta > 4:
            exp = -8.0 / (6 - beta)
        return tau_d * (nu_f / nu_i) ** exp
