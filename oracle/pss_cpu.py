"""pss_cpu -- CPU ORACLE for PsrSigSim's filterbank synthesis path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker / the timed CPU baseline -- never as the product.  The product
(``psrsigsim_amd``) runs exclusively through the HIP library and fails loudly
without it.

This is a from-scratch float64 NumPy restatement of the reference's algorithm,
written from reading /root/reference (cited file:line per function), keeping
the reference's *call structure* (per-channel ``np.fft.rfft``/``irfft`` delay
loop, legacy ``RandomState`` chi-square draws, scipy PCHIP) so that it is both
a faithful checker and an honest single-threaded CPU baseline.

Parity pinning: every function here is checked against golden vectors recorded
from the unmodified reference (``tests/golden/make_golden.py`` ->
``tests/golden/fixtures``) by ``tests/test_oracle_golden.py``; random draws are
replayed from the fixtures ("draw injection") so the comparisons are exact.

Units: everything is plain float64 in the reference's working units --
frequencies MHz, times s (delays ms, as the reference stores them), flux Jy,
temperatures K.
"""
import numpy as np
from scipy import stats
from scipy.interpolate import PchipInterpolator
import scipy.signal as spsig

DM_K = 1.0 / 2.41e-4          # MHz^2 s cm^3 / pc     (utils/constants.py:13)
KOLMOGOROV_BETA = 11.0 / 3    # (utils/constants.py:16)
KB_RADIO = 1.38064852e+03     # Jy m^2 / K           (telescope/telescope.py:12)


# ---------------------------------------------------------------------------
# draw providers
# ---------------------------------------------------------------------------
class LegacyDraws(object):
    """Draws from the global legacy numpy RandomState, exactly as scipy's
    ``chi2(df).rvs(size)`` (= ``RandomState.chisquare``) and
    ``np.random.choice`` consume it in the reference."""

    def __init__(self, seed=None, state=None):
        self.rs = state if state is not None else np.random.RandomState(seed)
        self.log = []

    def chi2(self, df, size):
        a = self.rs.chisquare(float(df), size)
        self.log.append(("chi2", float(df), np.array(a)))
        return a

    def choice(self, n, k):
        a = self.rs.choice(int(n), int(k), replace=False)
        self.log.append(("choice", float(n), np.array(a)))
        return a

    def normal(self, size):
        """scipy ``norm().rvs(size)`` = ``RandomState.standard_normal``
        (pulsar.py:166, 183)."""
        a = self.rs.standard_normal(size)
        self.log.append(("normal", 0.0, np.array(a)))
        return a


class InjectedDraws(object):
    """Replays a recorded list of (kind, df, array) in order; checks kind, df
    and size so a divergence in call structure is caught immediately."""

    def __init__(self, draws):
        self.draws = list(draws)
        self.i = 0

    def _next(self, kind, df, size):
        k, d, a = self.draws[self.i]
        self.i += 1
        if k != kind:
            raise AssertionError("draw %d: expected %s got %s" % (self.i - 1, kind, k))
        if kind == "chi2" and not np.isclose(d, float(df), rtol=1e-12, atol=0):
            raise AssertionError("draw %d: df %r != %r" % (self.i - 1, d, df))
        want = tuple(np.atleast_1d(size)) if np.ndim(size) else (int(size),)
        if tuple(a.shape) != want:
            raise AssertionError("draw %d: shape %r != %r" % (self.i - 1, a.shape, want))
        return np.array(a)

    def chi2(self, df, size):
        return self._next("chi2", df, size)

    def choice(self, n, k):
        return self._next("choice", n, k)

    def normal(self, size):
        return self._next("normal", 0.0, size)


# ---------------------------------------------------------------------------
# utils (utils/utils.py)
# ---------------------------------------------------------------------------
def shift_t(y, shift, dt=1):
    """utils/utils.py:17-59: integer roll when (int shift and dt == 1), else
    rfft -> exp(-2 pi i f shift) -> irfft (no ``n=``: odd N loses a sample)."""
    if isinstance(shift, int) and dt == 1:
        return np.roll(y, shift)
    spec = np.fft.rfft(y)
    f = np.fft.rfftfreq(len(y), d=dt)
    return np.fft.irfft(spec * np.exp(-2j * np.pi * f * shift))


def down_sample(ar, fact):
    """utils/utils.py:62-68."""
    return ar.reshape(-1, fact).mean(axis=1)


def rebin(ar, newlen):
    """utils/utils.py:71-91: ceil-edged windows, nan-padded, nanmean."""
    edges = np.linspace(0, ar.size, newlen, endpoint=False)
    stride = edges[1] - edges[0]
    width = int(np.ceil(stride))
    tmp = np.full((newlen, width), np.nan)
    for i, lo in enumerate(edges):
        hi = min(int(np.ceil(lo + stride)), ar.size)
        lo = int(np.ceil(lo))
        tmp[i, :hi - lo] = ar[lo:hi]
    return np.nanmean(tmp, axis=1)


# ---------------------------------------------------------------------------
# signal (signal/fb_signal.py)
# ---------------------------------------------------------------------------
class Signal(object):
    """State of a FilterBankSignal (signal/fb_signal.py:64-121)."""

    def __init__(self, fcent, bw, nchan=512, samprate=None, sublen=None,
                 dtype=np.float32, fold=True):
        self.fcent = float(fcent)
        self.bw = abs(float(bw))
        self.fold = fold
        self.sublen = float(sublen) if (fold and sublen is not None) else sublen
        # (fb_signal.py:91-92) default 1/20.48 us expressed in MHz
        self.samprate = (1.0 / 20.48) if samprate is None else float(samprate)
        self.nchan = int(nchan)
        first = self.fcent - self.bw / 2
        last = self.fcent + self.bw / 2
        self.dat_freq = np.arange(first, last, self.bw / self.nchan)   # lower edges
        self.dtype = dtype
        self.draw_max = None
        self.draw_norm = 1
        self.set_draw_norm()
        self.delay = None       # accumulated delay [ms] (None until a shift)
        self.dm = None
        self.dispersed = False
        self.data = None
        self.tobs = self.nsamp = self.nsub = self.Nfold = self.Smax = None

    def set_draw_norm(self, df=1):
        """fb_signal.py:114-121 (identity tests on the dtype, as there)."""
        if self.dtype is np.float32:
            self.draw_max = 200
            self.draw_norm = 1
        if self.dtype is np.int8:
            limit = stats.chi2.ppf(0.999, df)
            self.draw_max = np.iinfo(np.int8).max
            self.draw_norm = self.draw_max / limit


# ---------------------------------------------------------------------------
# profiles (pulsar/portraits.py, pulsar/profiles.py)
# ---------------------------------------------------------------------------
def _gauss_1d(ph, peak, width, amp):
    if np.any(ph > 1) or np.any(ph < 0):                 # portraits.py:279-280
        raise ValueError('Phase values must all lie within [0,1].')
    return amp * np.exp(-0.5 * ((ph - peak) / width) ** 2)


def _gauss_multi(ph, peaks, widths, amps):
    if np.any(ph > 1) or np.any(ph < 0):                 # portraits.py:285-286
        raise ValueError('Phase values must all lie within [0,1].')
    g = amps[:, None] * np.exp(-0.5 * ((ph[None, :] - peaks[:, None]) / widths[:, None]) ** 2)
    return g.sum(axis=0)


class _Portrait(object):
    _Amax = None
    _profiles = None
    _max_profile = None

    def __call__(self):
        return self._profiles

    def _pick_max_profile(self):
        # portraits.py:45 -- first row whose max is exactly 1.0
        self._max_profile = [p for p in self._profiles if p.max() == 1.0][0]

    def offpulse_window(self, Nphase):
        """portraits.py:62-82: argmin of a sliding trapezoid of width Nph/8."""
        ws = Nphase / 8
        half = ws // 2
        integral = np.zeros_like(self._max_profile)
        for i in np.arange(0, Nphase):
            win = np.arange(i - half, i + half) % Nphase
            integral[i] = np.trapezoid(self._max_profile[win.astype(int)])
        m = np.argmin(integral)
        return np.arange(m - half, m + half + 1) % Nphase


class GaussPortrait(_Portrait):
    """portraits.py:94-198 (GaussProfile = the same class, profiles.py:68-97)."""

    def __init__(self, peak=0.5, width=0.05, amp=1):
        self.peak, self.width, self.amp = peak, width, amp

    def calc(self, phases, nchan=None):
        ph = np.array(phases)
        if hasattr(self.peak, 'ndim') and self.peak.ndim == 2:
            prof = np.array([_gauss_multi(ph, self.peak[:], self.width[:], self.amp[:])
                             for _ in range(self.peak.shape[0])])
        else:
            if nchan is None:
                raise ValueError('Nchan must be provided if only 1-dim profile information provided.')
            if hasattr(self.peak, 'ndim') and self.peak.ndim == 1:
                one = _gauss_multi(ph, self.peak, self.width, self.amp)
            else:
                one = _gauss_1d(ph, self.peak, self.width, self.amp)
            prof = np.tile(one, (nchan, 1))
        if self._Amax is None:                            # portraits.py:177
            self._Amax = np.amax(prof)
        return prof / self._Amax

    def init_profiles(self, Nphase, nchan=None):
        """portraits.py:131-140 (no renormalisation here)."""
        self._profiles = self.calc(np.arange(Nphase) / Nphase, nchan)
        self._pick_max_profile()


class DataPortrait(_Portrait):
    """portraits.py:200-267: PCHIP generator over (possibly closed) knots."""

    def __init__(self, profiles, phases=None):
        profiles = np.asarray(profiles, dtype=float)
        if np.any(profiles < 0.0):                        # portraits.py:224-229
            for row in profiles:
                row[row < 0.0] = 0.0
        if phases is None:
            n = profiles.shape[1]
            if np.any(profiles[:, 0] != profiles[:, -1]):
                profiles = np.append(profiles, profiles[:, :1], axis=1)
                phases = np.arange(n + 1) / n
            else:
                phases = np.arange(n) / n
        else:
            phases = np.asarray(phases, dtype=float)
            if phases[-1] != 1:
                phases = np.append(phases, 1)
                profiles = np.append(profiles, profiles[:, :1], axis=1)
            elif np.any(profiles[:, 0] != profiles[:, -1]):
                profiles[:, -1] = profiles[:, 0]
        self.knot_x = phases
        self.knot_y = profiles
        self.gen = PchipInterpolator(phases, profiles, axis=1)

    def calc(self, phases, nchan=None):
        out = self.gen(phases)
        amax = self._Amax if self._Amax is not None else np.max(out)
        return out / amax

    def init_profiles(self, Nphase, nchan=None):
        """portraits.py:32-45: evaluate, renormalise to max 1, cache Amax."""
        self._profiles = self.calc(np.arange(Nphase) / Nphase, nchan)
        self._Amax = self._profiles.max()
        self._profiles = self._profiles / self._Amax
        self._pick_max_profile()


def DataProfile(profile, phases=None, nchan=None):
    """profiles.py:155-188: 1-D template tiled to ``nchan`` rows (default 1).
    Negative bins are zeroed through ``np.where(...)[0]`` exactly as there."""
    profile = np.array(profile, dtype=float)
    if np.any(profile < 0.0):
        profile[np.where(profile < 0.0)[0]] = 0.0
    if profile.ndim == 1:
        profile = np.tile(profile, (1 if nchan is None else nchan, 1))
    return DataPortrait(profile, phases)


# ---------------------------------------------------------------------------
# pulsar (pulsar/pulsar.py)
# ---------------------------------------------------------------------------
class Pulsar(object):
    def __init__(self, period, Smean, profiles=None, specidx=0.0, ref_freq=None):
        self.period = float(period)
        self.Smean = float(Smean)
        self.specidx = specidx
        self.ref_freq = None if ref_freq is None else float(ref_freq)
        self.Profiles = GaussPortrait() if profiles is None else profiles


def nph_of(sig, psr):
    """``int((samprate * period).decompose())`` (pulsar.py:96, 124)."""
    return int((sig.samprate * psr.period) * 1e6)


def add_spec_idx(sig, psr):
    """pulsar.py:86-105."""
    C = ((sig.dat_freq / psr.ref_freq) ** psr.specidx).reshape(sig.nchan, 1)
    Nph = nph_of(sig, psr)
    psr.Profiles.init_profiles(Nph, sig.nchan)
    full = psr.Profiles.calc(np.linspace(0.0, 1.0, Nph), sig.nchan)
    full *= C          # in place: raises for a 1-row portrait and Nchan > 1
    psr.Profiles = DataPortrait(full)


def make_pulses(sig, psr, tobs, draws):
    """pulsar.py:107-151 + _make_pow_pulses 185-244 (filterbank only)."""
    sig.tobs = float(tobs)
    if psr.ref_freq is None:
        psr.ref_freq = sig.fcent
    add_spec_idx(sig, psr)
    Nph = nph_of(sig, psr)
    psr.Profiles.init_profiles(Nph, sig.nchan)
    if sig.fold:
        if sig.sublen is None:
            sig.sublen = sig.tobs
            sig.nsub = 1
        else:
            sig.nsub = int(np.round(sig.tobs / sig.sublen))
        sig.nsamp = int((sig.nsub * (psr.period * sig.samprate)) * 1e6)
        tiled = np.tile(psr.Profiles(), sig.nsub)
        sig.Nfold = sig.sublen / psr.period
        sig.set_draw_norm(df=sig.Nfold)
        sig.data = tiled * draws.chi2(sig.Nfold, tiled.shape) * sig.draw_norm
    else:
        sig.sublen = psr.period
        sig.nsub = int(np.round(sig.tobs / sig.sublen))
        sig.set_draw_norm(df=1)
        sig.nsamp = int((sig.tobs * sig.samprate) * 1e6)
        phs = np.arange(sig.nsamp) / ((sig.samprate * psr.period) * 1e6)
        phs %= 1
        full = psr.Profiles.calc(phs, sig.nchan)
        sig.data = full * draws.chi2(1, (sig.nchan, sig.nsamp)) * sig.draw_norm
    pr = psr.Profiles._max_profile
    sig.Smax = psr.Smean * len(pr) / np.sum(pr)


class BasebandSignal(object):
    """State of a BasebandSignal (signal/bb_signal.py:34-52): Nchan
    polarisation channels, default sample rate 2 bw (Nyquist)."""

    def __init__(self, fcent, bw, samprate=None, dtype=np.float32, nchan=2):
        self.fcent = float(fcent)
        self.bw = float(bw)
        self.nchan = int(nchan)
        self.samprate = 2 * self.bw if samprate is None else float(samprate)
        self.dtype = dtype
        self.delay = None
        self.dm = None
        self.dispersed = False
        self.data = None
        self.tobs = self.nsamp = self.Smax = None


def make_amp_pulses(sig, psr, tobs, draws):
    """pulsar.py:107-151 (no spectral index for baseband) + _make_amp_pulses
    153-183: sqrt(calc_profiles(n / (samprate P) mod 1)) x N(0, 1)."""
    sig.tobs = float(tobs)
    if psr.ref_freq is None:
        psr.ref_freq = sig.fcent
    Nph = nph_of(sig, psr)
    psr.Profiles.init_profiles(Nph, sig.nchan)
    sig.nsamp = int((sig.tobs * sig.samprate) * 1e6)
    phs = np.arange(sig.nsamp) / ((sig.samprate * psr.period) * 1e6)
    phs %= 1
    full = np.sqrt(psr.Profiles.calc(phs, sig.nchan))
    sig.data = full * draws.normal((sig.nchan, sig.nsamp))
    pr = psr.Profiles._max_profile
    sig.Smax = psr.Smean * len(pr) / np.sum(pr)


def baseband_transfer(sig, dm, N):
    """H on the rfft bins of an N-sample row (ism.py:84-93): u =
    rfftfreq(2 len(rfft) - 1, dt[s]) -- Hz values labelled MHz by
    make_quant -- f = u - bw/2, H = exp(2 pi i DM_K dm f^2 / ((f + f0)
    f0^2)), the exponent's MHz s converted to 1e6."""
    dt_s = (1.0 / sig.samprate) * 1e-6
    u = np.fft.rfftfreq(2 * (N // 2 + 1) - 1, d=dt_s)
    f = u - sig.bw / 2.0
    return np.exp(1j * 2 * np.pi * (DM_K / ((f + sig.fcent) * sig.fcent ** 2) * dm * f ** 2 * 1e6))


def disperse_baseband(sig, dm):
    """ism.py:20-38, 76-98: per channel irfft(rfft(x) H)."""
    if sig.dispersed:
        raise ValueError('Signal has already been dispersed!')
    sig.dm = float(dm)
    H = baseband_transfer(sig, sig.dm, sig.data.shape[1])
    for x in range(sig.nchan):
        sig.data[x] = np.fft.irfft(np.fft.rfft(sig.data[x]) * H)
    sig.dispersed = True


def null(sig, psr, null_frac, draws, length=None, frequency=None):
    """pulsar.py:246-333 (both branches)."""
    npulse = int(np.round(sig.nsub * null_frac))
    Nph = nph_of(sig, psr)
    opw = psr.Profiles.offpulse_window(Nph)
    df = sig.Nfold if sig.fold else 1
    check_df = 100 if (not sig.fold or sig.Nfold < 100) else sig.Nfold
    row0 = sig.data[0, :Nph]
    shift_val = Nph // 2 - np.where(row0 == np.max(row0))[0]
    if length is not None or frequency is not None:
        raise NotImplementedError("Length and Frequency not been implimented yet")
    pulses = draws.choice(sig.nsub, npulse)
    N = sig.data.shape[1]
    opm = np.mean(psr.Profiles._max_profile[opw.astype(int)])
    box_row = np.zeros(N)          # test-side record of the (pre-shift) box values
    rep_dense = None
    mask_shifted = None
    if sig.delay is None:
        for p in pulses:
            bins = np.arange(Nph * p, Nph * (p + 1)) + shift_val
            bins = bins[bins < N]
            noise = draws.chi2(df, len(bins)) * sig.draw_norm
            sig.data[:, bins] = noise * opm
            box_row[bins] = noise * opm
    else:
        mask = np.zeros(sig.data.shape)
        for p in pulses:
            bins = np.arange(Nph * p, Nph * (p + 1)) + shift_val
            bins = bins[bins < N]
            mask[:, bins] = draws.chi2(check_df, len(bins)) * sig.draw_norm
        box_row[:] = mask[0]
        dt_ms = (1.0 / sig.samprate) * 1e-3     # (1/samprate).to('ms')
        for c in range(sig.nchan):
            mask[c, :] = shift_t(mask[c, :], sig.delay[c], dt=dt_ms)
        mask_shifted = mask
        hit = np.where(mask > 1)
        if hasattr(draws, "chi2_at"):
            # test hook: a provider that keys its draws by position (the
            # device's counter-based Philox, replayed), given the positions
            noise = draws.chi2_at(df, hit) * sig.draw_norm
        else:
            noise = draws.chi2(df, np.shape(hit)[1]) * sig.draw_norm
        sig.data[hit] = noise * opm
        rep_dense = np.zeros(sig.data.shape)
        rep_dense[hit] = noise * opm
    return {"shift_val": shift_val, "pulses": pulses, "opw": opw, "opm": opm,
            "box_row": box_row, "rep_dense": rep_dense, "mask_shifted": mask_shifted}


# ---------------------------------------------------------------------------
# ism (ism/ism.py)
# ---------------------------------------------------------------------------
def _accumulate(sig, delays_ms):
    sig.delay = np.array(delays_ms, dtype=float) if sig.delay is None else sig.delay + delays_ms


def _shift_channels(sig, delays_ms):
    dt_ms = (1.0 / sig.samprate) * 1e-3
    for c in range(sig.nchan):
        sig.data[c, :] = shift_t(sig.data[c, :], float(delays_ms[c]), dt=dt_ms)


def dm_delays_ms(sig, dm):
    """ism.py:42-43: DM_K * dm * f^-2 with f the channel lower edge, in ms."""
    return (DM_K * dm * np.power(sig.dat_freq, -2.0)) * 1e3


def disperse(sig, dm):
    """ism.py:20-74 (filterbank)."""
    sig.dm = float(dm)
    if sig.dispersed:
        raise ValueError('Signal has already been dispersed!')
    d = dm_delays_ms(sig, dm)
    _accumulate(sig, d)
    _shift_channels(sig, d)
    sig.dispersed = True
    return d


def fd_delays_ms(sig, FD_params):
    """ism.py:113-121: sum_i FD_i[s] * 1e3 * ln(f/1000 MHz)^(i+1)."""
    d = np.zeros(sig.nchan)
    for i, c in enumerate(FD_params):
        d += (float(c) * 1e3) * np.power(np.log(sig.dat_freq / 1000.0), i + 1)
    return d


def FD_shift(sig, FD_params):
    """ism.py:100-156."""
    d = fd_delays_ms(sig, FD_params)
    _accumulate(sig, d)
    _shift_channels(sig, d)
    return d


def scale_tau_d(tau_d, nu_i, nu_f, beta=KOLMOGOROV_BETA):
    """ism.py:340-358."""
    if beta < 4:
        exp = -2.0 * beta / (beta - 2)
    elif beta > 4:
        exp = -8.0 / (6 - beta)
    return tau_d * (nu_f / nu_i) ** exp


def scatter_broaden(sig, tau_d, ref_freq, beta=KOLMOGOROV_BETA, convolve=False, pulsar=None):
    """ism.py:158-240.  tau_d in s; delays stored in ms."""
    tau_ms = scale_tau_d(float(tau_d) * 1e3, float(ref_freq), sig.dat_freq, beta)
    if not convolve:
        _accumulate(sig, tau_ms)
        _shift_channels(sig, tau_ms)
        return tau_ms
    Nph = nph_of(sig, pulsar)
    pulsar.Profiles.init_profiles(Nph, sig.nchan)
    full = pulsar.Profiles.calc(np.linspace(0.0, 1.0, Nph), sig.nchan)
    t = np.linspace(0, pulsar.period, Nph)
    tails = np.zeros((sig.nchan, Nph))
    for c in range(sig.nchan):
        tails[c, :] = np.exp(-t * 1e3 / tau_ms[c])      # t[s] / tau[ms]
    pulsar.Profiles = DataPortrait(convolve_profile(full, tails, width=Nph))
    return tau_ms


def convolve_profile(profiles, kernels, width=2048):
    """ism.py:243-288: linear FFT convolution of normalised rows, truncated
    to ``width`` and rescaled by the profile sum."""
    for c in range(kernels.shape[0]):
        ps = np.sum(profiles[c, :])
        pn = profiles[c, :] / ps if ps != 0.0 else profiles[c, :]
        ks = np.sum(kernels[c, :])
        kn = kernels[c, :] / ks if ks != 0.0 else kernels[c, :]
        conv = spsig.convolve(pn, kn, mode='full', method='fft')
        profiles[c, :] = ps * conv[:width]
    return profiles


# ---------------------------------------------------------------------------
# telescope (telescope/telescope.py, receiver.py, backend.py)
# ---------------------------------------------------------------------------
class System(object):
    """A (Receiver, Backend) pair.  ``samprate_scale`` is the Hz-per-unit of
    the unit the backend sample rate was given in (1e6 for the MHz floats of
    the presets; 1.0 for a ``1/Quantity(s)`` as in tests/test_telescope.py):
    observe's float comparisons happen in that unit (see observe_branch)."""

    def __init__(self, rcvr_Trec=35.0, backend_samprate=12.5, samprate_scale=1e6):
        self.Trec = float(rcvr_Trec)
        self.backend_samprate = float(backend_samprate)
        self.samprate_scale = float(samprate_scale)


class Telescope(object):
    """telescope.py:14-38: gain = area / (2 kB) in K/Jy."""

    def __init__(self, aperture, area=None, Tsys=None):
        self.area = np.pi * (aperture / 2) ** 2 if area is None else float(area)
        self.gain = self.area / (2 * KB_RADIO)
        self.Tsys = None if Tsys is None else float(Tsys)
        self.systems = {}


def GBT():
    t = Telescope(100.0, area=5500.0, Tsys=35.0)          # telescope.py:192-205
    for name, sr in (("820_GUPPI", 3.125), ("Lband_GUPPI", 12.5),
                     ("800_GASP", 0.25), ("Lband_GASP", 0.25)):
        t.systems[name] = System(35.0, sr)
    return t


def Arecibo():
    t = Telescope(300.0, area=22000.0, Tsys=35.0)         # telescope.py:215-237
    for name, sr in (("430_PUPPI", 1.5625), ("Lband_PUPPI", 12.5),
                     ("Sband_PUPPI", 12.5), ("327_ASP", 0.25), ("430_ASP", 0.25),
                     ("Lband_ASP", 0.25), ("Sband_ASP", 0.25)):
        t.systems[name] = System(35.0, sr)
    return t


def noise_norm(sig, psr, Tsys, gain):
    """receiver.py:140-172 scale factor: Tsys/gain/sqrt(2 dt bw/C) * draw_norm
    / Smax * nbins / sum(max_profile)."""
    nbins = sig.nsamp / sig.nsub
    dt = sig.sublen / nbins
    sigS = Tsys / gain / np.sqrt(2 * dt * (sig.bw / sig.nchan)) * 1e-3   # Jy
    U = 1.0 / (np.sum(psr.Profiles._max_profile) / nbins)
    return (sigS * sig.draw_norm / sig.Smax) * U


def radiometer_noise(sig, psr, draws, gain=1.0, Tsys=None, Tenv=None, Trec=35.0):
    """receiver.py:82-121 (filterbank)."""
    if Tsys is None and Tenv is None:
        Tsys = Trec
    elif Tenv is not None:
        if Tsys is not None:
            raise ValueError("specify EITHER Tsys OR Tenv, not both")
        Tsys = Tenv + Trec
    norm = noise_norm(sig, psr, Tsys, gain)
    df = sig.Nfold if sig.fold else 1
    sig.data = sig.data + norm * draws.chi2(df, sig.data.shape)
    return norm


def observe_branch(sig, backend_samprate, samprate_scale=1e6):
    """telescope.py:94-126 dt comparisons.  dt_tel = 1/(2*samprate) is in the
    inverse of the backend rate's unit U; dt_sig is in s.  Each comparison
    converts its second operand into the first operand's unit with the ratio
    of the two units' scales (as the reference's unit layer does), which is
    what decides the float ``==`` / ``%`` branch tests."""
    tel_scale = 1.0 / samprate_scale            # seconds per unit of dt_tel
    tel_to_s = tel_scale / 1.0
    s_to_tel = 1.0 / tel_scale
    dt_tel = 1 / (2 * backend_samprate)
    if sig.sublen is not None:
        dt_sig = sig.sublen / (sig.nsamp / sig.nsub)     # s
    else:
        dt_sig = sig.tobs / sig.nsamp
    if dt_sig == dt_tel * tel_to_s:
        return "copy", None
    dt_sig_t = dt_sig * s_to_tel
    if np.remainder(dt_tel, dt_sig_t) == 0:
        return "down", int(np.floor_divide(dt_tel, dt_sig_t))
    if dt_tel > dt_sig_t:
        return "rebin", int(np.floor_divide(sig.tobs, dt_tel * tel_to_s))
    return "copy", None


def observe(sig, psr, tel, system, draws, noise=False):
    """telescope.py:72-149 (filterbank); returns the clipped/cast ``out``."""
    sysobj = tel.systems[system]
    kind, arg = observe_branch(sig, sysobj.backend_samprate, sysobj.samprate_scale)
    if kind == "copy":
        out = np.array(sig.data, dtype=float)
    elif kind == "down":
        new_Nt = int(sig.nsamp // arg)
        out = np.zeros((sig.nchan, new_Nt))
        for c, row in enumerate(sig.data):
            out[c, :] = down_sample(row, arg)
    else:
        out = np.zeros((sig.nchan, arg))
        for c, row in enumerate(sig.data):
            out[c, :] = rebin(row, arg)
    if noise:
        radiometer_noise(sig, psr, draws, gain=tel.gain, Tsys=tel.Tsys, Trec=sysobj.Trec)
    out[out > sig.draw_max] = sig.draw_max
    return np.array(out, dtype=sig.dtype)


def backend_fold(sig, psr):
    """backend.py:34-49: Npbins from the *signal* sample rate; the reshape
    only succeeds for Nt == 2*Npbins (or 1.5*Npbins), else ValueError."""
    Nf, Nt = sig.data.shape
    Npbins = int((psr.period * 2 * sig.samprate) * 1e6)
    N_fold = Nt // Npbins
    return np.sum(sig.data[:, Npbins:Npbins * (N_fold + 1)].reshape(Nf, N_fold, Npbins // 2), axis=1)
