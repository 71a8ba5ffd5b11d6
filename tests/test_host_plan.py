"""CPU checks of the host plan layer against the reference's golden vectors:
derived integers/scalars (nsamp, nsub, Nfold, Smax, draw_norm), channel
frequencies, accumulated delays, the device PCHIP table (evaluated on the
host exactly as the kernel does), the radiometer noise scale and observe's
branch decisions.  No GPU needed (stages are only recorded, not run)."""
import numpy as np
import pytest

from oracle import pss_cpu as O
from tests import replay
from tests.fixtures_util import load


def _product(name):
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile, DataProfile
    case = replay.CASES[name]
    sg = case["sig"]
    sig = FilterBankSignal(sg["fcent"], sg["bw"], Nsubband=sg["nchan"], sample_rate=sg.get("samprate"),
                           sublen=sg.get("sublen"), dtype=sg.get("dtype", np.float32),
                           fold=sg.get("fold", True))
    ps = case["psr"]
    spec = ps["prof"]
    if spec[0] == "gauss":
        prof = GaussProfile(*spec[1:])
    elif spec[0] == "gaussarr":
        prof = GaussProfile(np.array([0.3, 0.6]), np.array([0.02, 0.05]), np.array([0.5, 1.0]))
    else:
        prof = DataProfile(replay._prof(), Nchan=spec[1])
    psr = Pulsar(ps["period"], ps["Smean"], profiles=prof, specidx=ps.get("specidx", 0.0),
                 ref_freq=ps.get("ref_freq"))
    return case, sig, psr


@pytest.mark.parametrize("name", sorted(replay.CASES))
def test_derived_quantities(name):
    from psrsigsim_amd.ism import ISM
    meta, A, _ = load(name)
    case, sig, psr = _product(name)
    ism = ISM()
    for op in case["ops"]:
        if op[0] == "scatter_conv":
            ism.scatter_broaden(sig, op[1], op[2], convolve=True, pulsar=psr)
        elif op[0] == "make_pulses":
            psr.make_pulses(sig, op[1])
            break
    assert sig.nsamp == meta["nsamp"] and sig.nsub == meta["nsub"]
    if meta.get("Nfold") is not None:
        assert np.isclose(float(sig.Nfold), meta["Nfold"], rtol=1e-12)
    assert np.isclose(float(sig._Smax.value), meta["Smax"], rtol=1e-12)
    assert np.isclose(sig._draw_norm, meta["draw_norm"], rtol=1e-12)
    assert sig._draw_max == meta["draw_max"]
    np.testing.assert_array_equal(sig.dat_freq.value, A["dat_freq"])
    assert sig._ncols == A["data_pulses"].shape[1]
    np.testing.assert_allclose(psr.Profiles._max_profile, A["max_profile"], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("name", ["northstar_mini", "j1713_search", "null_undelayed"])
def test_device_pchip_table_matches_reference_generator(name):
    """The fp32 table the kernel evaluates (local coordinate u) reproduces the
    reference's PchipInterpolator coefficients (recorded) at every sample."""
    meta, A, _ = load(name)
    case, sig, psr = _product(name)
    from psrsigsim_amd.ism import ISM
    for op in case["ops"]:
        if op[0] == "scatter_conv":
            ISM().scatter_broaden(sig, op[1], op[2], convolve=True, pulsar=psr)
        elif op[0] == "make_pulses":
            psr.make_pulses(sig, op[1])
            break
    src = sig._pending.source
    tab = src.table.astype(np.float64)
    n = np.arange(sig._ncols, dtype=np.uint64)
    ph = (n * np.uint64(src.phase_step)).astype(np.uint64)          # wrapping, like the kernel
    hi = ((ph >> np.uint64(32)).astype(np.float64) * src.M) / 2.0 ** 32
    iv = np.minimum(np.floor(hi).astype(np.int64), src.nint - 1)
    u = hi - iv
    rows = tab[np.zeros(1, int) if tab.shape[0] == 1 else np.arange(tab.shape[0])]
    c = rows[:, iv, :]
    val = ((c[..., 0] * u + c[..., 1]) * u + c[..., 2]) * u + c[..., 3]
    # reference: data_pulses = PCHIP(phase) * chi2 draw  -> divide the draws out
    draws = load(name)[2][0][2]
    ref = A["data_pulses"] / draws
    np.testing.assert_allclose(np.broadcast_to(val, ref.shape), ref, rtol=0, atol=2e-6 * np.max(ref))


@pytest.mark.parametrize("name", ["tutorial1", "northstar_mini", "fold_sublen", "specidx_int8"])
def test_delays_and_noise_scale(name):
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    from psrsigsim_amd.telescope.receiver import Receiver
    meta, A, draws = load(name)
    case, sig, psr = _product(name)
    ism = ISM()
    mo, Ao, inj = replay.oracle_run(name)   # oracle (pinned) for the noise scale
    for op in case["ops"]:
        k = op[0]
        if k == "scatter_conv":
            ism.scatter_broaden(sig, op[1], op[2], convolve=True, pulsar=psr)
        elif k == "make_pulses":
            psr.make_pulses(sig, op[1])
        elif k == "disperse":
            ism.disperse(sig, op[1])
        elif k == "fd":
            ism.FD_shift(sig, op[1])
        elif k == "scatter_shift":
            ism.scatter_broaden(sig, op[1], op[2], convolve=False)
    np.testing.assert_allclose(sig.delay.value, A["delay_ms"], rtol=1e-13)
    tel = T.Arecibo() if "Arecibo" in str(case["ops"][-1]) else T.GBT()
    norm = Receiver.noise_norm(sig, psr, tel.Tsys, tel.gain)
    ref_noise = (A["data_noise"] - (A["data_null"] if "data_null" in A else A["data_disperse"]))
    ref_norm = np.median(ref_noise / draws[-1][2])
    assert np.isclose(norm, ref_norm, rtol=1e-9), (norm, ref_norm)


@pytest.mark.parametrize("tag,kind", [("eq", "copy"), ("down", "down"), ("rebin", "rebin")])
def test_observe_branch_decisions(tag, kind):
    from psrsigsim_amd.telescope import Telescope, Backend
    from psrsigsim_amd._units import Quantity
    case, sig, psr = _product("observe_" + tag)
    psr.make_pulses(sig, 0.02)
    dt = case["ops"][-1][1][1]
    got, _ = Telescope.resample_branch(sig, Backend(samprate=1.0 / Quantity(dt, "s")))
    assert got == kind


def test_dataprofile_nchan_mismatch_raises():
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, DataProfile
    sig = FilterBankSignal(1500, 800, Nsubband=4, sample_rate=0.048828125, fold=False)
    psr = Pulsar(1.0 / 218.8118437960826270, 0.009, profiles=DataProfile(replay._prof()))
    with pytest.raises(ValueError):
        psr.make_pulses(sig, 4096 * 20.48e-6)


def test_disperse_twice_raises():
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar
    from psrsigsim_amd.ism import ISM
    sig = FilterBankSignal(1400, 400, Nsubband=2, fold=False)
    Pulsar(0.005, 1.0).make_pulses(sig, 4096 * 20.48e-6)
    ism = ISM()
    ism.disperse(sig, 10)
    assert sig.dm.value == 10
    with pytest.raises(ValueError):
        ism.disperse(sig, 10)


def test_receiver_errors():
    from psrsigsim_amd.telescope import Receiver
    from psrsigsim_amd.telescope.receiver import _flat_response
    with pytest.raises(ValueError):
        Receiver(fcent=None, bandwidth=400, name="Lband")
    with pytest.raises(NotImplementedError):
        Receiver(response=_flat_response(1400, 400), name="Lband")


def test_pchip_matches_scipy():
    from scipy.interpolate import PchipInterpolator
    from psrsigsim_amd.pulsar.portraits import pchip_coefficients, ppoly_eval
    rng = np.random.default_rng(0)
    x = np.arange(245) / 244
    y = rng.random((6, 245))
    y[:, 3] = y[:, 4]
    y[1, 10:20] = 0.3
    y[2] = np.maximum(0, np.sin(6 * x))
    c = pchip_coefficients(x, y)
    P = PchipInterpolator(x, y, axis=1)
    ph = np.linspace(-0.01, 1.02, 2000)
    np.testing.assert_allclose(ppoly_eval(x, c, ph), P(ph), rtol=0, atol=1e-13)


@pytest.mark.parametrize("nchan", [1, 2, 3, 8, 64, 2048])
def test_scatter_convolution_bitwise_vs_reference_structure(nchan):
    """The batched host convolution equals the reference's per-row
    scipy.signal.convolve(method='fft') (via the oracle) bit for bit, and so
    does the periodic-closure decision that depends on it (portraits.py:234)."""
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    sig = FilterBankSignal(1400, 400, Nsubband=nchan, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    ISM().scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    osig = O.Signal(1400, 400, nchan=nchan, fold=False)
    opsr = O.Pulsar(0.005, 1.0, profiles=O.GaussPortrait(0.5, 0.05, 1))
    O.scatter_broaden(osig, 1e-4, 1400, convolve=True, pulsar=opsr)
    np.testing.assert_array_equal(psr.Profiles._kvals, opsr.Profiles.knot_y)
    psr.make_pulses(sig, (1 << 16) * 20.48e-6)
    opsr.ref_freq = 1400.0
    O.add_spec_idx(osig, opsr)
    # knot intervals (the periodic-closure decision); the device table itself
    # always spans the period (nint == M, extrapolated pieces appended)
    assert psr.Profiles.uniform_knots()[1] == opsr.Profiles.knot_x.size - 1
    assert sig._pending.source.nint == sig._pending.source.M


@pytest.mark.parametrize("nchan,nph", [(300, 512), (37, 1000), (129, 244)])
def test_uniform_profile_convolution_equals_per_row_reference(nchan, nph):
    """A profile tiled over the channels is convolved as ONE row against every
    channel's tail (ism._convolve_rows): each row equals the reference's own
    per-row scipy.signal.convolve(method='fft') (ism.py:243-288) bit for bit
    at lengths whose batched transform does not (the FFT of a many-row batch
    rounds differently from a single row's at e.g. 1023 / 1999 points)."""
    import scipy.signal as spsig
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.pulsar.portraits import tile_rows
    p1 = np.exp(-0.5 * ((np.linspace(0.0, 1.0, nph) - 0.5) / 0.05) ** 2)
    t = np.linspace(0, 0.005, nph)
    tau = np.linspace(0.05, 3.0, nchan)
    got = ISM()._convolve_rows(tile_rows(p1, nchan), lambda a, b: np.exp(-(t[None, :] * 1e3) / tau[a:b, None]), nph)
    for i in range(nchan):
        k = np.exp(-(t * 1e3) / tau[i])
        ref = p1.sum() * spsig.convolve(p1 / p1.sum(), k / k.sum(), mode='full', method='fft')[:nph]
        np.testing.assert_array_equal(got[i], ref)


def test_native_fused_pchip_bitwise():
    """pss_host_pchip_eval / pss_host_pchip_table (fit and evaluation, fit
    and device table, fused per row) == the unfused passes, bit for bit."""
    from psrsigsim_amd import _lib
    for x, y in _pchip_cases():
        c = _lib.host_pchip_coef(x, y)
        ph = np.concatenate([np.linspace(-0.1, 1.1, 333), x, [0.5 / 244.0]])
        for div in (1.0, 0.7316):
            ref = _lib.host_ppoly_eval(x, c, ph)
            if div != 1.0:
                ref = ref / div
            np.testing.assert_array_equal(_lib.host_pchip_eval(x, y, ph, div), ref)
        h = 1.0 / max(x.size - 1, 1)
        for amax in (1.0, 0.7316):
            np.testing.assert_array_equal(_lib.host_pchip_table(x, y, h, amax), _lib.host_device_table(c, h, amax))


# ---------------------------------------------------------------------------
# native host planning (pss_host_*) == the NumPy statements, bit for bit
# ---------------------------------------------------------------------------
def _pchip_cases():
    rng = np.random.default_rng(5)
    x = np.arange(245) / 244.0
    y = rng.random((300, 245))
    y[:40, 100:130] = 0.25                 # flat runs (zero slopes)
    y[40:80] = np.sin(np.linspace(0, 12, 245))[None, :] * rng.random((40, 1))   # sign changes
    y[80:90] = 0.0                         # all-zero rows
    y[90:100, ::7] = -y[90:100, ::7]       # alternating monotonicity breaks
    xs = np.sort(np.concatenate([[0.0, 1.0], rng.random(30)]))   # non-uniform knots
    return [(x, y), (x[:3], y[:5, :3]), (x[:2], y[:4, :2]), (xs, rng.random((70, xs.size)))]


@pytest.mark.parametrize("case", range(4))
def test_native_pchip_bitwise(case):
    from psrsigsim_amd import _lib
    from psrsigsim_amd.pulsar.portraits import pchip_coefficients_np, ppoly_eval_np
    x, y = _pchip_cases()[case]
    c_np = pchip_coefficients_np(x, y)
    c = _lib.host_pchip_coef(x, y)
    np.testing.assert_array_equal(c, c_np)
    ph = np.concatenate([np.linspace(-0.1, 1.1, 333), x, [0.5 / 244.0]])
    np.testing.assert_array_equal(_lib.host_ppoly_eval(x, c_np, ph), ppoly_eval_np(x, c_np, ph))


def test_native_device_table_bitwise():
    from psrsigsim_amd import _lib
    from psrsigsim_amd.pulsar.portraits import pchip_coefficients_np
    x, y = _pchip_cases()[0]
    c = pchip_coefficients_np(x, y)
    h = 1.0 / 244
    for amax in (1.0, 0.7316):
        ref = c * np.array([h ** 3, h ** 2, h, 1.0])
        if amax != 1.0:
            ref = ref / amax
        np.testing.assert_array_equal(_lib.host_device_table(c, h, amax), ref.astype(np.float32))


def test_native_threads_invariant():
    """The row passes' results do not depend on the thread count (the count
    goes to the native call directly: _lib.host_threads() is read once)."""
    from psrsigsim_amd import _lib
    L = _lib.load()
    x, y = _pchip_cases()[0]
    y = np.repeat(y, 4, axis=0)            # 1200 rows: the row-block path
    outs = []
    for nt in (1, 7):
        c = np.empty((y.shape[0], x.size - 1, 4))
        _lib.check(L.pss_host_pchip_coef(_lib._dptr(x), x.size, _lib._dptr(y), y.shape[0], _lib._dptr(c), nt),
                   "coef")
        outs.append(c)
    np.testing.assert_array_equal(outs[0], outs[1])


def _long_rows():
    rng = np.random.default_rng(11)
    K = 48829                              # the tutorial-1 profile's phase count + 1
    x = np.arange(K) / (K - 1.0)
    y = rng.random((3, K))
    y[0, 1000:9000] = 0.5                  # a flat run across span boundaries
    y[1] = np.sin(np.linspace(0, 40, K))   # sign changes
    y[2, 6000:6300] = 0.0
    return x, y


@pytest.mark.parametrize("rows", [1, 3])
def test_native_pchip_long_rows_spans_bitwise(rows):
    """A few long rows are cut into spans over the host threads
    (pss_host.cpp parallel_spans): coefficients and the fused device table
    equal the NumPy statement bit for bit at any thread count."""
    from psrsigsim_amd import _lib
    from psrsigsim_amd.pulsar.portraits import pchip_coefficients_np
    L = _lib.load()
    x, y = _long_rows()
    y = np.ascontiguousarray(y[:rows])
    K = x.size
    c_np = pchip_coefficients_np(x, y)
    h = 1.0 / (K - 1)
    for nt in (1, 3, 8):
        c = np.empty_like(c_np)
        _lib.check(L.pss_host_pchip_coef(_lib._dptr(x), K, _lib._dptr(y), rows, _lib._dptr(c), nt), "coef")
        np.testing.assert_array_equal(c, c_np)
        for amax in (1.0, 0.7316):
            t = np.empty((rows, K - 1, 4), np.float32)
            _lib.check(L.pss_host_pchip_table(_lib._dptr(x), K, _lib._dptr(y), rows, h, amax, _lib._dptr(t), nt),
                       "table")
            np.testing.assert_array_equal(t, _lib.host_device_table(c_np, h, amax))
