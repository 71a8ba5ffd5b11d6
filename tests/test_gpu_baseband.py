"""Baseband path on the GPU: amplitude pulses
(pulsar.py:153-183) and coherent dispersion (ism.py:76-98) through the C-ABI,
against the golden vectors recorded from the reference (exact mode: its own
normal draws injected) and, for the Philox draws, in distribution.
Tolerance: normwise 1e-5 (north_star fp32), plus, for dispersion, the float64
conditioning of the reference's own phase (see test_oracle_golden)."""
import numpy as np
import pytest

from tests.fixtures_util import load

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))


def _maxphase(sr, dm, N):
    u = np.fft.rfftfreq(2 * (N // 2 + 1) - 1, d=(1.0 / sr) * 1e-6)
    f = u - 200.0
    return float(np.max(np.abs(2 * np.pi * (1.0 / 2.41e-4) / ((f + 1400.0) * 1400.0 ** 2) * dm * f ** 2 * 1e6)))


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_baseband_golden_exact(tag, hip_lib):
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import BasebandSignal
    from psrsigsim_amd.pulsar import Pulsar, DataProfile
    from psrsigsim_amd.ism import ISM
    meta, A, draws = load("baseband")
    sr, per, tobs, dm = meta["geom_" + tag]
    normal = [a for k, _, a in draws if k == "normal"]["abc".index(tag)]
    sig = BasebandSignal(1400, 400, sample_rate=sr, Nchan=2)
    pro = None if tag == "c" else DataProfile(A["input_profile"])      # c: default GaussProfile
    psr = Pulsar(per, 10, profiles=pro, name='J1746-0118')
    pss.inject(gen=normal)
    psr.make_pulses(sig, tobs)
    assert sig.nsamp == meta["nsamp_" + tag]
    from psrsigsim_amd._units import to_value
    assert np.isclose(float(to_value(sig._Smax, 'Jy')), meta["Smax_" + tag], rtol=1e-12)
    assert _err(sig.data.cpu().numpy(), A["data_pulses_" + tag]) <= TOL
    ISM().disperse(sig, dm)
    tol = TOL + 4 * _maxphase(sr, dm, sig.nsamp) * 2.0 ** -53
    assert _err(sig.data.cpu().numpy(), A["data_disperse_" + tag]) <= tol
    with pytest.raises(ValueError):
        ISM().disperse(sig, dm)


@pytest.mark.parametrize("N", [4096, 51200, 1 << 16, 100002, 20480, 1 << 22, 1 << 23, 1 << 24, 196608, 3125000])
def test_filter_rows_vs_numpy(N, hip_lib):
    """The transfer-function run against numpy irfft(rfft(x) H) in float64:
    single pass (4096), the pair four-step with H in the row pass (2^16,
    2^22; 8192-point rows at 2^23 = 1024 x 8192 and 2^24 = 2048 x 8192; the
    mixed-radix 10 x 2048 split at 20480 and 24 x 8192 at 196608; the radix-5
    1250 x 2500 split at 3 125 000), Bluestein (51200, 100002).  (ADVICE r04:
    every row-pass instantiation the htab runs can take.)"""
    import torch
    from psrsigsim_amd import _engine
    rng = np.random.default_rng(N)
    x = rng.standard_normal((3, N)).astype(np.float32)
    H = np.exp(1j * 2 * np.pi * rng.random(N // 2 + 1) * 50.0)

    class _S:
        def __init__(self, t):
            self.data = t

    s = _S(torch.from_numpy(x).cuda())
    _engine.filter_rows(s, H)
    got = s.data.cpu().numpy()
    ref = np.fft.irfft(np.fft.rfft(x.astype(np.float64), axis=1) * H.astype(np.complex64), axis=1)
    assert _err(got, ref) <= TOL


def test_amp_pulses_distribution(hip_lib):
    """Philox amplitude pulses from a flat profile are N(0, 1): per-channel
    mean/variance and a KS test (north_star stochastic gates)."""
    from scipy import stats
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import BasebandSignal
    from psrsigsim_amd.pulsar import Pulsar, DataProfile
    pss.seed(11)
    sig = BasebandSignal(1400, 400, sample_rate=1.024, Nchan=2)
    psr = Pulsar(0.005, 10, profiles=DataProfile(np.ones(64)))
    psr.make_pulses(sig, ((1 << 20) + 0.5) / 1.024e6)
    d = sig.data.cpu().numpy().astype(np.float64)
    assert d.shape == (2, 1 << 20)
    for row in d:
        assert abs(row.mean()) < 0.005 and abs(row.var() - 1.0) < 0.005
        assert stats.kstest(row[::16], "norm").pvalue > 0.01


def test_baseband_errors(hip_lib):
    from psrsigsim_amd.signal import BasebandSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile, DataProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import Telescope, Receiver, Backend
    bb = BasebandSignal(1400, 400, sample_rate=1.0 * 2048 * 10 ** -6, Nchan=2)
    assert bb.to_Baseband() is bb
    with pytest.raises(NotImplementedError):
        bb.to_RF()
    with pytest.raises(NotImplementedError):
        bb.to_FilterBank()
    psr = Pulsar(1.0, 1.0, profiles=DataProfile(np.hanning(256) + 0.01))
    odd = BasebandSignal(1400, 400, sample_rate=1.0 * 2048 * 10 ** -6, Nchan=2)
    psr.make_pulses(odd, 2047 / 2048.0 + 1e-9)
    assert odd.nsamp % 2 == 1
    with pytest.raises(ValueError):
        ISM().disperse(odd, 3.0)
    tel = Telescope(20.0, area=None, Tsys=25.0, name="T")
    tel.add_system(name="S", receiver=Receiver(fcent=1400, bandwidth=400, name="L"),
                   backend=Backend(samprate=1.0, name="B"))
    psr.make_pulses(bb, 2.0)
    with pytest.raises(NotImplementedError):
        tel.observe(bb, psr, system="S", noise=False)


def test_bb_obs_reference_sequence(hip_lib):
    """tests/test_telescope.py::test_bb_obs: default-rate BasebandSignal,
    default GaussProfile pulsar, make_pulses(0.01 s) -- 8e6 samples of
    amplitude pulses on the device -- then observe raises
    NotImplementedError; pulses are finite and N(0, prof) shaped."""
    from psrsigsim_amd.signal import BasebandSignal
    from psrsigsim_amd.pulsar import Pulsar
    from psrsigsim_amd.telescope import Telescope, Receiver, Backend
    from psrsigsim_amd.utils import make_quant
    bb = BasebandSignal(1400, 400)
    psr = Pulsar(make_quant(5, 'ms'), 10, name='J1746-0118')
    tel = Telescope(20.0, area=None, Tsys=25.0, name="Twenty_Meter")
    tel.add_system(name="Twnty_M", receiver=Receiver(fcent=1400, bandwidth=400, name="Lband"),
                   backend=Backend(samprate=0.3125, name="Cyborg"))
    psr.make_pulses(bb, make_quant(0.01, 's'))
    d = bb.data
    assert tuple(d.shape) == (2, 8000000)
    x = d.cpu().numpy()
    assert np.isfinite(x).all()
    # phase 0.5 (the Gaussian peak, |x| ~ N(0,1)) vs phase 0 (exp(-50): ~0)
    spp = 800e6 * 5e-3
    on = x[:, int(spp * 0.5) - 500: int(spp * 0.5) + 500]
    off = x[:, :200]
    assert 0.5 < on.std() < 1.5 and off.std() < 1e-8
    with pytest.raises(NotImplementedError):
        tel.observe(bb, psr, system="Twnty_M", noise=False)
