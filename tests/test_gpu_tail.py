"""Scattering tail on the time series (EXTENSION of ISM.scatter_broaden,
keyword ``tail=True``; north_star K2 "scattering-tail transfer function in
the fused forward/inverse pass").  The reference has no counterpart
(ism.py:158-240 only delays, or convolves the profile before make_pulses;
SURVEY.md App. A.11), so these tests are analytic: every channel's samples
are circularly convolved with the normalised exponential h[n] = (1 - a) a^n,
a = exp(-dt/tau_c), tau_c = tau_d (f_c / f_ref)^(-22/5) -- i.e. an impulse
comes out as (1 - a) a^((n - n0) mod N) / (1 - a^N) -- on every FFT path
(four-step pair rows, single pass, mixed radix, Bluestein), alone and fused
with a dispersion delay (checked against a float64 NumPy restatement)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _signal(nchan, N, data):
    from psrsigsim_amd.signal import FilterBankSignal
    sig = FilterBankSignal(1400, 400, Nsubband=nchan, fold=False)
    sig._buf = torch.as_tensor(np.asarray(data, dtype=np.float32)).cuda().contiguous()
    sig._ncols = N
    sig._nsamp = N
    return sig


def _a_of(sig, tau_d, ref):
    from psrsigsim_amd.ism import ISM
    tau_ms = ISM().scale_tau_d(tau_d * 1e3, ref, sig._freqs_MHz())
    return np.exp(-sig._dt_ms() / tau_ms)


@pytest.mark.parametrize("N", [1 << 16, 4096, 30720, 100002])
def test_tail_impulse_response_analytic(N, hip_lib):
    from psrsigsim_amd.ism import ISM
    nchan = 3
    n0 = np.array([0, 17, N // 3])
    x = np.zeros((nchan, N))
    x[np.arange(nchan), n0] = 1.0
    sig = _signal(nchan, N, x)
    tau_d, ref = 2e-4, 1400.0
    a = _a_of(sig, tau_d, ref)
    ISM().scatter_broaden(sig, tau_d, ref, tail=True)
    got = sig.data.cpu().numpy().astype(np.float64)
    assert sig.delay is None                         # a filter, not a delay
    for c in range(nchan):
        m = (np.arange(N) - n0[c]) % N
        ref_c = (1 - a[c]) * a[c] ** m / (1 - a[c] ** N)
        err = np.max(np.abs(got[c] - ref_c)) / np.max(ref_c)
        assert err < TOL, (N, c, err)
        assert abs(got[c].sum() - 1.0) < 1e-4           # H(0) = 1: flux preserved


def _np_tail_delay(x, a, s):
    """float64 restatement: irfft(rfft(x) * exp(-2 pi i k s / N) * H(k))
    with the reference's Nyquist rule for the delay (cos(pi s))."""
    N = x.size
    X = np.fft.rfft(x)
    k = np.arange(X.size)
    ramp = np.exp(-2j * np.pi * k * s / N)
    H = (1 - a) / (1 - a * np.exp(-2j * np.pi * k / N))
    Y = X * ramp * H
    if N % 2 == 0:
        Y[-1] = X[-1] * np.cos(np.pi * s) * H[-1].real
    return np.fft.irfft(Y, n=N)


@pytest.mark.parametrize("N", [1 << 16, 1 << 14, 4096, 100002])
def test_tail_fused_with_dispersion(N, hip_lib):
    from psrsigsim_amd.ism import ISM
    rng = np.random.default_rng(N)
    nchan = 4
    x = rng.random((nchan, N)) * 10
    sig = _signal(nchan, N, x)
    ism = ISM()
    a = _a_of(sig, 1e-4, 1500.0)
    ism.scatter_broaden(sig, 1e-4, 1500.0, tail=True)
    from psrsigsim_amd.ism.ism import push_delay
    delays_ms = np.linspace(3.0, 9.0, nchan)           # a delay stage in the same fused pass
    push_delay(sig, delays_ms)
    got = sig.data.cpu().numpy().astype(np.float64)
    s = delays_ms / sig._dt_ms()
    for c in range(nchan):
        ref = _np_tail_delay(x[c].astype(np.float32).astype(np.float64), a[c], s[c])
        err = np.max(np.abs(got[c] - ref)) / np.max(np.abs(ref))
        assert err < TOL, (N, c, err)


def test_tail_with_delayed_null_off_fourstep_is_unsupported(hip_lib):
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    pss.seed(4)
    sig = FilterBankSignal(1400, 400, Nsubband=2, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, tobs=4096 * 20.48e-6)
    ISM().disperse(sig, 10)
    ISM().scatter_broaden(sig, 1e-4, 1400, tail=True)
    psr.null(sig, 0.3)
    with pytest.raises(NotImplementedError):
        _ = sig.data


def test_tail_disperse_delayed_null_2p22_vs_oracle(hip_lib):
    """The tail extension together with disperse and a DELAYED null at the
    north-star length 2^22 on the pair four-step (the mask-table null path):
    against the oracle run with injected draws (legacy RandomState) and the
    float64 restatement of the tail (tests/replay.py 'scatter_tail'; the tail
    is a filter, so the null mask is shifted by the dispersion delay only,
    pulsar.py:306-330)."""
    from tests import replay
    case = dict(sig=dict(fcent=1400, bw=400, nchan=2, fold=False),
                psr=dict(period=0.005, Smean=1.0, prof=("gauss", 0.5, 0.05, 1)),
                ops=[("make_pulses", (1 << 22) * 20.48e-6, "pulses"), ("scatter_tail", 2e-4, 1400.0, None),
                     ("disperse", 100, "disperse"), ("null", 0.1, "null"),
                     ("observe", "Arecibo", "Lband_PUPPI", True, "noise")])
    errs = replay.run_case(None, fused=True, case=case, seed=2222)
    bad = {k: v for k, v in errs.items() if not v <= TOL}
    assert errs and not bad, errs
    assert replay.STATS.get("ambiguous_path") == "table"
