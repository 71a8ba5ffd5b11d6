"""GPU parity: the HIP path (through the C-ABI via psrsigsim_amd) against the
reference's golden vectors (exact mode: the reference's own draws injected)
and against the CPU oracle.  Tolerance: per-channel max|d| / max|ref| <= 1e-5
(fp32 device vs float64 reference, BASELINE.json north_star)."""
import numpy as np
import pytest

from oracle import pss_cpu as O
from tests import replay

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.mark.parametrize("fused", [True, False], ids=["fused", "staged"])
@pytest.mark.parametrize("name", sorted(replay.CASES))
def test_golden_replay(name, fused, hip_lib):
    errs = replay.run_case(name, fused=fused)
    assert errs, "nothing compared"
    bad = {k: v for k, v in errs.items() if not v <= TOL}
    assert not bad, errs


SIZES = [64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536, 1 << 17, 1 << 18,
         1 << 20, 1 << 23, 244, 1000, 30720,
         # mixed-radix four-step: N1 x N2 = 6 x 2048, 10 x 4096, 30 x 2048, 30 x 4096, 24 x 8192
         12288, 40960, 61440, 122880, 196608,
         # Bluestein (chirp-z) fallback: M1 x M2 = 8 x 4096 (2 x 5003), 64 x 4096,
         # 1024 x 4096 (2^20 - 2), 4096 x 8192 (2^24 - 2); and the reference
         # simulate fixture's 3 125 000 = 2^3 5^8 (radix-5 four-step 1250 x 2500)
         10006, 100002, (1 << 20) - 2, 3125000, (1 << 24) - 2]


@pytest.mark.parametrize("N", SIZES)
def test_shift_t_rows_vs_oracle(N, hip_lib):
    from psrsigsim_amd.utils import shift_t
    rng = np.random.default_rng(N)
    R = 3 if N <= (1 << 18) else (2 if N <= (1 << 22) else 1)
    x = rng.random((R, N)).astype(np.float32)
    shifts = np.array([0.37, -1234.5678, 3.0 * N + 17.25][:R])
    got = shift_t(x, shifts, dt=1.0)
    for r in range(R):
        ref = O.shift_t(x[r].astype(np.float64), float(shifts[r]), dt=1.0)
        err = np.max(np.abs(got[r] - ref)) / np.max(np.abs(ref))
        assert err < TOL, (N, r, err)


@pytest.mark.parametrize("N", [10006, 100002])
def test_bluestein_matches_direct_dft(N, hip_lib):
    """The Bluestein path and the O(N^2) direct DFT (PSS_FLAG_DIRECT_DFT) agree
    on the same rows (both fp32 on the device, direct accumulating in f64)."""
    from psrsigsim_amd import _lib
    from psrsigsim_amd.utils import shift_t
    x = np.random.default_rng(N).random((2, N)).astype(np.float32)
    s = np.array([12.345, -N / 3.0])
    a = shift_t(x, s, dt=1.0)
    L = _lib.load()
    old = L.pss_set_flags(_lib.FLAG_DIRECT_DFT)
    try:
        b = shift_t(x, s, dt=1.0)
    finally:
        L.pss_set_flags(old)
    assert np.max(np.abs(a - b)) / np.max(np.abs(b)) < TOL


def test_shift_t_integer_is_roll_full_size(hip_lib):
    """Size-independent property at a BASELINE row length (2^22): a shift by
    an integer number of samples through the Fourier path equals np.roll
    (Nyquist factor cos(pi s) = +-1 exactly)."""
    import torch
    from psrsigsim_amd.utils import shift_t
    N = 1 << 22
    x = torch.rand((2, N), device="cuda")
    s = np.array([1234567.0, -77.0])
    y = shift_t(x.clone(), s, dt=1.0).cpu().numpy()
    xh = x.cpu().numpy()
    for r in range(2):
        ref = np.roll(xh[r], int(s[r]))
        assert np.max(np.abs(y[r] - ref)) < 2e-5


def test_shift_t_int_roll_path(hip_lib):
    from psrsigsim_amd.utils import shift_t
    y = np.arange(10.0)
    np.testing.assert_array_equal(shift_t(y, 2, dt=1), np.roll(y, 2))


def test_odd_length_disperse_raises(hip_lib):
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar
    from psrsigsim_amd.ism import ISM
    sig = FilterBankSignal(1400, 400, Nsubband=2, fold=False)
    psr = Pulsar(0.005, 1.0)
    psr.make_pulses(sig, 9765 * 20.48e-6 * 1.00001)
    assert sig.nsamp % 2 == 1
    with pytest.raises(ValueError):
        ISM().disperse(sig, 10)


def test_null_tied_channel0_raises_on_every_readout(hip_lib):
    """A null() whose channel-0 maximum is not unique (the reference's
    pulsar.py:286 broadcast ValueError) raises on observe's returned copy and on
    every later read of the data, not only the first."""
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, DataProfile
    from psrsigsim_amd.telescope import telescope as T
    n = 1 << 14
    sig = FilterBankSignal(1400, 400, Nsubband=2, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=DataProfile(np.ones(256), Nchan=2))
    pss.inject(gen=np.ones((2, n)))            # flat channel 0: every sample ties
    psr.make_pulses(sig, n * 20.48e-6)
    psr.null(sig, 0.1)
    with pytest.raises(ValueError):
        T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True, ret_resampsig=True)
    for _ in range(2):
        with pytest.raises(ValueError):
            sig.data
    # new pulses replace the data: the earlier null's error no longer applies
    # (ADVICE r03), as with the reference, which raised once at null() time
    import torch
    psr.make_pulses(sig, n * 20.48e-6)
    d = sig.data
    assert d.shape == (2, n) and bool(torch.isfinite(d).all())


def _big_case(log2n, nchan, null=True, fd=True):
    ops = [("scatter_conv", 1e-4, 1400, None), ("make_pulses", (1 << log2n) * 20.48e-6, "pulses"),
           ("disperse", 100, "disperse")]
    if fd:
        ops.append(("fd", [2e-4, -3e-5], "fd"))
    if null:
        ops.append(("null", 0.1, "null"))
    ops.append(("observe", "Arecibo", "Lband_PUPPI", True, "noise"))
    return dict(sig=dict(fcent=1400, bw=400, nchan=nchan, fold=False),
                psr=dict(period=0.005, Smean=1.0, prof=("gauss", 0.5, 0.05, 1)), ops=ops)


@pytest.mark.parametrize("fused", [True, False], ids=["fused", "staged"])
@pytest.mark.parametrize("log2n,nchan,null", [(14, 3, True), (16, 3, True), (17, 2, True),
                                               (17, 3, False), (20, 1, True), (22, 3, True)])
def test_fourstep_pair_path_vs_oracle(log2n, nchan, null, fused, hip_lib):
    """The four-step PAIR path (odd and even channel counts, with and without
    the delayed-null mask, fused and staged = mask-only FFT) against the
    oracle run with legacy RandomState draws, injected into the GPU run."""
    errs = replay.run_case(None, fused=fused, case=_big_case(log2n, nchan, null=null), seed=log2n)
    bad = {k: v for k, v in errs.items() if not v <= TOL}
    assert not bad, errs


F0_B1855 = 186.4940812499314404


def _c4_case(nchan, null, prof=None):
    """BASELINE config C4 (fold mode: 30 subints x 1024 bins = 30720 samples
    per channel, DM 13.3, radiometer noise) at a few channels: the
    mixed-radix four-step (30 x 1024) -- or, with a delayed null, the direct
    path -- against the oracle."""
    ops = [("make_pulses", 1800.0, "pulses"), ("disperse", 13.299393, "disperse")]
    if null:
        ops.append(("null", 0.1, "null"))
    ops.append(("observe", "Arecibo", "Lband_PUPPI", True, "noise"))
    return dict(sig=dict(fcent=1400, bw=400, nchan=nchan, samprate=F0_B1855 * 1024 * 1e-6, sublen=60.0,
                         fold=True),
                psr=dict(period=1.0 / F0_B1855, Smean=0.005, prof=prof or ("gauss", 0.5, 0.05, 1)), ops=ops)


@pytest.mark.parametrize("nchan,null,template", [(3, False, False), (4, False, False), (2, True, False),
                                                  (4, False, True), (2, True, True)])
def test_c4_fold_mixed_radix_vs_oracle(nchan, null, template, hip_lib):
    """C4 with a Gaussian portrait and with the config's own B1855+09
    template portrait (the reference's PSRFITS template read by
    psrsigsim_amd.io.psrfits, resampled 2048 -> 1024 bins by the PCHIP
    DataPortrait)."""
    prof = ("b1855", nchan) if template else None
    errs = replay.run_case(None, fused=True, case=_c4_case(nchan, null, prof), seed=nchan)
    bad = {k: v for k, v in errs.items() if not v <= TOL}
    assert not bad, errs


@pytest.mark.parametrize("log2n,null", [(12, False), (16, True), (22, False)])
def test_nonuniform_portrait_phases_vs_oracle(log2n, null, hip_lib):
    """A DataPortrait on NON-uniform phases (split-cell device table,
    PssPipeline.prof_split; the reference's PchipInterpolator over those
    knots) through pulses, dispersion, (delayed null) and noise, against the
    oracle with injected draws: single pass (2^12), four-step pair path."""
    ops = [("make_pulses", (1 << log2n) * 20.48e-6, "pulses"), ("disperse", 100, "disperse")]
    if null:
        ops.append(("null", 0.1, "null"))
    ops.append(("observe", "Arecibo", "Lband_PUPPI", True, "noise"))
    case = dict(sig=dict(fcent=1400, bw=400, nchan=3, fold=False),
                psr=dict(period=0.005, Smean=1.0, prof=("dataph", 3)), ops=ops)
    errs = replay.run_case(None, fused=True, case=case, seed=log2n + 7)
    bad = {k: v for k, v in errs.items() if not v <= TOL}
    assert not bad, errs


@pytest.mark.parametrize("fused", [True, False], ids=["fused", "staged"])
@pytest.mark.parametrize("N,nchan,null", [(10006, 3, True), (100002, 2, True), (100002, 3, False)])
def test_bluestein_pipeline_vs_oracle(N, nchan, null, fused, hip_lib):
    """The whole C3-style chain (scatter convolve, pulses, DM, FD, delayed
    null, noise) at even lengths with a large prime factor (Bluestein path)
    against the oracle with injected draws."""
    case = _big_case(0, nchan, null=null)
    case["ops"][1] = ("make_pulses", (N + 0.5) * 20.48e-6, "pulses")
    errs = replay.run_case(None, fused=fused, case=case, seed=N + nchan)
    bad = {k: v for k, v in errs.items() if not v <= TOL}
    assert not bad, errs


@pytest.mark.parametrize("nbin,nper,extra", [(244, 17, 5), (1024, 30, 0), (2048, 3, 100)])
def test_fold_periods_vs_numpy(nbin, nper, extra, hip_lib):
    """Backend.fold_periods (corrected fold, extension): sum over whole
    periods = numpy reshape-sum in float64, trailing partial period dropped."""
    import torch
    from psrsigsim_amd.telescope import Backend

    class _Sig:
        def __init__(self, d):
            self.data = d

    rng = np.random.default_rng(nbin)
    x = rng.random((3, nbin * nper + extra)).astype(np.float32) * 100
    out = Backend(samprate=1.0, name="b").fold_periods(_Sig(torch.from_numpy(x).cuda()), None, nbin=nbin)
    ref = x[:, :nbin * nper].astype(np.float64).reshape(3, nper, nbin).sum(axis=1)
    np.testing.assert_allclose(out.cpu().numpy(), ref.astype(np.float32), rtol=1e-6)


def test_fold_periods_full_c3_size(hip_lib):
    """At a BASELINE length (2^22 samples, 244-sample periods): the fold of a
    periodic signal is nper x one period (size-independent property)."""
    import torch
    from psrsigsim_amd.telescope import Backend

    class _Sig:
        def __init__(self, d):
            self.data = d

    nbin, N = 244, 1 << 22
    nper = N // nbin
    one = torch.arange(nbin, dtype=torch.float32, device="cuda") * 0.25
    x = torch.zeros((2, N), device="cuda")
    x[:, :nper * nbin] = one.repeat(nper)
    out = Backend(samprate=1.0, name="b").fold_periods(_Sig(x), None, nbin=nbin)
    np.testing.assert_array_equal(out.cpu().numpy(), (one.cpu().numpy().astype(np.float64) * nper)[None].repeat(2, 0).astype(np.float32))


@pytest.mark.parametrize("fold", [True, False])
def test_null_refine_list_equals_per_sample(fold, hip_lib):
    """The float64 null decisions of the packed paths: the compacted candidate
    list (four candidates per wave) and the per-sample kernel (the list's
    overflow path, PSS_FLAG_REFINE_PER_SAMPLE) give the same bits -- C4's
    fold-mode geometry with a null (Bluestein at 30720, dense candidates) and
    a search-mode Bluestein length."""
    import psrsigsim_amd as pss
    from psrsigsim_amd import _lib
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T

    def run():
        pss.seed(31)
        if fold:
            sig = FilterBankSignal(1400, 400, Nsubband=6, sample_rate=F0_B1855 * 1024 * 1e-6, sublen=60.0, fold=True)
            psr = Pulsar(1.0 / F0_B1855, 0.005, profiles=GaussProfile(0.5, 0.05, 1))
            psr.make_pulses(sig, tobs=1800.0)
            ISM().disperse(sig, 13.299393)
        else:
            sig = FilterBankSignal(1400, 400, Nsubband=5, fold=False)
            psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
            psr.make_pulses(sig, tobs=(100002 + 0.5) * 20.48e-6)
            ISM().disperse(sig, 30)
        psr.null(sig, 0.1)
        T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
        return sig.data.cpu().numpy()

    L = _lib.load()
    a = run()
    old = L.pss_set_flags(_lib.FLAG_REFINE_PER_SAMPLE)
    try:
        b = run()
    finally:
        L.pss_set_flags(old)
    np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("N", [10006, 100002, (1 << 20) - 2])
def test_bluestein_fused_rows_fast_equals_generic(N, hip_lib):
    """Bluestein pair mode on device-resident rows: the one-sample-per-item
    first / last column passes (coalesced row loads and stores) give the bits
    of the generic 4-sample-item passes (PSS_FLAG_NO_FAST); odd row count, so
    the last pair (a lone row) takes the generic form in both runs."""
    import torch
    from psrsigsim_amd import _lib
    from psrsigsim_amd.utils import shift_t
    x = torch.rand((5, N), device="cuda", generator=torch.Generator(device="cuda").manual_seed(N))
    s = np.linspace(-77.3, 1234.5, 5)
    a = shift_t(x.clone(), s, dt=1.0)
    L = _lib.load()
    old = L.pss_set_flags(_lib.FLAG_NO_FAST)
    try:
        b = shift_t(x.clone(), s, dt=1.0)
    finally:
        L.pss_set_flags(old)
    a = a.cpu().numpy() if hasattr(a, "cpu") else np.asarray(a)
    b = b.cpu().numpy() if hasattr(b, "cpu") else np.asarray(b)
    np.testing.assert_array_equal(a, b)
