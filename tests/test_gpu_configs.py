"""GPU parity for the BASELINE configs and reference fixtures not covered by
the golden replays (VERDICT r01 "next round" item 1):

* C5 -- the 2^24-sample power-of-two four-step at DM 500 (with a delayed
  null: the 2048 x 8192 split and its mask table; without: 1024 x 16384 and
  the 16384-point row pass), channels of the 8192-channel band, against the
  oracle with injected draws (so the generic column passes: the fast ones
  draw their own Philox values, tests/test_gpu_fastpath_oracle.py); the
  split each run takes is asserted (pss_plan_collect); full-size properties at 2^24
  (integer shift == np.roll; the fast/generic bitwise check is in
  test_gpu_stats.py);
* C2 -- NANOGrav search mode, 2^20 samples, J1713+0747 DataProfile, GBT
  Lband_GUPPI: a 4-channel shard of the 512-channel band against the oracle;
* Backend.fold (telescope/backend.py:34-49) against the reference's recorded
  ``backend_fold`` fixture;
* utils.shift_t / down_sample / rebin against the ``utils`` fixture, including
  the reference's odd-length behaviour (utils.py:57: N - 1 samples back).

Tolerance: per-channel max|d| / max|ref| <= 1e-5 (north_star, fp32)."""
import numpy as np
import pytest

from oracle import pss_cpu as O
from tests import replay
from tests.fixtures_util import load

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _ok(errs):
    bad = {k: v for k, v in errs.items() if not v <= TOL}
    assert errs and not bad, errs


# ---------------------------------------------------------------------------
# C5: 2^24 power-of-two four-step, DM 500
# ---------------------------------------------------------------------------
def _c5_case(chans, null=True):
    ops = [("make_pulses", (1 << 24) * 20.48e-6, "pulses"), ("disperse", 500, "disperse")]
    if null:
        ops.append(("null", 0.1, "null"))
    ops.append(("observe", "Arecibo", "Lband_PUPPI", True, "noise"))
    return dict(sig=dict(fcent=1400, bw=400, nchan=8192, fold=False, chans=chans),
                psr=dict(period=0.005, Smean=1.0, prof=("gauss", 0.5, 0.05, 1)), ops=ops)


@pytest.mark.parametrize("chans,null", [((0, 2), True), ((6142, 6145), False)],
                         ids=["ch0-1_null", "ch6142-6144"])
def test_c5_2p24_fourstep_vs_oracle(chans, null, hip_lib):
    """Global channels of C5's 8192-channel band (lowest band edge: the
    largest delay, ~7e4 samples; an odd-sized shard off the pair parity),
    staged and fused are the same kernels at this size: fused only."""
    from psrsigsim_amd import _lib
    _lib.plan_collect()
    _ok(replay.run_case(None, fused=True, case=_c5_case(chans, null), seed=24 + chans[0]))
    plan = ("2048x8192", "R:pair_row_seq", "N:table") if null else ("1024x16384", "R:pair_row_seq")
    replay.assert_plan(_lib.plan_collect(), chans[1] - chans[0], 1 << 24, ("fourstep",) + plan)


def test_c5_integer_shift_is_roll(hip_lib):
    """Size-independent property at 2^24: an integer delay through the
    Fourier path equals np.roll (Nyquist factor cos(pi s) = +-1 exactly)."""
    import torch
    from psrsigsim_amd.utils import shift_t
    N = 1 << 24
    x = torch.rand((1, N), device="cuda")
    s = np.array([70123.0])
    y = shift_t(x.clone(), s, dt=1.0).cpu().numpy()[0]
    ref = np.roll(x.cpu().numpy()[0], int(s[0]))
    assert np.max(np.abs(y - ref)) < 2e-5


# ---------------------------------------------------------------------------
# C2: NANOGrav L-band search mode, J1713+0747 template, GBT
# ---------------------------------------------------------------------------
def _c2_case(chans):
    return dict(sig=dict(fcent=1500, bw=800, nchan=512, samprate=0.048828125, fold=False, chans=chans),
                psr=dict(period=1.0 / 218.8118437960826270, Smean=0.009, prof=("data", 512)),
                ops=[("make_pulses", (1 << 20) * 20.48e-6, "pulses"), ("disperse", 15.917131, "disperse"),
                     ("observe", "GBT", "Lband_GUPPI", True, "noise")])


def test_c2_j1713_2p20_vs_oracle(hip_lib):
    _ok(replay.run_case(None, fused=True, case=_c2_case((0, 4)), seed=2))


def test_c2_full_band_rows_match_shard(hip_lib):
    """The full 512-channel C2 run (Philox draws) reproduces the rows of a
    4-channel shard bit for bit (shard invariance at the config's size)."""
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, DataProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T

    def run(shard):
        pss.seed(99)
        sig = FilterBankSignal(1500, 800, Nsubband=512, sample_rate=0.048828125, fold=False, shard=shard)
        psr = Pulsar(1.0 / 218.8118437960826270, 0.009, profiles=DataProfile(replay._prof(), Nchan=512))
        psr.make_pulses(sig, (1 << 20) * 20.48e-6)
        ISM().disperse(sig, 15.917131)
        T.GBT().observe(sig, psr, system="Lband_GUPPI", noise=True)
        return sig.data

    full = run(None)
    part = run((256, 260)).cpu().numpy()
    np.testing.assert_array_equal(full[256:260].cpu().numpy(), part)
    assert full.shape == (512, 1 << 20)


# ---------------------------------------------------------------------------
# Backend.fold, utils
# ---------------------------------------------------------------------------
def test_backend_fold_vs_fixture(hip_lib):
    """telescope/backend.py:34-49 at its one working geometry (4 periods)."""
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.telescope import Backend
    meta, A, draws = load("backend_fold")
    sig = FilterBankSignal(1400, 400, Nsubband=2, fold=False, sample_rate=(1.0 / 0.005) * 2048 * 10 ** -6)
    psr = Pulsar(0.005, 10, profiles=GaussProfile(0.5, 0.05, 1))
    pss.inject(gen=draws[0][2])
    psr.make_pulses(sig, 0.02)
    assert replay._err(sig.data.cpu().numpy(), A["data_pulses"]) <= TOL
    folded = Backend(samprate=12.5, name="b").fold(sig, psr).cpu().numpy()
    assert folded.shape == A["folded"].shape
    assert replay._err(folded, A["folded"]) <= TOL


def test_backend_fold_wrong_geometry_raises(hip_lib):
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.telescope import Backend
    pss.seed(3)
    sig = FilterBankSignal(1400, 400, Nsubband=2, fold=False, sample_rate=(1.0 / 0.005) * 2048 * 10 ** -6)
    psr = Pulsar(0.005, 10, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, 0.03)                     # 6 periods: the reference's reshape fails
    with pytest.raises(ValueError):
        Backend(samprate=12.5, name="b").fold(sig, psr)


def test_utils_fixture_replay(hip_lib):
    from psrsigsim_amd.utils import shift_t, down_sample, rebin
    meta, A, _ = load("utils")
    for i, (s, dt, isint) in enumerate(meta["shifts"]):
        s = int(s) if isint else s
        dt = int(dt) if isint else dt
        assert replay._err(shift_t(A["y_even"], s, dt=dt), A["shift_even_%d" % i]) <= TOL, i
    assert replay._err(shift_t(A["y_np2"], 4321.123, dt=1.0), A["shift_np2"]) <= TOL
    assert replay._err(down_sample(A["ds_in"], 4), A["ds_4"]) <= 1e-6
    for n in (7, 100, 333, 1199):
        assert replay._err(rebin(A["rebin_in"], n), A["rebin_%d" % n]) <= 1e-6, n


@pytest.mark.parametrize("N", [3, 5, 999, 1001, 4097, 30001])
def test_shift_t_odd_length(N, hip_lib):
    """utils.py:57: for odd N the reference's irfft (no n=) returns N - 1
    samples -- the (N-1)-point inverse of the N-point spectrum's bins."""
    from psrsigsim_amd.utils import shift_t
    meta, _, _ = load("utils")
    rng = np.random.default_rng(N)
    y = rng.random(N)
    for s in (0.37, -12.25, 3.5 * N):
        got = shift_t(y, s, dt=1.0)
        ref = O.shift_t(y, s, dt=1.0)
        assert len(got) == len(ref) == N - 1
        assert replay._err(got, ref) <= TOL, (N, s)
    if N == meta["odd_len_in"]:
        assert len(shift_t(np.zeros(N), 3.3, dt=1.0)) == meta["odd_len_out"]
    # a batch of rows, one shift each, on the device
    import torch
    x = torch.from_numpy(rng.random((3, N)).astype(np.float32)).cuda()
    shifts = np.array([1.5, -0.25, 100.125])
    x0 = x.clone()
    out = shift_t(x, shifts, dt=1.0).cpu().numpy()
    assert torch.equal(x, x0)              # a new array, as the reference returns
    assert out.shape == (3, N - 1)
    for r in range(3):
        ref = O.shift_t(x[r].cpu().numpy().astype(np.float64), float(shifts[r]), dt=1.0)
        assert replay._err(out[r], ref) <= TOL
