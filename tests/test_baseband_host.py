"""Host side of the baseband path (no GPU): the transfer function the device
filter receives equals the oracle's restatement of ism.py:84-93, and the
fused-run plan of amplitude pulses selects the right source (PCHIP table or
analytic Gaussian components) with the reference's nsamp / phase step."""
import math

import numpy as np
import pytest

from oracle import pss_cpu as O
from tests.fixtures_util import load


def _bb(sr):
    from psrsigsim_amd.signal import BasebandSignal
    return BasebandSignal(1400, 400, sample_rate=sr, Nchan=2)


@pytest.mark.parametrize("sr,per,tobs,dm", [(1.024, 0.005, 0.05, 10.0), (0.002048, 1.0, 2.0, 3.0)])
def test_disperse_baseband_transfer_matches_oracle(sr, per, tobs, dm, monkeypatch):
    from psrsigsim_amd import _engine
    from psrsigsim_amd.pulsar import Pulsar, DataProfile
    from psrsigsim_amd.ism import ISM
    got = {}
    monkeypatch.setattr(_engine, "filter_rows", lambda sig, H: got.setdefault("H", np.asarray(H)))
    _, A, _ = load("baseband")
    sig = _bb(sr)
    Pulsar(per, 10, profiles=DataProfile(A["input_profile"])).make_pulses(sig, tobs)
    ISM().disperse(sig, dm)
    osig = O.BasebandSignal(1400, 400, samprate=sr, nchan=2)
    ref = O.baseband_transfer(osig, dm, sig._ncols)
    assert got["H"].shape == ref.shape == (sig._ncols // 2 + 1,)
    # same formula, same float64 operations up to the order of the 1e6 scale
    dphase = np.angle(got["H"] * np.conj(ref))
    u = np.fft.rfftfreq(2 * (sig._ncols // 2 + 1) - 1, d=(1.0 / sr) * 1e-6)
    f = u - 200.0
    maxph = np.max(np.abs(2 * np.pi * O.DM_K / ((f + 1400.0) * 1400.0 ** 2) * dm * f ** 2 * 1e6))
    assert np.max(np.abs(dphase)) <= max(1e-12, 8 * maxph * 2.0 ** -53)
    with pytest.raises(ValueError):
        ISM().disperse(sig, dm)


@pytest.mark.parametrize("kind", ["gauss", "pchip"])
def test_amp_pulse_plan(kind):
    from psrsigsim_amd import _engine, _lib
    from psrsigsim_amd.pulsar import Pulsar, DataProfile
    _, A, _ = load("baseband")
    sig = _bb(1.024)
    prof = None if kind == "gauss" else DataProfile(A["input_profile"])
    psr = Pulsar(0.005, 10, profiles=prof)
    psr.make_pulses(sig, 0.02)
    assert sig.nsamp == int((0.02 * 1.024) * 1e6) == sig._ncols
    P = _engine.plan_pipeline(sig, sig._pending, 2, 0)
    assert P["src"] == _lib.SRC_SEARCH and P["gen_amp"] == (2 if kind == "gauss" else 1)
    assert P["draw_norm"] == 1.0
    inv = 1.0 / ((1.024 * 0.005) * 1e6)
    assert P["phase_step"] == int(round(math.ldexp(inv - math.floor(inv), 64))) % (1 << 64)
    if kind == "gauss":
        t = sig._pending.source.table
        assert t.shape == (1, 1, 4) and P["knot_m"] == 1
        np.testing.assert_allclose(t[0, 0, :3], [0.5, 1 / 0.05, 1.0 / float(psr.Profiles.Amax)], rtol=1e-7)
