"""Pin the CPU oracle (oracle/pss_cpu.py) against golden vectors recorded from
the unmodified reference (tests/golden/make_golden.py).  Random draws are
replayed from the fixtures, so every stage must agree to float64 round-off."""
import os

import numpy as np
import pytest

from oracle import pss_cpu as O
from tests.fixtures_util import load

RTOL = 1e-9   # float64 restatement vs reference: round-off only


def close(a, b, rtol=RTOL):
    a = np.asarray(a, dtype=float)
    b = np.asarray(b, dtype=float)
    assert a.shape == b.shape, (a.shape, b.shape)
    scale = max(np.max(np.abs(b)), 1e-300)
    err = np.max(np.abs(a - b)) / scale if a.size else 0.0
    assert err <= rtol, "normwise err %.3g > %.3g" % (err, rtol)


def check_meta(sig, meta):
    assert sig.nsamp == meta["nsamp"]
    assert sig.nsub == meta["nsub"]
    if meta.get("Nfold") is not None:
        assert np.isclose(sig.Nfold, meta["Nfold"], rtol=1e-12)
    assert np.isclose(sig.Smax, meta["Smax"], rtol=1e-12)
    assert np.isclose(sig.draw_norm, meta["draw_norm"], rtol=1e-12)
    assert sig.draw_max == meta["draw_max"]


def test_tutorial1():
    meta, A, draws = load("tutorial1")
    d = O.InjectedDraws(draws)
    sig = O.Signal(1400, 400, nchan=2)
    psr = O.Pulsar(0.005, 10, profiles=O.GaussPortrait(0.5, 0.05, 1))
    O.make_pulses(sig, psr, 1.0, d)
    close(sig.data, A["data_pulses"], 1e-13)
    close(psr.Profiles.gen.c, A["pchip_c"], 1e-12)
    close(psr.Profiles._max_profile, A["max_profile"], 1e-13)
    O.disperse(sig, 10)
    close(sig.data, A["data_disperse"])
    out = O.observe(sig, psr, O.Arecibo(), "Lband_PUPPI", d, noise=True)
    assert out.dtype == np.dtype(meta["out_dtype"])
    close(out, A["out"], 1e-7)
    close(sig.data, A["data_noise"])
    check_meta(sig, meta)
    close(sig.delay, A["delay_ms"], 1e-13)
    close(sig.dat_freq, A["dat_freq"], 0)


def test_northstar_mini():
    meta, A, draws = load("northstar_mini")
    d = O.InjectedDraws(draws)
    sig = O.Signal(1400, 400, nchan=4, fold=False)
    psr = O.Pulsar(0.005, 1.0, profiles=O.GaussPortrait(0.5, 0.05, 1))
    O.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    close(psr.Profiles.gen.c[-1], A["convolved_profiles"], 1e-12)
    O.make_pulses(sig, psr, 8192 * 20.48e-6, d)
    close(sig.data, A["data_pulses"], 1e-12)
    O.disperse(sig, 100)
    close(sig.data, A["data_disperse"])
    O.FD_shift(sig, [2e-4, -3e-5])
    close(sig.data, A["data_fd"])
    O.scatter_broaden(sig, 3e-4, 1400, convolve=False)
    close(sig.data, A["data_scatter"])
    O.null(sig, psr, 0.1, d)
    close(sig.data, A["data_null"])
    out = O.observe(sig, psr, O.Arecibo(), "Lband_PUPPI", d, noise=True)
    close(out, A["out"], 1e-7)
    close(sig.data, A["data_noise"])
    check_meta(sig, meta)
    close(sig.delay, A["delay_ms"], 1e-13)
    assert d.i == len(draws)


def test_j1713_search():
    meta, A, draws = load("j1713_search")
    d = O.InjectedDraws(draws)
    sig = O.Signal(1500, 800, nchan=4, samprate=0.048828125, fold=False)
    psr = O.Pulsar(1.0 / 218.8118437960826270, 0.009,
                   profiles=O.DataProfile(A["input_profile"], nchan=4))
    O.make_pulses(sig, psr, 4096 * 20.48e-6, d)
    close(sig.data, A["data_pulses"], 1e-12)
    O.disperse(sig, 15.917131)
    close(sig.data, A["data_disperse"])
    out = O.observe(sig, psr, O.GBT(), "Lband_GUPPI", d, noise=True)
    close(out, A["out"], 1e-7)
    close(sig.data, A["data_noise"])
    check_meta(sig, meta)


def test_dataprofile_nchan_mismatch_raises():
    """The reference fails broadcasting a 1-row DataProfile into Nchan>1
    channels in place (pulsar.py:103) -- the oracle keeps that error."""
    _, A, _ = load("j1713_search")
    sig = O.Signal(1500, 800, nchan=4, samprate=0.048828125, fold=False)
    psr = O.Pulsar(1.0 / 218.8118437960826270, 0.009, profiles=O.DataProfile(A["input_profile"]))
    with pytest.raises(ValueError):
        O.make_pulses(sig, psr, 4096 * 20.48e-6, O.LegacyDraws(0))


def test_fold_sublen():
    meta, A, draws = load("fold_sublen")
    d = O.InjectedDraws(draws)
    prof = np.load(os.path.join(os.path.dirname(__file__), "golden", "fixtures",
                                "j1713_search.npz"))["input_profile"]
    sig = O.Signal(1400, 400, nchan=2, samprate=1.0 * 2048 * 10 ** -6, sublen=0.5)
    psr = O.Pulsar(1.0, 1.0, profiles=O.DataProfile(prof, nchan=2))
    O.make_pulses(sig, psr, 2.0, d)
    close(sig.data, A["data_pulses"], 1e-12)
    O.disperse(sig, 10.0)
    close(sig.data, A["data_disperse"])
    O.null(sig, psr, 0.34, d)
    close(sig.data, A["data_null"])
    out = O.observe(sig, psr, O.GBT(), "Lband_GUPPI", d, noise=True)
    close(out, A["out"], 1e-7)
    close(sig.data, A["data_noise"])
    check_meta(sig, meta)


def test_null_undelayed():
    meta, A, draws = load("null_undelayed")
    d = O.InjectedDraws(draws)
    sig = O.Signal(1400, 400, nchan=3, fold=False)
    psr = O.Pulsar(0.005, 2.0, profiles=O.GaussPortrait(0.45, 0.03, 1))
    O.make_pulses(sig, psr, 4096 * 20.48e-6, d)
    close(sig.data, A["data_pulses"], 1e-12)
    O.null(sig, psr, 0.3, d)
    close(sig.data, A["data_null"], 1e-12)
    O.disperse(sig, 5)
    close(sig.data, A["data_disperse"])
    out = O.observe(sig, psr, O.Arecibo(), "Lband_PUPPI", d, noise=False)
    close(out, A["out"], 1e-7)
    assert d.i == len(draws)


def test_specidx_int8():
    meta, A, draws = load("specidx_int8")
    d = O.InjectedDraws(draws)
    sig = O.Signal(1400, 400, nchan=4, dtype=np.int8)
    prof = O.GaussPortrait(np.array([0.3, 0.6]), np.array([0.02, 0.05]), np.array([0.5, 1.0]))
    psr = O.Pulsar(0.005, 1.0, profiles=prof, specidx=-1.6, ref_freq=1300)
    O.make_pulses(sig, psr, 1.0, d)
    close(sig.data, A["data_pulses"], 1e-12)
    O.disperse(sig, 20)
    close(sig.data, A["data_disperse"])
    out = O.observe(sig, psr, O.Arecibo(), "Lband_PUPPI", d, noise=True)
    assert out.dtype == np.int8
    # int8 truncation of values that agree to 1e-9 can only differ at exact
    # integer boundaries; require exact equality here (it holds).
    np.testing.assert_array_equal(out, A["out"])
    close(sig.data, A["data_noise"])
    check_meta(sig, meta)


@pytest.mark.parametrize("tag,dt_s", [("eq", 4.8828125e-06), ("down", 9.765625e-06), ("rebin", 7.5e-06)])
def test_observe_branches(tag, dt_s):
    meta, A, draws = load("observe_" + tag)
    d = O.InjectedDraws(draws)
    sig = O.Signal(1400, 400, nchan=2, fold=False, samprate=(1.0 / 0.005) * 2048 * 10 ** -6)
    psr = O.Pulsar(0.005, 10, profiles=O.GaussPortrait(0.5, 0.05, 1))
    O.make_pulses(sig, psr, 0.02, d)
    close(sig.data, A["data_pulses"], 1e-12)
    tel = O.Telescope(20.0, area=None, Tsys=25.0)
    # backend rate given as 1/Quantity(dt, 's') -> value in 1/s (scale 1)
    tel.systems["T"] = O.System(35.0, meta["backend_samprate_MHz"], samprate_scale=1.0)
    kind, _ = O.observe_branch(sig, meta["backend_samprate_MHz"], 1.0)
    assert kind == {"eq": "copy", "down": "down", "rebin": "rebin"}[tag]
    out = O.observe(sig, psr, tel, "T", d, noise=True)
    close(out, A["out"], 1e-7)
    close(sig.data, A["data_noise"], 1e-12)


def test_backend_fold():
    meta, A, draws = load("backend_fold")
    d = O.InjectedDraws(draws)
    sig = O.Signal(1400, 400, nchan=2, fold=False, samprate=(1.0 / 0.005) * 2048 * 10 ** -6)
    psr = O.Pulsar(0.005, 10, profiles=O.GaussPortrait(0.5, 0.05, 1))
    O.make_pulses(sig, psr, 0.02, d)
    close(O.backend_fold(sig, psr), A["folded"], 1e-13)


def test_utils_shift_downsample_rebin():
    meta, A, _ = load("utils")
    for i, (s, dt, isint) in enumerate(meta["shifts"]):
        s = int(s) if isint else s
        dt = int(dt) if isint else dt
        close(O.shift_t(A["y_even"], s, dt=dt), A["shift_even_%d" % i], 1e-12)
    close(O.shift_t(A["y_np2"], 4321.123, dt=1.0), A["shift_np2"], 1e-12)
    odd = O.shift_t(np.zeros(meta["odd_len_in"]), 3.3, dt=1.0)
    assert len(odd) == meta["odd_len_out"] == meta["odd_len_in"] - 1
    close(O.down_sample(A["ds_in"], 4), A["ds_4"], 1e-15)
    for n in (7, 100, 333, 1199):
        close(O.rebin(A["rebin_in"], n), A["rebin_%d" % n], 1e-15)


def test_baseband():
    """Baseband path (§8(f) row 4): amplitude pulses sqrt(PCHIP) x N(0,1)
    and coherent dispersion irfft(rfft x H) at the reference's own baseband
    test geometries, injected normal draws."""
    meta, A, draws = load("baseband")
    d = O.InjectedDraws(draws)
    for tag in ("a", "b", "c"):
        sr, per, tobs, dm = meta["geom_" + tag]
        sig = O.BasebandSignal(1400, 400, samprate=sr, nchan=2)
        psr = O.Pulsar(per, 10, profiles=None if tag == "c" else O.DataProfile(A["input_profile"]))
        O.make_amp_pulses(sig, psr, tobs, d)
        assert sig.nsamp == meta["nsamp_" + tag]
        assert np.isclose(sig.Smax, meta["Smax_" + tag], rtol=1e-12)
        close(sig.data, A["data_pulses_" + tag], 1e-12)
        # The reference's grid labels Hz as MHz (SURVEY §8 a-row note in
        # oracle.baseband_transfer), so the phase reaches ~7e10 rad at
        # geometry a: one float64 ulp of it is ~1e-5 rad, and any change of
        # operation order (the shim's unit scale included) moves H by that
        # much.  Tolerance: 4 ulp of the largest phase (b: ~1e-9).
        dt_s = (1.0 / sr) * 1e-6
        u = np.fft.rfftfreq(2 * (sig.nsamp // 2 + 1) - 1, d=dt_s)
        f = u - 200.0
        maxph = np.max(np.abs(2 * np.pi * O.DM_K / ((f + 1400.0) * 1400.0 ** 2) * dm * f ** 2 * 1e6))
        O.disperse_baseband(sig, dm)
        close(sig.data, A["data_disperse_" + tag], max(1e-9, 4 * maxph * 2.0 ** -53))
        with pytest.raises(ValueError):
            O.disperse_baseband(sig, dm)


def _simulate_oracle(d):
    """The reference's Simulation.simulate sequence (simulate.py:292-326) at
    tests/test_simulate.py's `simulation` fixture parameters, on the oracle."""
    sig = O.Signal(430, 100, nchan=64, samprate=1.0 * 2048 * 10 ** -6, sublen=2.0, fold=True)
    psr = O.Pulsar(1.0, 1.0, profiles=O.GaussPortrait())     # profiles=None -> default Gaussian
    O.scatter_broaden(sig, 50e-9, 1500.0, convolve=True, pulsar=psr)
    O.make_pulses(sig, psr, 4.0, d)
    O.disperse(sig, 10.0)
    tel = O.Telescope(100.0, area=5500.0, Tsys=35.0)
    tel.systems["TestSys"] = O.System(35.0, 1.5625)
    out = O.observe(sig, psr, tel, "TestSys", d, noise=True)
    return sig, psr, out


def test_simulate():
    """Simulation.simulate end to end, recorded from the reference
    (tests/golden/make_golden.py case_simulate)."""
    meta, A, draws = load("simulate")
    sig, psr, _ = _simulate_oracle(O.InjectedDraws(draws))
    assert sig.nsamp == meta["nsamp"] and sig.nsub == meta["nsub"]
    assert np.isclose(sig.Smax, meta["Smax"], rtol=1e-12)
    close(sig.data, A["data_final"], 1e-9)
