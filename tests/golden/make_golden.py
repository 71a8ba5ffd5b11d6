#!/usr/bin/env python
"""Generate the golden vectors that pin the oracle (TEST INFRASTRUCTURE ONLY).

Runs the *unmodified* reference PsrSigSim from /root/reference (survey
container only; the reference never travels to the GPU box) through the
test-only astropy.units stand-in in ``tests/golden/refshim`` and records, for a
set of small cases modelled on the reference's own test geometries
(SURVEY.md §4, §8(c)):

* every random draw the reference consumed, in order (scipy ``chi2.rvs`` and
  ``np.random.choice`` are wrapped and recorded), so that the oracle and the
  HIP path can replay them exactly ("draw injection");
* the signal data after every stage (make_pulses, each delay stage, null,
  observe noise) and observe's returned array;
* every derived scalar/integer (nsamp, Nph, nsub, Nfold, Smax, draw_norm,
  per-stage delays, profile knot tables, ...).

Outputs: ``tests/golden/fixtures/<case>.npz`` (plain arrays, no pickles) and
``<case>.json``.  Re-run with ``python -B tests/golden/make_golden.py``.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("PSS_REFERENCE", "/root/reference")
OUT = os.path.join(HERE, "fixtures")
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(HERE, "refshim"))
sys.path.insert(0, REF)

import scipy.stats._continuous_distns as _cd  # noqa: E402

import psrsigsim  # noqa: E402,F401
from psrsigsim.signal.fb_signal import FilterBankSignal  # noqa: E402
from psrsigsim.pulsar.pulsar import Pulsar  # noqa: E402
from psrsigsim.pulsar.profiles import GaussProfile, DataProfile  # noqa: E402
from psrsigsim.ism.ism import ISM  # noqa: E402
from psrsigsim.telescope import telescope as _tel  # noqa: E402
from psrsigsim.telescope.telescope import Telescope  # noqa: E402
from psrsigsim.telescope.receiver import Receiver  # noqa: E402
from psrsigsim.telescope.backend import Backend  # noqa: E402
from psrsigsim.utils import utils as _ut  # noqa: E402
from astropy import units as u  # noqa: E402  (the shim)

# --------------------------------------------------------------------------
# draw recorder
# --------------------------------------------------------------------------
_DRAWS = []
_orig_rvs = _cd.chi2_gen._rvs
_orig_choice = np.random.choice


def _rec_rvs(self, df, size=None, random_state=None):
    out = _orig_rvs(self, df, size=size, random_state=random_state)
    _DRAWS.append(("chi2", float(np.asarray(df)), np.array(out, dtype=np.float64)))
    return out


def _rec_choice(a, size=None, replace=True, p=None):
    out = _orig_choice(a, size, replace=replace, p=p)
    _DRAWS.append(("choice", float(a), np.array(out, dtype=np.int64)))
    return out


_orig_norm = _cd.norm_gen._rvs


def _rec_norm(self, size=None, random_state=None):
    out = _orig_norm(self, size=size, random_state=random_state)
    _DRAWS.append(("normal", 0.0, np.array(out, dtype=np.float64)))
    return out


_cd.chi2_gen._rvs = _rec_rvs
_cd.norm_gen._rvs = _rec_norm
np.random.choice = _rec_choice


def _v(q):
    """Plain float/ndarray value of a shim Quantity (or pass through)."""
    if hasattr(q, "value"):
        v = q.value
        return float(v) if np.ndim(v) == 0 else np.array(v, dtype=np.float64)
    return q


class Case(object):
    def __init__(self, name, seed):
        self.name = name
        self.arrays = {}
        self.meta = {"case": name, "seed": seed, "stages": [], "draws": []}
        _DRAWS.clear()
        np.random.seed(seed)

    def snap(self, tag, sig, **extra):
        self.arrays["data_" + tag] = np.array(sig.data, dtype=np.float64)
        st = {"tag": tag, "ndraws": len(_DRAWS)}
        st.update(extra)
        self.meta["stages"].append(st)

    def signal_meta(self, sig):
        m = self.meta
        m["Nchan"] = int(sig.Nchan)
        m["fcent"] = _v(sig.fcent)
        m["bw"] = _v(sig.bw)
        m["samprate_MHz"] = _v(sig.samprate)
        m["fold"] = bool(sig.fold)
        m["dtype"] = np.dtype(sig.dtype).name
        m["draw_max"] = float(sig._draw_max)
        m["draw_norm"] = float(sig._draw_norm)
        self.arrays["dat_freq"] = _v(sig.dat_freq)
        for k in ("_tobs", "_nsamp", "_nsub", "_sublen", "_Nfold", "_Smax"):
            if getattr(sig, k, None) is not None:
                m[k.lstrip("_")] = _v(getattr(sig, k))
        if sig.delay is not None:
            self.arrays["delay_ms"] = _v(sig.delay)
        if getattr(sig, "_dm", None) is not None:
            m["dm"] = _v(sig._dm)

    def profile_meta(self, psr):
        pr = psr.Profiles
        gen = getattr(pr, "_generator", None)
        if gen is not None:
            self.arrays["pchip_x"] = np.array(gen.x, dtype=np.float64)
            self.arrays["pchip_c"] = np.array(gen.c, dtype=np.float64)
        if getattr(pr, "_profiles", None) is not None:
            self.arrays["profiles"] = np.array(pr._profiles, dtype=np.float64)
        self.arrays["max_profile"] = np.array(pr._max_profile, dtype=np.float64)
        self.meta["Amax"] = float(pr.Amax) if getattr(pr, "_Amax", None) is not None else None

    def save(self):
        for i, (kind, df, arr) in enumerate(_DRAWS):
            self.arrays["draw%02d" % i] = arr
            self.meta["draws"].append({"kind": kind, "df": df, "shape": list(arr.shape)})
        os.makedirs(OUT, exist_ok=True)
        np.savez_compressed(os.path.join(OUT, self.name + ".npz"), **self.arrays)
        with open(os.path.join(OUT, self.name + ".json"), "w") as f:
            json.dump(self.meta, f, indent=1, sort_keys=True, default=float)
        print("wrote", self.name, sorted(self.arrays), file=sys.stderr)


def _observe(case, tel, sig, psr, system, noise=True):
    out = tel.observe(sig, psr, system=system, noise=noise, ret_resampsig=True)
    case.arrays["out"] = np.array(out)
    case.meta["out_dtype"] = np.dtype(out.dtype).name
    bak = tel.systems[system][1]
    case.meta["backend_samprate_MHz"] = _v(bak.samprate)
    rc = tel.systems[system][0]
    case.meta["Trec"] = _v(rc.Trec)
    case.meta["tel_Tsys"] = _v(tel.Tsys) if tel.Tsys is not None else None
    case.meta["tel_area"] = _v(tel.area)
    case.meta["tel_gain"] = _v(tel.gain.to("K/Jy"))


# --------------------------------------------------------------------------
# cases
# --------------------------------------------------------------------------
def case_tutorial1():
    """C1: docs/tutorial_1 geometry (fold, nsub=1, N=244 = 2^2*61)."""
    c = Case("tutorial1", 1776)
    sig = FilterBankSignal(1400, 400, Nsubband=2)
    psr = Pulsar(0.005, 10, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, tobs=1.0)
    c.snap("pulses", sig)
    c.profile_meta(psr)
    ISM().disperse(sig, 10)
    c.snap("disperse", sig)
    _observe(c, _tel.Arecibo(), sig, psr, "Lband_PUPPI")
    c.snap("noise", sig)
    c.signal_meta(sig)
    c.save()


def case_northstar_mini():
    """C3 in miniature: search mode, GaussProfile P=5 ms, scatter convolve,
    DM=100 (delays wrap), FD + scatter shift, delayed null, Arecibo noise."""
    c = Case("northstar_mini", 1776)
    sig = FilterBankSignal(1400, 400, Nsubband=4, fold=False)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    ism = ISM()
    ism.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    c.arrays["convolved_profiles"] = np.array(psr.Profiles._generator.c[-1], dtype=np.float64)
    psr.make_pulses(sig, tobs=8192 * 20.48e-6)
    c.snap("pulses", sig)
    c.profile_meta(psr)
    ism.disperse(sig, 100)
    c.snap("disperse", sig)
    ism.FD_shift(sig, [2e-4, -3e-5])
    c.snap("fd", sig)
    ism.scatter_broaden(sig, 3e-4, 1400, convolve=False)
    c.snap("scatter", sig)
    psr.null(sig, 0.1)
    c.snap("null", sig)
    _observe(c, _tel.Arecibo(), sig, psr, "Lband_PUPPI")
    c.snap("noise", sig)
    c.signal_meta(sig)
    c.save()


def case_j1713_search():
    """C2 in miniature: DataProfile(J1713), NANOGrav P, DM 15.917131, GBT."""
    c = Case("j1713_search", 4242)
    prof = np.load(os.path.join(REF, "psrsigsim/data/J1713+0747_profile.npy"))
    c.arrays["input_profile"] = np.array(prof, dtype=np.float64)
    sig = FilterBankSignal(1500, 800, Nsubband=4, sample_rate=0.048828125, fold=False)
    psr = Pulsar(1.0 / 218.8118437960826270, 0.009, profiles=DataProfile(prof, Nchan=4))
    psr.make_pulses(sig, tobs=4096 * 20.48e-6)
    c.snap("pulses", sig)
    c.profile_meta(psr)
    ISM().disperse(sig, 15.917131)
    c.snap("disperse", sig)
    _observe(c, _tel.GBT(), sig, psr, "Lband_GUPPI")
    c.snap("noise", sig)
    c.signal_meta(sig)
    c.save()


def case_fold_sublen():
    """tests/test_pulsar.py fbsignal geometry: fold, sublen 0.5 s, nsub=4,
    Nph=2048, J1713 profile, disperse + delayed null(0.34), GBT noise."""
    c = Case("fold_sublen", 7)
    prof = np.load(os.path.join(REF, "psrsigsim/data/J1713+0747_profile.npy"))
    sig = FilterBankSignal(1400, 400, Nsubband=2, sample_rate=1.0 * 2048 * 10 ** -6, sublen=0.5)
    psr = Pulsar(1.0, 1.0, profiles=DataProfile(prof, phases=None, Nchan=2))
    psr.make_pulses(sig, 2.0)
    c.snap("pulses", sig)
    c.profile_meta(psr)
    ISM().disperse(sig, 10.0)
    c.snap("disperse", sig)
    psr.null(sig, 0.34)
    c.snap("null", sig)
    _observe(c, _tel.GBT(), sig, psr, "Lband_GUPPI")
    c.snap("noise", sig)
    c.signal_meta(sig)
    c.save()


def case_null_undelayed():
    """null() before any delay (the undelayed branch), then disperse."""
    c = Case("null_undelayed", 99)
    sig = FilterBankSignal(1400, 400, Nsubband=3, fold=False)
    psr = Pulsar(0.005, 2.0, profiles=GaussProfile(0.45, 0.03, 1))
    psr.make_pulses(sig, tobs=4096 * 20.48e-6)
    c.snap("pulses", sig)
    c.profile_meta(psr)
    psr.null(sig, 0.3)
    c.snap("null", sig)
    ISM().disperse(sig, 5)
    c.snap("disperse", sig)
    _observe(c, _tel.Arecibo(), sig, psr, "Lband_PUPPI", noise=False)
    c.signal_meta(sig)
    c.save()


def case_specidx_int8():
    """fold, int8 dtype (draw_norm from chi2.ppf), multi-Gaussian profile,
    spectral index with explicit ref_freq."""
    c = Case("specidx_int8", 5)
    sig = FilterBankSignal(1400, 400, Nsubband=4, dtype=np.int8)
    prof = GaussProfile(np.array([0.3, 0.6]), np.array([0.02, 0.05]), np.array([0.5, 1.0]))
    psr = Pulsar(0.005, 1.0, profiles=prof, specidx=-1.6, ref_freq=1300)
    psr.make_pulses(sig, tobs=1.0)
    c.snap("pulses", sig)
    c.profile_meta(psr)
    ISM().disperse(sig, 20)
    c.snap("disperse", sig)
    _observe(c, _tel.Arecibo(), sig, psr, "Lband_PUPPI")
    c.snap("noise", sig)
    c.signal_meta(sig)
    c.save()


def _sampling_signal():
    sig = FilterBankSignal(1400, 400, Nsubband=2, fold=False, sample_rate=(1.0 / 0.005) * 2048 * 10 ** -6)
    psr = Pulsar(0.005, 10, profiles=GaussProfile(0.5, 0.05, 1))
    return sig, psr


def case_observe_branches():
    """tests/test_telescope.py::test_sampling geometry: the ==, %==0
    (down_sample) and rebin branches of Telescope.observe, plus Backend.fold."""
    for tag, dt_s in (("eq", 4.8828125e-06), ("down", 9.765625e-06), ("rebin", 7.5e-06)):
        c = Case("observe_" + tag, 11)
        sig, psr = _sampling_signal()
        psr.make_pulses(sig, 0.02)
        c.snap("pulses", sig)
        c.profile_meta(psr)
        tel = Telescope(20.0, area=None, Tsys=25.0, name="Twenty_Meter")
        tel.add_system(name="T", receiver=Receiver(fcent=1400, bandwidth=400, name="Lband"),
                       backend=Backend(samprate=1.0 / u.Quantity(dt_s, "s"), name="Cyborg"))
        _observe(c, tel, sig, psr, "T")
        c.snap("noise", sig)
        c.signal_meta(sig)
        c.save()
    c = Case("backend_fold", 12)
    sig, psr = _sampling_signal()
    psr.make_pulses(sig, 0.02)
    c.snap("pulses", sig)
    bk = Backend(samprate=(1.0 / u.Quantity(81.92, "us")).to("MHz"), name="Cyborg")
    c.arrays["folded"] = np.array(bk.fold(sig, psr))
    c.signal_meta(sig)
    c.save()


def case_utils():
    """shift_t / down_sample / rebin on seeded inputs (no astropy needed)."""
    c = Case("utils", 0)
    rng = np.random.RandomState(0)
    y_even = rng.standard_normal(4096)
    y_odd = rng.standard_normal(1001)
    y_np2 = rng.standard_normal(48828)
    c.arrays["y_even"] = y_even
    c.arrays["y_np2"] = y_np2
    shifts = [(0.37, 1.0), (2, 1), (-13.25, 1.0), (1234.5, 0.5), (5000.0, 1.0), (0.5, 1.0)]
    c.meta["shifts"] = [[float(s), float(d), isinstance(s, int)] for s, d in shifts]
    for i, (s, d) in enumerate(shifts):
        c.arrays["shift_even_%d" % i] = _ut.shift_t(y_even, s, dt=d)
    c.arrays["shift_np2"] = _ut.shift_t(y_np2, 4321.123, dt=1.0)
    odd = _ut.shift_t(y_odd, 3.3, dt=1.0)
    c.meta["odd_len_in"] = 1001
    c.meta["odd_len_out"] = int(len(odd))
    y = rng.standard_normal(1200)
    c.arrays["ds_in"] = y
    c.arrays["ds_4"] = _ut.down_sample(y, 4)
    c.arrays["rebin_in"] = y
    for n in (7, 100, 333, 1199):
        c.arrays["rebin_%d" % n] = _ut.rebin(y, n)
    c.save()


def case_baseband():
    """Baseband path at the reference's own test
    geometries: tests/test_ism.py bbsignal (1400 MHz, 400 MHz, 1.024 MHz
    sampling, 2 pols) with the J1713 DataProfile, P = 5 ms, tobs 0.05 s
    (51 200 samples), disperse(10); and tests/test_pulsar.py bbsignal
    (2.048 kHz sampling, P = 1 s, tobs 2 s: 4096 samples), disperse(3)."""
    from psrsigsim.signal.bb_signal import BasebandSignal
    c = Case("baseband", 1746)
    prof = np.load(os.path.join(REF, "psrsigsim/data/J1713+0747_profile.npy"))
    c.arrays["input_profile"] = np.array(prof, dtype=np.float64)
    for tag, (sr, per, tobs, dm) in (("a", (500.0 * 2048 * 10 ** -6, 0.005, 0.05, 10.0)),
                                     ("b", (1.0 * 2048 * 10 ** -6, 1.0, 2.0, 3.0)),
                                     ("c", (1.024, 0.005, 0.02, 10.0))):
        sig = BasebandSignal(1400, 400, sample_rate=sr, Nchan=2)
        # c: the default GaussProfile (tests/test_telescope.py::test_bb_obs
        # makes amplitude pulses with it), at a fixture-sized geometry
        pro = None if tag == "c" else DataProfile(prof)
        psr = Pulsar(per, 10, profiles=pro, name='J1746-0118')
        psr.make_pulses(sig, tobs)
        c.snap("pulses_" + tag, sig)
        c.meta["nsamp_" + tag] = int(sig.nsamp)
        c.meta["Smax_" + tag] = float(_v(sig._Smax))
        ISM().disperse(sig, dm)
        c.snap("disperse_" + tag, sig)
        c.meta["geom_" + tag] = [sr, per, tobs, dm]
    c.save()


def case_simulate():
    """Simulation.simulate (simulate/simulate.py:292-326) end to end with the
    reference's own tests/test_simulate.py `simulation` fixture parameters
    (430 MHz, 100 MHz, 64 channels, 2048e-6 MHz sampling, fold with 2-s
    subints, P = 1 s, default Gaussian profile, tobs 4 s, DM 10, scattering
    tau_d 50 ns @ 1500 MHz, TestScope 100 m / 5500 m^2 / 35 K, TestSys
    backend 1.5625 MHz); the template-file argument is not used by
    simulate(from_template=False)."""
    from psrsigsim.simulate.simulate import Simulation
    c = Case("simulate", 2023)
    sim = Simulation(fcent=430, bandwidth=100, sample_rate=1.0 * 2048 * 10 ** -6, dtype=np.float32, Npols=1,
                     Nchan=64, sublen=2.0, fold=True, period=1.0, Smean=1.0, profiles=None, tobs=4.0,
                     name='J0000+0000', dm=10.0, tau_d=50e-9, tau_d_ref_f=1500.0, aperture=100.0, area=5500.0,
                     Tsys=35.0, tscope_name="TestScope", system_name="TestSys", rcvr_fcent=430, rcvr_bw=100,
                     rcvr_name="TestRCVR", backend_samprate=1.5625, backend_name="TestBack", tempfile=None,
                     parfile=None, psrdict=None)
    sim.simulate()
    c.snap("final", sim.signal)
    c.signal_meta(sim.signal)
    c.meta["Amax"] = float(sim.pulsar.Profiles.Amax)
    c.save()


if __name__ == "__main__":
    if sys.argv[1:]:
        for name in sys.argv[1:]:
            globals()["case_" + name]()
        sys.exit(0)
    case_tutorial1()
    case_northstar_mini()
    case_j1713_search()
    case_fold_sublen()
    case_null_undelayed()
    case_specidx_int8()
    case_observe_branches()
    case_utils()
    case_baseband()
    case_simulate()
