"""Simulation driver (reference simulate/simulate.py) and the pdv writer
(io/txtfile.py).  Parameters follow the reference's own tests/test_simulate.py
fixtures."""
import glob
import os

import numpy as np
import pytest


def _param_dict():
    return {'fcent': 430, 'bandwidth': 100, 'sample_rate': 1.5625, 'dtype': np.float32, 'Npols': 1,
            'Nchan': 64, 'sublen': 2.0, 'fold': True, 'period': 1.0, 'Smean': 1.0,
            'profiles': [0.5, 0.5, 1.0], 'tobs': 4.0, 'name': 'J0000+0000', 'dm': 10.0,
            'tau_d': 50e-9, 'tau_d_ref_f': 1500.0, 'aperture': 100.0, 'area': 5500.0, 'Tsys': 35.0,
            'tscope_name': "TestScope", 'system_name': "TestSys", 'rcvr_fcent': 430, 'rcvr_bw': 100,
            'rcvr_name': "TestRCVR", 'backend_samprate': 1.5625, 'backend_name': "TestBack",
            'tempfile': None, 'parfile': None}


def _sim(**kw):
    from psrsigsim_amd.simulate import Simulation
    args = dict(fcent=430, bandwidth=100, sample_rate=1.0 * 2048 * 10 ** -6, dtype=np.float32, Npols=1,
                Nchan=64, sublen=2.0, fold=True, period=1.0, Smean=1.0, profiles=None, tobs=4.0,
                name='J0000+0000', dm=10.0, tau_d=50e-9, tau_d_ref_f=1500.0, aperture=100.0, area=5500.0,
                Tsys=35.0, tscope_name="TestScope", system_name="TestSys", rcvr_fcent=430, rcvr_bw=100,
                rcvr_name="TestRCVR", backend_samprate=1.5625, backend_name="TestBack", tempfile=None,
                parfile=None, psrdict=None)
    args.update(kw)
    return Simulation(**args)


def test_init_from_dict_and_par():
    from psrsigsim_amd.simulate import Simulation
    sim = Simulation(psrdict=_param_dict())
    assert sim.Nchan == 64 and sim.samprate == 1.5625 and sim.tscope_name == "TestScope"
    with pytest.raises(NotImplementedError):
        Simulation(parfile="testpar.par")


def test_init_stages_host():
    from psrsigsim_amd.pulsar import GaussPortrait, DataProfile
    sim = _sim()
    sim.init_signal()
    assert sim.signal.Nchan == 64
    with pytest.raises(ValueError):                  # no template file (tempfile=None)
        sim.init_signal(from_template=True)
    sim.init_profile()                               # None -> default Gaussian
    assert isinstance(sim.profiles, GaussPortrait)
    sim2 = _sim(profiles=[0.5, 0.5, 1.0])
    sim2.init_profile()
    assert isinstance(sim2.profiles, GaussPortrait)
    sim3 = _sim(profiles=np.exp(-0.5 * ((np.arange(64) / 64.0 - 0.5) / 0.05) ** 2))
    sim3.init_profile()
    assert isinstance(sim3.profiles, DataProfile)
    with pytest.raises(RuntimeError):
        _sim(profiles=[0.5, 0.5]).init_profile()
    sim.init_pulsar()
    sim.init_ism()
    sim.init_telescope()
    assert "TestSys" in sim.tscope.systems
    multi = _sim(system_name=["A", "B"], rcvr_fcent=[430, 1400], rcvr_bw=[100, 400], rcvr_name=["R1", "R2"],
                 backend_samprate=[1.5625, 12.5], backend_name=["B1", "B2"])
    multi.init_telescope()
    assert set(multi.tscope.systems) >= {"A", "B"}
    bad = _sim(system_name=["A"], rcvr_fcent=[430, 1400], rcvr_bw=[100], rcvr_name=["R1"],
               backend_samprate=[1.5625], backend_name=["B1"])
    with pytest.raises(RuntimeError):
        bad.init_telescope()


def test_save_errors():
    sim = _sim()
    with pytest.raises(RuntimeError):
        sim.save_simulation(out_format="psrfits")        # no template, as in the reference
    with pytest.raises(RuntimeError):
        sim.save_simulation(out_format="hdf5")


@pytest.mark.gpu
def test_simulate_vs_reference_fixture(hip_lib):
    """simulate() on the GPU with the reference's own recorded draws
    injected, against the reference's Simulation.simulate output at its
    tests/test_simulate.py `simulation` fixture parameters
    (tests/golden/fixtures/simulate.*, recorded by make_golden.py)."""
    import psrsigsim_amd as pss
    from tests.fixtures_util import load
    from tests.replay import _err
    meta, A, draws = load("simulate")
    sim = _sim()
    pss.inject(gen=draws[0][2])
    # the noise draws are consumed by observe(), the last stage
    pss.inject(noise=draws[1][2])
    sim.simulate()
    got = sim.signal.data.cpu().numpy()
    assert sim.signal.nsamp == meta["nsamp"] and got.shape == A["data_final"].shape
    assert abs(float(getattr(sim.signal._Smax, "value", sim.signal._Smax)) / meta["Smax"] - 1) < 1e-12
    assert _err(got, A["data_final"]) <= 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("rate", [1.5625, 1.0 * 2048 * 10 ** -6], ids=["fixture", "2048bin"])
def test_simulate_equals_manual_calls(rate, hip_lib):
    """simulate() = the reference's call sequence (simulate.py:292-326) made
    by hand with the same seed: bitwise (one fused run either way).  The
    reference fixture's 1.5625 MHz gives 3 125 000 = 2^3 5^8 samples per
    channel (radix-5 four-step 1250 x 2500); the 2048-bin variant is a power
    of two."""
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussPortrait
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import Telescope, Receiver, Backend
    pss.seed(5)
    p = _param_dict()
    p['sample_rate'] = rate
    sim = _sim(psrdict=p)
    sim.simulate()
    got = sim.signal.data.cpu().numpy()
    pss.seed(5)
    sig = FilterBankSignal(p['fcent'], p['bandwidth'], Nsubband=p['Nchan'], sample_rate=p['sample_rate'],
                           fold=True, sublen=p['sublen'])
    psr = Pulsar(p['period'], p['Smean'], profiles=GaussPortrait(peak=0.5, width=0.5, amp=1.0), name=p['name'])
    ism = ISM()
    ism.scatter_broaden(sig, p['tau_d'], p['tau_d_ref_f'], convolve=True, pulsar=psr)
    psr.make_pulses(sig, tobs=p['tobs'])
    ism.disperse(sig, p['dm'])
    tel = Telescope(p['aperture'], area=p['area'], Tsys=p['Tsys'], name=p['tscope_name'])
    tel.add_system(name=p['system_name'], receiver=Receiver(fcent=430, bandwidth=100, name="TestRCVR"),
                   backend=Backend(samprate=1.5625, name="TestBack"))
    tel.observe(sig, psr, system=p['system_name'], noise=True)
    np.testing.assert_array_equal(got, sig.data.cpu().numpy())
    assert np.isfinite(got).all() and got.shape[0] == 64


@pytest.mark.gpu
def test_save_pdv(tmp_path, hip_lib):
    import psrsigsim_amd as pss
    pss.seed(3)
    sim = _sim(Nchan=8)
    sim.simulate()
    out = str(tmp_path / "sim")
    sim.save_simulation(outfile=out, out_format="pdv")
    files = sorted(glob.glob(out + "_*.txt"))
    assert files == [out + "_0.txt"]
    lines = open(files[0]).read().splitlines()
    nbin = 2048                                      # samprate 2048e-6 MHz x 1 s
    assert lines[0].startswith("# File: %s Src: J0000+0000 Nsub: 2 Nch: 8 Npol: 1 Nbin: %d RMS: " % (out, nbin))
    assert len(lines) == 1 + 2 * 8 * (1 + nbin)
    d = sim.signal.data.cpu().numpy()
    f, b = 5, 77
    assert lines[1 + 8 * (1 + nbin) + f * (1 + nbin) + 1 + b] == "1 %d %d %s " % (f, b, d[f, b])
    assert os.path.getsize(files[0]) > 0
