"""Self-written fold-mode PSRFITS writer (reference io/psrfits.py:305-424
layout; the reference's template-copy writer needs pdat/fitsio/PINT, absent
here, so parity of the file itself is unpinned: these tests check the
layout the reference's save() builds and a byte-exact round trip)."""
import numpy as np
import pytest

from psrsigsim_amd.io import PSRFITS, read_psrfits
from psrsigsim_amd._units import Quantity


class _FakeSig(object):
    def __init__(self, nchan, nsub, nbin, rng):
        self.Nchan = nchan
        self.nsub = nsub
        self.samprate = Quantity(nbin * 1e-6, "MHz")     # 1-s period -> nbin samples
        self.sublen = Quantity(2.0, "s")
        self.tobs = Quantity(2.0 * nsub, "s")
        self.fcent = Quantity(430.0, "MHz")
        self.bw = Quantity(100.0, "MHz")
        self.dat_freq = Quantity(380.0 + np.arange(nchan) * 100.0 / nchan, "MHz")
        self.dm = Quantity(10.0, "pc/cm^3")
        self.data = rng.normal(0, 300, (nchan, nsub * nbin + 7))


class _FakePsr(object):
    name = "J0000+0000"
    period = Quantity(1.0, "s")


def test_psrfits_layout_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    sig = _FakeSig(8, 3, 128, rng)
    path = str(tmp_path / "sim.fits")
    PSRFITS(path=path).save(sig, _FakePsr(), ref_MJD=56000.25, MJD_start=56000.25)
    prim, sub, rec = read_psrfits(path)
    assert prim["OBS_MODE"] == "PSR" and prim["OBSNCHAN"] == 8 and prim["SRC_NAME"] == "J0000+0000"
    assert prim["OBSFREQ"] == 430.0 and prim["OBSBW"] == 100.0 and prim["CHAN_DM"] == 10.0
    assert prim["STT_IMJD"] == 56000 and prim["STT_SMJD"] == 21600 and prim["STT_OFFS"] == 0.0
    assert sub["NBIN"] == 128 and sub["NCHAN"] == 8 and sub["NPOL"] == 1 and sub["POL_TYPE"] == "AA+BB"
    assert sub["TBIN"] == 1.0 / 128 and sub["CHAN_BW"] == 12.5 and sub["DM"] == 10.0
    assert rec.shape == (3,)
    np.testing.assert_array_equal(rec["OFFS_SUB"], [1.0, 3.0, 5.0])       # sublen/2 + i sublen
    np.testing.assert_array_equal(rec["TSUBINT"], 2.0)
    np.testing.assert_array_equal(rec["DAT_FREQ"][1], np.asarray(sig.dat_freq.value))
    np.testing.assert_array_equal(rec["DAT_WTS"], 1.0)
    np.testing.assert_array_equal(rec["DAT_SCL"], 1.0)
    np.testing.assert_array_equal(rec["DAT_OFFS"], 0.0)
    d16 = sig.data[:, :3 * 128].astype(np.int16)
    for i in range(3):                               # Out[i, 0] = data[:, i nbin:(i+1) nbin] ('>i2')
        np.testing.assert_array_equal(rec["DATA"][i, 0], d16[:, i * 128:(i + 1) * 128])
    raw = open(path, "rb").read()
    assert len(raw) % 2880 == 0 and raw[:30] == b"SIMPLE  =                    T"


def test_psrfits_refuses_template():
    with pytest.raises(NotImplementedError):
        PSRFITS(path="x.fits", template="data/B1855+09.L-wide.PUPPI.11y.x.sum.sm", fits_mode="copy")


@pytest.mark.gpu
def test_psrfits_from_device_simulation(tmp_path, hip_lib):
    """A fold-mode simulation on the GPU written to PSRFITS: DATA is the
    device data truncated to int16."""
    import psrsigsim_amd as pss
    from psrsigsim_amd.simulate import Simulation
    pss.seed(2)
    sim = Simulation(fcent=430, bandwidth=100, sample_rate=1.0 * 2048 * 10 ** -6, Nchan=16, sublen=2.0, fold=True,
                     period=1.0, Smean=1.0, profiles=[0.5, 0.05, 1.0], tobs=6.0, name="J0000+0000", dm=10.0,
                     tscope_name="Arecibo", system_name="Lband_PUPPI")
    sim.simulate()
    path = str(tmp_path / "dev.fits")
    PSRFITS(path=path).save(sim.signal, sim.pulsar)
    prim, sub, rec = read_psrfits(path)
    d = sim.signal.data.cpu().numpy()
    nbin = sub["NBIN"]
    assert nbin == 2048 and rec.shape == (3,)
    np.testing.assert_array_equal(rec["DATA"][2, 0], np.trunc(d[:, 2 * nbin:3 * nbin]).astype(np.int16))


TEMPLATE = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))), "data", "B1855+09.L-wide.PUPPI.11y.x.sum.sm")


def test_read_reference_template():
    """The reference's PSRFITS template (data/B1855+09.L-wide.PUPPI.11y.x.sum.sm,
    config C4's portrait) parses: its HDUs, the SUBINT header and the int16
    DATA with its scale/offset (outval = DATA * DAT_SCL + DAT_OFFS)."""
    from psrsigsim_amd.io.psrfits import read_fits, template_profile
    h = read_fits(TEMPLATE)
    assert list(h) == ["PRIMARY", "HISTORY", "PSRPARAM", "POLYCO", "SUBINT"]
    prim, _ = h["PRIMARY"]
    sub, rec = h["SUBINT"]
    assert prim["OBS_MODE"] == "PSR" and prim["SRC_NAME"] == "B1855+09"
    assert sub["NBIN"] == 2048 and sub["NCHAN"] == 1 and sub["NPOL"] == 1 and sub["DM"] == 13.299393
    assert rec.shape == (1,) and rec["DATA"].dtype == np.dtype(">i2") and rec["DATA"].shape == (1, 1, 1, 2048)
    raw = rec["DATA"][0, 0, 0].astype(np.float64)
    prof = template_profile(TEMPLATE, baseline=None)
    np.testing.assert_array_equal(prof, raw * np.float64(rec["DAT_SCL"][0]) + np.float64(rec["DAT_OFFS"][0]))
    p2 = template_profile(TEMPLATE)
    assert abs(np.median(p2)) < 1e-12 and np.argmax(p2) == np.argmax(raw)
    # the PSRPARAM table holds the pulsar frequency the reference reads (F0)
    pp = h["PSRPARAM"][1]
    lines = [bytes(x).decode().strip() for x in pp["PARAM"]]
    assert lines[0].split() == ["PSR", "B1855+09"]
    assert any(l.split()[0] in ("F0", "F") for l in lines)


def test_writer_subint_layout_matches_template(tmp_path):
    """The writer's SUBINT columns -- names, order, TFORM codes and repeat
    counts, TDIM of DATA -- are the template's, at the template's geometry
    (1 channel x 2048 bins), so the row layouts are identical."""
    from psrsigsim_amd.io.psrfits import read_fits
    rng = np.random.default_rng(3)
    sig = _FakeSig(1, 2, 2048, rng)
    path = str(tmp_path / "one.fits")
    PSRFITS(path=path).save(sig, _FakePsr())
    ours, rec = read_fits(path)["SUBINT"]
    tmpl, trec = read_fits(TEMPLATE)["SUBINT"]
    nf = int(tmpl["TFIELDS"])
    assert int(ours["TFIELDS"]) == nf

    def form(h, i):
        f = str(h["TFORM%d" % i]).strip()
        k = len(f) - len(f.lstrip("0123456789"))
        return int(f[:k] or 1), f[k]
    for i in range(1, nf + 1):
        assert ours["TTYPE%d" % i] == tmpl["TTYPE%d" % i], i
        assert form(ours, i) == form(tmpl, i), (i, ours["TTYPE%d" % i])
    idx = [i for i in range(1, nf + 1) if tmpl["TTYPE%d" % i] == "DATA"][0]
    assert ours["TDIM%d" % idx].replace(" ", "") == tmpl["TDIM%d" % idx].replace(" ", "")
    assert rec.dtype == trec.dtype and ours["NAXIS1"] == tmpl["NAXIS1"]
    for k in ("NBIN", "NCHAN", "NPOL", "NSBLK"):
        assert ours[k] == tmpl[k], k
