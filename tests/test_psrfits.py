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
        self.nsamp = nsub * nbin
        self.Npols = 1


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


_PRIMARY_EDITS = ("OBSFREQ", "OBSBW", "CHAN_DM", "STT_IMJD", "STT_SMJD", "STT_OFFS", "BE_DELAY")
_DELETED = ("BINARY", "A1", "E", "T0", "PB", "OM", "SINI", "M2", "F1", "PMDEC", "PMRA", "TZRMJD", "TZRFRQ",
            "TZRSITE")


def _cards(h):
    return {c[:8].rstrip(): c for c in h["cards"]}


def _template_copy(tmp_path, monkeypatch, sig, **kw):
    from psrsigsim_amd.io.psrfits import _raw_hdus
    monkeypatch.chdir(tmp_path)                     # make_par writes <name>_sim.par here
    path = str(tmp_path / "tpl.fits")
    pf = PSRFITS(path=path, template=TEMPLATE, fits_mode="copy", obs_mode="PSR")
    pf.get_signal_params(signal=sig)
    pf.save(sig, _FakePsr(), **kw)
    return _raw_hdus(path), _raw_hdus(TEMPLATE), path


def test_template_copy_bytes_and_reference_edits(tmp_path, monkeypatch):
    """Template mode (psrfits.py:305-424, the reference's only mode): the
    HDUs come in the template's order; POLYCO is byte-identical (PINT absent:
    not regenerated); every PRIMARY / HISTORY / PSRPARAM / SUBINT card image
    and table byte the reference does not edit is the template's; the edited
    ones follow the reference's formulas (_gen_metadata's MJD split,
    _edit_psrfits_header's HISTORY / SUBINT values and PSRPARAM deletions);
    DATA is numpy's astype('>i2') of the data, out-of-range values (wrapped)
    included (psrfits.py:353)."""
    rng = np.random.default_rng(7)
    sig = _FakeSig(8, 3, 128, rng)
    sig.data[0, :5] = [40000.7, -40000.7, 1e10, 70000.2, -1e10]   # beyond int16
    ours, tmpl, path = _template_copy(tmp_path, monkeypatch, sig, ref_MJD=56000.0, MJD_start=55999.9861)
    assert [h["name"] for h in ours] == [h["name"] for h in tmpl] == \
        ["PRIMARY", "HISTORY", "PSRPARAM", "POLYCO", "SUBINT"]
    O, T = {h["name"]: h for h in ours}, {h["name"]: h for h in tmpl}
    # POLYCO: verbatim
    assert O["POLYCO"]["cards"] == T["POLYCO"]["cards"] and O["POLYCO"]["data"] == T["POLYCO"]["data"]
    # PRIMARY: verbatim but the reference's primary_dict keys
    co, ct = _cards(O["PRIMARY"]), _cards(T["PRIMARY"])
    assert set(co) == set(ct)
    assert all(co[k] == ct[k] for k in ct if k not in _PRIMARY_EDITS)
    ph = O["PRIMARY"]["hdr"]
    # inc_len = MJD_start - ref_MJD = -0.0139 d: MJD 56000 + floor(-0.0139) = 55999,
    # seconds 0 + floor(0.9861 d in s), fraction of that (psrfits.py:224-243)
    inc = 55999.9861 - 56000.0
    left = (inc - np.floor(inc)) * 86400.0
    assert ph["STT_IMJD"] == 55999 and ph["STT_SMJD"] == int(np.floor(left))
    assert abs(ph["STT_OFFS"] - (left - np.floor(left))) < 1e-9
    assert ph["OBSFREQ"] == 430.0 and ph["OBSBW"] == 100.0 and ph["CHAN_DM"] == 10.0 and ph["BE_DELAY"] == 0.0
    # HISTORY: header verbatim, rows 1.. verbatim, row 0 edited fields only
    from psrsigsim_amd.io.psrfits import _table_dtype
    assert O["HISTORY"]["cards"] == T["HISTORY"]["cards"]
    dt = _table_dtype(T["HISTORY"]["hdr"])
    ro, rt = (np.frombuffer(h["data"], dtype=dt) for h in (O["HISTORY"], T["HISTORY"]))
    assert ro[1:].tobytes() == rt[1:].tobytes()
    want = {"POL_TYPE": b"AA+BB", "NSUB": 3, "NPOL": 1, "NBIN": 128, "NBIN_PRD": 128, "TBIN": 1.0 / 128,
            "CTR_FREQ": 430.0, "NCHAN": 8, "CHAN_BW": 12.5, "DM": 10.0}
    for f in dt.names:
        assert (ro[0][f] == want[f]) if f in want else (ro[0][f].tobytes() == rt[0][f].tobytes()), f
    # PSRPARAM: the template's lines minus the reference's hard-coded deletions
    pt = np.frombuffer(T["PSRPARAM"]["data"], dtype=_table_dtype(T["PSRPARAM"]["hdr"]))
    po = np.frombuffer(O["PSRPARAM"]["data"], dtype=_table_dtype(O["PSRPARAM"]["hdr"]))
    keep = [r.tobytes() for r in pt if bytes(r[0]).split()[0].decode() not in _DELETED]
    assert [r.tobytes() for r in po] == keep and 0 < len(keep) < len(pt)
    # SUBINT: the template's column set resized to the signal, the reference's edits
    prim, sub, rec = read_psrfits(path)
    for k, v in (("NBIN", 128), ("NCHAN", 8), ("NPOL", 1), ("POL_TYPE", "AA+BB"), ("TBIN", 1.0 / 128),
                 ("CHAN_BW", 12.5), ("DM", 10.0), ("EPOCHS", "MIDTIME"), ("NSBLK", 1)):
        assert sub[k] == v, k
    cs, ts = _cards(O["SUBINT"]), _cards(T["SUBINT"])
    edited = {"NAXIS1", "NAXIS2", "NBIN", "NCHAN", "NPOL", "NSBLK", "POL_TYPE", "TBIN", "CHAN_BW", "DM", "EPOCHS",
              "TFORM16", "TFORM17", "TFORM18", "TFORM19", "TFORM20", "TDIM20"}
    assert all(cs[k] == ts[k] for k in ts if k not in edited)
    assert rec.shape == (3,)
    np.testing.assert_array_equal(rec["OFFS_SUB"], [1.0, 3.0, 5.0])
    np.testing.assert_array_equal(rec["TSUBINT"], 2.0)
    np.testing.assert_array_equal(rec["DAT_FREQ"][0], np.asarray(sig.dat_freq.value))
    assert (rec["DAT_WTS"] == 1).all() and (rec["DAT_SCL"] == 1).all() and (rec["DAT_OFFS"] == 0).all()
    d16 = sig.data[:, :3 * 128].astype(">i2")
    assert list(d16[0, :5]) == [-25536, 25536, 0, 4464, 0]       # numpy's wrap of the out-of-range values
    for i in range(3):
        np.testing.assert_array_equal(rec["DATA"][i, 0], d16[:, i * 128:(i + 1) * 128])
    assert (tmp_path / "J0000+0000_sim.par").exists()            # make_par (no parfile given)


def test_template_copy_pint_required(tmp_path, monkeypatch):
    """usePint=False raises as the reference's _gen_polyco does."""
    with pytest.raises(NotImplementedError):
        _template_copy(tmp_path, monkeypatch, _FakeSig(2, 1, 64, np.random.default_rng(0)), usePint=False)


def test_signal_from_template():
    """make_signal_from_psrfits (psrfits.py:439-483): the template's geometry,
    sample rate F0 x NBIN from PSRPARAM."""
    from psrsigsim_amd.io.psrfits import read_fits
    S = PSRFITS(path="x.fits", template=TEMPLATE, fits_mode="copy", obs_mode="PSR").make_signal_from_psrfits()
    h = read_fits(TEMPLATE)
    f0 = [float(bytes(x).split()[1].replace(b"D", b"E")) for x in h["PSRPARAM"][1]["PARAM"]
          if bytes(x).split()[0] == b"F0"][0]
    assert S.Nchan == 1 and S.fold and abs(S.samprate.value - f0 * 2048 * 1e-6) < 1e-15
    assert S.dm.value == 13.299393 and S.fcent.value == h["PRIMARY"][0]["OBSFREQ"]


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


@pytest.mark.gpu
def test_save_simulation_psrfits_template(tmp_path, monkeypatch, hip_lib):
    """simulate() on the GPU -> save_simulation('psrfits') with the
    reference's template (simulate.py:354-370): DATA is the reference's
    astype('>i2') of the device data, values beyond int16 included (a tiny
    Smean makes the radiometer noise huge), and the default par file is made."""
    import psrsigsim_amd as pss
    from psrsigsim_amd.simulate import Simulation
    monkeypatch.chdir(tmp_path)
    pss.seed(5)
    sim = Simulation(fcent=430, bandwidth=100, sample_rate=1.0 * 2048 * 10 ** -6, Nchan=16, sublen=2.0, fold=True,
                     period=1.0, Smean=1e-5, profiles=[0.5, 0.05, 1.0], tobs=6.0, name="J0000+0000", dm=10.0,
                     tscope_name="Arecibo", system_name="Lband_PUPPI", tempfile=TEMPLATE)
    sim.simulate()
    path = str(tmp_path / "sim.fits")
    sim.save_simulation(outfile=path)
    prim, sub, rec = read_psrfits(path)
    d = sim.signal.data.cpu().numpy().astype(np.float64)
    nsub = int(sim.signal.nsub)
    nbin = int(sim.signal.nsamp / nsub)
    assert sub["NBIN"] == nbin and sub["NCHAN"] == 16 and rec.shape == (nsub,)
    assert (np.abs(d[:, :nbin * nsub]) > 32767).any()
    exp = d[:, :nbin * nsub].astype(">i2")
    for i in range(nsub):
        np.testing.assert_array_equal(rec["DATA"][i, 0], exp[:, i * nbin:(i + 1) * nbin])
    assert prim["STT_IMJD"] == 55999 and (tmp_path / "simpar.par").exists()
