"""Fold-mode PSRFITS output (reference: psrsigsim/io/psrfits.py:22-738).

Template mode (the reference's: ``PSRFITS(path, template=..., fits_mode=
'copy')``, what ``Simulation.save_simulation('psrfits')`` calls): the
template's HDUs are copied in order and edited exactly where the reference
edits them (psrfits.py:184-303, 305-424, 485-509):

* PRIMARY: OBSFREQ, OBSBW, CHAN_DM, STT_IMJD / STT_SMJD / STT_OFFS (the
  reference's _gen_metadata arithmetic, float-repr string splits included)
  and BE_DELAY; every other card image verbatim;
* HISTORY row 0: POL_TYPE, NSUB, NPOL, NBIN, NBIN_PRD, TBIN, CTR_FREQ, NCHAN,
  CHAN_BW, DM; the other rows and the header verbatim;
* PSRPARAM: the reference's hard-coded deletions (BINARY, A1, E, ... TZRSITE);
* POLYCO: verbatim -- the reference regenerates it with PINT, which is absent
  from this environment (a warning says so; files are not phase-connected);
* SUBINT: nsub new rows with the template's columns resized to the signal
  (DAT_FREQ / DAT_WTS [nchan], DAT_OFFS / DAT_SCL [nchan npol], DATA
  (NBIN, NCHAN, NPOL) int16 = the reference's ``astype('>i2')`` of the data,
  wrapped exactly as numpy wraps out-of-range values), OFFS_SUB / TSUBINT per
  row, and the header edits EPOCHS, CHAN_BW, POL_TYPE, TBIN, DM, NBIN.

The reference drives pdat/fitsio for this (absent here); this module restates
their effect on the file (parity of the file bytes is therefore unpinned:
tests/test_psrfits.py checks the copied bytes against the template and the
edited values against the reference's formulas).

Without a template a self-written layout of the same SUBINT columns is
written (an extension).  ``read_fits`` parses any FITS file of binary tables
(the reference's template included, for config C4's portrait:
:func:`template_profile`); ``read_psrfits`` returns the primary and SUBINT
parts of it.  The device data is read back once (one D2H copy of the folded
product; in a multi-GPU run gather it first with
``psrsigsim_amd.shard.gather_channels``).
"""
import logging
import math

import numpy as np

from .._units import Quantity

__all__ = ["PSRFITS", "read_psrfits", "read_fits", "template_profile"]

log = logging.getLogger("psrsigsim_amd")

# SUBINT columns of the reference's template, in its order (the pointing /
# angle columns carry zeros here: no telescope geometry is simulated)
_SUBINT_SCALARS = [("INDEXVAL", "D"), ("TSUBINT", "D"), ("OFFS_SUB", "D"), ("LST_SUB", "D"), ("RA_SUB", "D"),
                   ("DEC_SUB", "D"), ("GLON_SUB", "D"), ("GLAT_SUB", "D"), ("FD_ANG", "E"), ("POS_ANG", "E"),
                   ("PAR_ANG", "E"), ("TEL_AZ", "E"), ("TEL_ZEN", "E"), ("AUX_DM", "D"), ("AUX_RM", "D")]
_NP = {"D": ">f8", "E": ">f4", "I": ">i2", "J": ">i4", "K": ">i8", "B": "u1", "L": "u1", "A": "S1"}

_BLOCK = 2880


def _val(q):
    return q.value if isinstance(q, Quantity) else q


def _card(key, value=None, comment=""):
    if value is None:
        s = key.ljust(80)
    else:
        if isinstance(value, bool):
            v = ("T" if value else "F").rjust(20)
        elif isinstance(value, (int, np.integer)):
            v = str(int(value)).rjust(20)
        elif isinstance(value, (float, np.floating)):
            v = repr(float(value)).upper().rjust(20)       # shortest round-trip, FITS 'E' exponent
        else:
            v = ("'%s'" % str(value).replace("'", "''").ljust(8)).ljust(20)
        s = ("%-8s= %s" % (key, v))
        if comment:
            s += " / " + comment
    if len(s) > 80:
        raise ValueError("FITS card too long: %r" % s)
    return s.ljust(80)


def _header(cards):
    text = "".join(cards) + "END".ljust(80)
    pad = (-len(text)) % _BLOCK
    return (text + " " * pad).encode("ascii")


def _pad(b):
    return b + b"\0" * ((-len(b)) % _BLOCK)


# PSRPARAM lines the reference's _edit_psrfits_header drops (psrfits.py:296-302)
_DELETE_PARAMS = ("BINARY", "A1", "E", "T0", "PB", "OM", "SINI", "M2", "F1", "PMDEC", "PMRA", "TZRMJD",
                  "TZRFRQ", "TZRSITE")


def _card_comment(card):
    """The comment of an 80-char header card (after the '/' that follows the
    value; quotes respected), or ''."""
    v = card[10:]
    q = False
    for k, ch in enumerate(v):
        if ch == "'":
            q = not q
        elif ch == "/" and not q:
            return v[k + 1:].strip()
    return ""


def _set_cards(cards, values):
    """Header card images with ``values`` {key: value} replaced in place
    (keeping each card's comment) or appended when absent; every other card
    image is kept verbatim."""
    out = list(cards)
    for key, val in values.items():
        for n, c in enumerate(out):
            if c[:8].rstrip() == key and c[8:10] == "= ":
                cm = _card_comment(c)
                try:
                    out[n] = _card(key, val, cm)
                except ValueError:                         # value + old comment too long
                    out[n] = _card(key, val)
                break
        else:
            out.append(_card(key, val))
    return out


def _raw_hdus(path):
    """[{name, cards (80-char images, END excluded), hdr (parsed), data
    (bytes, unpadded)}] of a FITS file, in file order."""
    with open(path, "rb") as f:
        buf = f.read()
    out = []
    pos = 0
    while pos < len(buf):
        hdr, end = _parse_header(buf, pos)
        text = buf[pos:end].decode("ascii", errors="replace")
        cards = []
        for k in range(0, len(text), 80):
            c = text[k:k + 80]
            if c[:8].rstrip() == "END":
                break
            cards.append(c)
        if "SIMPLE" in hdr:
            name, size = "PRIMARY", 0
            if int(hdr.get("NAXIS", 0)) > 0:
                size = abs(int(hdr["BITPIX"])) // 8
                for a in range(1, int(hdr["NAXIS"]) + 1):
                    size *= int(hdr["NAXIS%d" % a])
        else:
            name = str(hdr.get("EXTNAME", "HDU%d" % len(out))).strip()
            size = int(hdr["NAXIS1"]) * int(hdr["NAXIS2"]) + int(hdr.get("PCOUNT", 0))
        out.append({"name": name, "cards": cards, "hdr": hdr, "data": buf[end:end + size]})
        pos = end + -(-size // _BLOCK) * _BLOCK
    return out


def _mjd_fields(ref_MJD, inc_len):
    """STT_IMJD / STT_SMJD / STT_OFFS exactly as the reference's
    _gen_metadata derives them (psrfits.py:206-243), string splitting of the
    float reprs included (make_quant turns ref_MJD into a float64 first)."""
    init_mjd = float(ref_MJD)
    init_frac_s = float("0." + str(init_mjd).split(".")[-1]) * 86400.0       # ('0.' + frac) day -> s
    init_smjd = float(str(init_frac_s).split(".")[0])
    init_offs = float("0." + str(init_frac_s).split(".")[-1])
    inc_len = float(inc_len)
    if inc_len == 0.0:
        next_mjd, next_s, next_frac = init_mjd, init_smjd, init_offs
    else:
        next_mjd = init_mjd + math.floor(inc_len)
        leftover_s = (inc_len - math.floor(inc_len)) * 86400.0
        next_s = init_smjd + math.floor(leftover_s)
        next_frac = init_offs + (leftover_s - math.floor(leftover_s))
    return int(next_mjd), int(next_s), float(next_frac)


def _wrap_i2(x):
    """numpy's ``astype('>i2')`` of the float64 data, the reference's cast
    (psrfits.py:353): truncation toward zero, out-of-range values wrapped as
    numpy does on this host (the values themselves, not a saturating cast)."""
    return np.asarray(x, dtype=np.float64).astype(">i2")


class PSRFITS(object):
    """psrfits.py:22-738: ``PSRFITS(path, obs_mode=None, template=None,
    copy_template=False, fits_mode='copy')``, ``get_signal_params``,
    ``save(signal, pulsar, parfile, MJD_start, segLength, inc_len, ref_MJD,
    usePint, eq_wts)``, ``make_signal_from_psrfits``.

    With a ``template`` (the reference's only mode) the file is the template
    copied HDU by HDU with the reference's edits (psrfits.py:184-303,
    305-424, 485-509): PRIMARY cards from _gen_metadata, HISTORY row 0, the
    PSRPARAM deletions, and a new SUBINT table of ``nsub`` rows.  Every card
    image and table byte the reference does not edit is the template's,
    verbatim.  The reference's pdat/fitsio layer is restated here (absent
    from this environment); the POLYCO table stays the template's because
    the reference regenerates it with PINT, which is absent too (a warning
    says so).  Without a template the self-written layout below is used
    (an extension; see the module docstring)."""

    def __init__(self, path=None, obs_mode=None, template=None, copy_template=False, fits_mode="copy"):
        self._path = path
        self._template = template
        self._fits_mode = fits_mode
        self._hdus = _raw_hdus(template) if template is not None else None
        if obs_mode is None:
            obs_mode = str(self._hdus[0]["hdr"].get("OBS_MODE", "PSR")).strip() if self._hdus else "PSR"
        if obs_mode not in ("PSR", "CAL"):
            raise NotImplementedError("only fold-mode (PSR) output is written")
        self.obs_mode = obs_mode
        self.nchan = self.nbin = self.npol = self.nrows = self.nsblk = self.nsubint = None
        self.tbin = self.obsfreq = self.obsbw = self.chan_bw = self.tsubint = None

    path = property(lambda self: self._path)

    # -- template access --------------------------------------------------
    def _hdu(self, name):
        for h in self._hdus:
            if h["name"] == name:
                return h
        raise KeyError(name)

    def _records(self, name):
        h = self._hdu(name)
        return np.frombuffer(h["data"], dtype=_table_dtype(h["hdr"]), count=int(h["hdr"]["NAXIS2"]))

    def _psrparam(self, key):
        """psrfits.py:633-640: the value of a PSRPARAM line, or None."""
        for row in self._records("PSRPARAM"):
            tok = bytes(row[0]).split()
            if tok and tok[0].decode() == key:
                return np.float64(tok[1].decode().replace("D", "E"))
        return None

    def get_signal_params(self, signal=None):
        """psrfits.py:533-581."""
        sub = self._hdu("SUBINT")["hdr"] if self._hdus else {}
        if signal is None:
            if not self._hdus:
                raise ValueError("no template to read the parameters from")
            prim = self._hdu("PRIMARY")["hdr"]
            self.nchan, self.tbin, self.nbin = int(sub["NCHAN"]), float(sub["TBIN"]), int(sub["NBIN"])
            self.npol, self.nrows, self.nsblk = int(sub["NPOL"]), int(sub["NAXIS2"]), int(sub["NSBLK"])
            self.obsfreq, self.obsbw, self.chan_bw = float(prim["OBSFREQ"]), float(prim["OBSBW"]), float(sub["CHAN_BW"])
            self.tsubint = float(self._records("SUBINT")["TSUBINT"][0])
        else:
            self.nchan = int(signal.Nchan)
            self.tbin = 1.0 / (float(_val(signal.samprate)) * 1e6)
            self.nbin = int(signal.nsamp / signal.nsub)
            self.npol = int(signal.Npols)
            self.nrows = int(signal.nsub)
            self.nsblk = int(sub.get("NSBLK", 1))
            self.obsfreq, self.obsbw = float(_val(signal.fcent)), float(_val(signal.bw))
            self.chan_bw = float(_val(signal.bw)) / signal.Nchan
            self.tsubint = float(_val(signal.sublen)) if signal.sublen is not None else float(_val(signal.tobs))
        self.nsubint = self.nrows if self.obs_mode == "PSR" else None

    def make_signal_from_psrfits(self):
        """psrfits.py:439-483: a fold-mode FilterBankSignal with the
        template's geometry (sample rate = F0 x NBIN from PSRPARAM)."""
        from ..signal import FilterBankSignal
        self.get_signal_params()
        f, f0 = self._psrparam("F"), self._psrparam("F0")
        if f0 is not None:
            s_rate = f0 * self.nbin * 1e-6
        elif f is not None:
            s_rate = f * self.nbin * 1e-6
        else:
            raise ValueError("No pulsar frequency defined in input fits file.")
        S = FilterBankSignal(fcent=self.obsfreq, bandwidth=self.obsbw, Nsubband=self.nchan, sample_rate=s_rate,
                             dtype=np.float32, fold=True, sublen=self.tsubint)
        S._dat_freq = Quantity(np.atleast_1d(np.asarray(self._records("SUBINT")["DAT_FREQ"][0], dtype=np.float64)),
                               "MHz")
        S._dm = Quantity(self._psrparam("DM"), "pc/cm^3")
        return S

    # -- save ---------------------------------------------------------------
    def save(self, signal, pulsar, parfile=None, MJD_start=56000.0, segLength=60.0, inc_len=0.0,
             ref_MJD=56000.0, usePint=True, eq_wts=True, telescope="GBT"):
        """psrfits.py:305-424 (template) or the self-written layout."""
        if self.path is None:
            raise ValueError("no output path")
        if self._hdus is None:
            return self._save_new(signal, pulsar, MJD_start, inc_len, ref_MJD, eq_wts, telescope)
        if inc_len == 0.0:
            inc_len = MJD_start - ref_MJD
        if self.nbin is None:
            self.get_signal_params(signal)
        if self.obs_mode != "SEARCH":
            self.nsblk = 1
        nsub, nbin, nchan, npol = int(self.nsubint), int(self.nbin), int(self.nchan), int(self.npol)
        stop = nbin * nsub
        data = signal.data
        if hasattr(data, "cpu"):
            data = data[:, :stop].cpu().numpy()
        sim_sig = _wrap_i2(np.asarray(data)[:, :stop])
        if sim_sig.shape[1] < stop:
            raise ValueError("signal holds %d samples per channel, %d subints x %d bins need %d"
                             % (sim_sig.shape[1], nsub, nbin, stop))
        if parfile is None:
            from ..utils import make_par
            print("No parfile provided, creating par file %s_sim.par" % (pulsar.name))
            make_par(signal, pulsar, outpar="%s_sim.par" % (pulsar.name))
            parfile = "%s_sim.par" % (pulsar.name)
        if not usePint:
            raise NotImplementedError("Only PINT is currently supported for generating polycos")
        log.warning("PINT is not available: the template's POLYCO table is kept (polycos for %s not regenerated)",
                    parfile)
        dm = float(_val(signal.dm))
        tbin = float(_val(pulsar.period)) / nbin
        imjd, smjd, offs = _mjd_fields(ref_MJD, inc_len)
        primary = {"OBSFREQ": float(self.obsfreq), "OBSBW": float(self.obsbw), "CHAN_DM": dm, "STT_IMJD": imjd,
                   "STT_SMJD": smjd, "STT_OFFS": offs, "BE_DELAY": 0.0}
        sub_cards = {"EPOCHS": "MIDTIME", "CHAN_BW": float(self.chan_bw), "POL_TYPE": "AA+BB", "TBIN": tbin,
                     "DM": dm, "NBIN": nbin}
        offs_sub = np.array([float(_val(signal.sublen)) / 2.0 + ii * float(_val(signal.sublen))
                             for ii in range(int(signal.nsub))], dtype=np.float64)
        out = []
        for h in self._hdus:
            name = h["name"]
            if name == "PRIMARY":
                out.append((_set_cards(h["cards"], primary), h["data"]))
            elif name == "HISTORY":
                rec = self._records("HISTORY").copy()
                for key, val in (("POL_TYPE", b"AA+BB"), ("NSUB", nsub), ("NPOL", npol), ("NBIN", nbin),
                                 ("NBIN_PRD", nbin), ("TBIN", tbin), ("CTR_FREQ", float(self.obsfreq)),
                                 ("NCHAN", nchan), ("CHAN_BW", float(self.chan_bw)), ("DM", dm)):
                    if key in rec.dtype.names:
                        rec[0][key] = val
                out.append((h["cards"], rec.tobytes()))
            elif name == "PSRPARAM":
                rec = self._records("PSRPARAM")
                keep = [r for r in rec if not (bytes(r[0]).split() and
                                               bytes(r[0]).split()[0].decode() in _DELETE_PARAMS)]
                kept = np.array(keep, dtype=rec.dtype) if keep else np.zeros(0, dtype=rec.dtype)
                out.append((_set_cards(h["cards"], {"NAXIS2": len(kept)}), kept.tobytes()))
            elif name == "SUBINT":
                out.append(self._subint(h, sim_sig, offs_sub, sub_cards, eq_wts, signal))
            else:
                out.append((h["cards"], h["data"]))      # POLYCO and any other table: verbatim
        with open(self.path, "wb") as f:
            for cards, data in out:
                f.write(_header(cards))
                if data:
                    f.write(_pad(bytes(data)))
        print("Finished writing and saving the file")

    def _subint(self, h, sim_sig, offs_sub, sub_cards, eq_wts, signal):
        """The new SUBINT table (pdat set_subint_dims + make_HDU_rec_array:
        the template's columns with DAT_FREQ / DAT_WTS [nchan], DAT_OFFS /
        DAT_SCL [nchan npol], DATA [nbin nchan npol] of nsub zero rows), then
        the reference's per-row assignments (psrfits.py:365-392, 284-287)."""
        hdr = h["hdr"]
        nsub, nbin, nchan, npol = int(self.nsubint), int(self.nbin), int(self.nchan), int(self.npol)
        sizes = {"DAT_FREQ": nchan, "DAT_WTS": nchan, "DAT_OFFS": nchan * npol, "DAT_SCL": nchan * npol,
                 "DATA": nbin * nchan * npol * int(self.nsblk)}
        cards = {}
        fields = []
        for i in range(1, int(hdr["TFIELDS"]) + 1):
            name = str(hdr["TTYPE%d" % i]).strip()
            form = str(hdr["TFORM%d" % i]).strip()
            k = 0
            while k < len(form) and form[k].isdigit():
                k += 1
            code = form[k]
            if name in sizes:
                n = sizes[name]
                cards["TFORM%d" % i] = "%d%s" % (n, code)
                if name == "DATA":
                    cards["TDIM%d" % i] = "(%d,%d,%d)" % (nbin, nchan, npol)
                    fields.append((name, _NP[code], (npol, nchan, nbin)))
                else:
                    fields.append((name, _NP[code], (n,)))
            else:
                n = int(form[:k] or 1)
                fields.append((name, "S%d" % n) if code == "A" else (name, _NP[code], (n,) if n > 1 else ()))
        dt = np.dtype(fields)
        tab = np.zeros(nsub, dtype=dt)
        tmpl = self._records("SUBINT")
        freqs = np.asarray(_val(signal.dat_freq), dtype=np.float64)
        for ii in range(nsub):
            tab[ii]["DATA"] = sim_sig[:, ii * nbin:(ii + 1) * nbin]
            tab[ii]["DAT_FREQ"] = freqs
            qq = min(ii, len(tmpl) - 1)       # more subints than the template: its last row's values
            if eq_wts:
                tab[ii]["DAT_SCL"] = 1.0
                tab[ii]["DAT_OFFS"] = 0.0
                tab[ii]["DAT_WTS"] = 1.0
            else:
                for key in ("DAT_SCL", "DAT_OFFS", "DAT_WTS"):
                    tab[ii][key] = np.resize(np.asarray(tmpl[qq][key]).ravel(), tab[ii][key].shape)
        tab["OFFS_SUB"][:len(offs_sub)] = offs_sub[:nsub]
        tab["TSUBINT"] = float(self.tsubint)
        cards.update({"NAXIS1": dt.itemsize, "NAXIS2": nsub, "NCHAN": nchan, "NPOL": npol, "NSBLK": int(self.nsblk)})
        cards.update(sub_cards)
        return _set_cards(h["cards"], cards), tab.tobytes()

    def _save_new(self, signal, pulsar, MJD_start, inc_len, ref_MJD, eq_wts, telescope):
        """The self-written layout (no template; extension)."""
        nchan = int(signal.Nchan)
        npol = 1
        period = float(_val(pulsar.period))
        nbin = int(_val(signal.samprate) * 1e6 * period)          # samples per period, as make_pulses
        nsub = int(signal.nsub)
        sublen = float(_val(signal.sublen)) if signal.sublen is not None else float(_val(signal.tobs))
        data = signal.data
        stop = nbin * nsub
        if hasattr(data, "cpu"):
            data = data[:, :stop].cpu().numpy()
        d16 = _wrap_i2(np.asarray(data)[:, :stop])
        if d16.shape[1] < stop:
            raise ValueError("signal holds %d samples per channel, %d subints x %d bins need %d"
                             % (d16.shape[1], nsub, nbin, stop))
        # [nsub][npol][nchan][nbin] (psrfits.py:357-366)
        out = d16.reshape(nchan, nsub, nbin).transpose(1, 0, 2)[:, None, :, :]
        freqs = np.asarray(_val(signal.dat_freq), dtype=np.float64)[:nchan]
        dm = float(_val(signal.dm)) if getattr(signal, "dm", None) is not None else 0.0
        if inc_len == 0.0:
            inc_len = MJD_start - ref_MJD
        # STT_* (psrfits.py:220-244): integer MJD, integer seconds, fraction
        start = ref_MJD + (math.floor(inc_len) if inc_len else 0.0)
        imjd = int(math.floor(start))
        secs = (start - imjd) * 86400.0 + ((inc_len - math.floor(inc_len)) * 86400.0 if inc_len else 0.0)
        smjd = int(math.floor(secs))
        offs = secs - smjd
        primary = [
            _card("SIMPLE", True, "file conforms to FITS standard"), _card("BITPIX", 8), _card("NAXIS", 0),
            _card("EXTEND", True), _card("HDRVER", "6.1"), _card("FITSTYPE", "PSRFITS"),
            _card("OBS_MODE", self.obs_mode), _card("TELESCOP", telescope), _card("FRONTEND", "sim"),
            _card("BACKEND", "psrsigsim_amd"), _card("FD_POLN", "LIN"), _card("SRC_NAME", str(pulsar.name)),
            _card("OBSFREQ", float(_val(signal.fcent))), _card("OBSBW", float(_val(signal.bw))),
            _card("OBSNCHAN", nchan), _card("CHAN_DM", dm), _card("STT_IMJD", imjd), _card("STT_SMJD", smjd),
            _card("STT_OFFS", offs), _card("BE_DELAY", 0.0),
        ]
        cols = [(n, "1" + c, None) for n, c in _SUBINT_SCALARS]
        cols += [("DAT_FREQ", "%dD" % nchan, None), ("DAT_WTS", "%dE" % nchan, None),
                 ("DAT_OFFS", "%dE" % (nchan * npol), None), ("DAT_SCL", "%dE" % (nchan * npol), None),
                 ("DATA", "%dI" % (nbin * nchan * npol), "(%d,%d,%d)" % (nbin, nchan, npol))]
        row = np.dtype([(n, _NP[c]) for n, c in _SUBINT_SCALARS] +
                       [("DAT_FREQ", ">f8", (nchan,)), ("DAT_WTS", ">f4", (nchan,)),
                        ("DAT_OFFS", ">f4", (nchan * npol,)), ("DAT_SCL", ">f4", (nchan * npol,)),
                        ("DATA", ">i2", (npol, nchan, nbin))])
        tab = np.zeros(nsub, dtype=row)
        tab["INDEXVAL"] = np.arange(nsub)
        tab["TSUBINT"] = sublen
        tab["OFFS_SUB"] = sublen / 2.0 + np.arange(nsub) * sublen
        tab["DAT_FREQ"] = freqs
        tab["DAT_WTS"] = 1.0
        tab["DAT_OFFS"] = 0.0
        tab["DAT_SCL"] = 1.0
        tab["DATA"] = out
        if not eq_wts:
            raise NotImplementedError("template weights need the template file")
        sub = [_card("XTENSION", "BINTABLE"), _card("BITPIX", 8), _card("NAXIS", 2),
               _card("NAXIS1", row.itemsize), _card("NAXIS2", nsub), _card("PCOUNT", 0), _card("GCOUNT", 1),
               _card("TFIELDS", len(cols))]
        for i, (name, form, dim) in enumerate(cols, 1):
            sub.append(_card("TTYPE%d" % i, name))
            sub.append(_card("TFORM%d" % i, form))
            if dim:
                sub.append(_card("TDIM%d" % i, dim))
        sub += [_card("EXTNAME", "SUBINT"), _card("EPOCHS", "MIDTIME"), _card("INT_TYPE", "TIME"),
                _card("INT_UNIT", "SEC"), _card("NPOL", npol), _card("POL_TYPE", "AA+BB"),
                _card("TBIN", period / nbin), _card("NBIN", nbin), _card("NCHAN", nchan),
                _card("CHAN_BW", float(_val(signal.bw)) / nchan), _card("DM", dm), _card("NSBLK", 1),
                _card("NBITS", 16)]
        with open(self.path, "wb") as f:
            f.write(_header(primary))
            f.write(_header(sub))
            f.write(_pad(tab.tobytes()))


def _parse_header(buf, pos):
    """(cards dict, position after the header) of the header at ``pos``."""
    cards = {}
    while True:
        block = buf[pos:pos + _BLOCK].decode("ascii", errors="replace")
        if len(block) < _BLOCK:
            raise ValueError("truncated FITS header")
        pos += _BLOCK
        for i in range(0, _BLOCK, 80):
            c = block[i:i + 80]
            key = c[:8].strip()
            if key == "END":
                return cards, pos
            if c[8:10] == "= ":
                v = c[10:]
                if v.lstrip().startswith("'"):
                    v = v.lstrip()
                    j = 1
                    out = []
                    while j < len(v):            # quoted string, '' escapes a quote
                        if v[j] == "'":
                            if j + 1 < len(v) and v[j + 1] == "'":
                                out.append("'")
                                j += 2
                                continue
                            break
                        out.append(v[j])
                        j += 1
                    v = "".join(out).rstrip()
                else:
                    v = v.split("/")[0].strip()
                    if v in ("T", "F"):
                        v = v == "T"
                    elif v == "":
                        v = None
                    else:
                        try:
                            v = int(v)
                        except ValueError:
                            v = float(v.replace("D", "E"))
                cards[key] = v


def _table_dtype(hdr):
    """numpy dtype of a BINTABLE row (TFORM rTa codes D E I J K B L A; TDIM
    reshapes, fastest axis first as FITS writes them)."""
    fields = []
    for i in range(1, int(hdr["TFIELDS"]) + 1):
        form = str(hdr["TFORM%d" % i]).strip()
        k = 0
        while k < len(form) and form[k].isdigit():
            k += 1
        n, code = int(form[:k] or 1), form[k]
        if code not in _NP:
            raise NotImplementedError("FITS column format %r" % form)
        shape = (n,) if n > 1 else ()
        dim = hdr.get("TDIM%d" % i)
        if dim and n > 1:
            shape = tuple(int(x) for x in str(dim).strip("() ").split(","))[::-1]
        if code == "A":
            fields.append((hdr["TTYPE%d" % i], "S%d" % n))
        else:
            fields.append((hdr["TTYPE%d" % i], _NP[code], shape))
    dt = np.dtype(fields)
    if dt.itemsize != int(hdr["NAXIS1"]):
        raise ValueError("row layout %d B != NAXIS1 %d" % (dt.itemsize, hdr["NAXIS1"]))
    return dt


def read_fits(path):
    """All HDUs of a FITS file of binary tables (PSRFITS):
    ``{"PRIMARY": (header, None), EXTNAME: (header, records or None)}``."""
    with open(path, "rb") as f:
        buf = f.read()
    out = {}
    pos = 0
    while pos < len(buf):
        hdr, pos = _parse_header(buf, pos)
        if "SIMPLE" in hdr:
            name, size = "PRIMARY", 0
            if int(hdr.get("NAXIS", 0)) > 0:
                size = abs(int(hdr["BITPIX"])) // 8
                for a in range(1, int(hdr["NAXIS"]) + 1):
                    size *= int(hdr["NAXIS%d" % a])
            out[name] = (hdr, None)
        else:
            name = str(hdr.get("EXTNAME", "HDU%d" % len(out))).strip()
            size = int(hdr["NAXIS1"]) * int(hdr["NAXIS2"]) + int(hdr.get("PCOUNT", 0))
            rec = None
            if hdr.get("XTENSION") == "BINTABLE":
                try:
                    rec = np.frombuffer(buf, dtype=_table_dtype(hdr), count=int(hdr["NAXIS2"]), offset=pos)
                except NotImplementedError:
                    rec = None
            out[name] = (hdr, rec)
        pos += -(-size // _BLOCK) * _BLOCK
    return out


def read_psrfits(path):
    """(primary header dict, SUBINT header dict, SUBINT records) of a PSRFITS
    file: one written by :meth:`PSRFITS.save`, or the reference's template."""
    hdus = read_fits(path)
    sub, rec = hdus["SUBINT"]
    return hdus["PRIMARY"][0], sub, rec


def template_profile(path, subint=0, chan=0, pol=0, baseline="median"):
    """Pulse profile of a fold-mode PSRFITS template: DATA * DAT_SCL +
    DAT_OFFS of one (subint, channel, polarisation) -- the PSRFITS scaling
    (template SUBINT: 'Data scale factor (outval=dataval*scl + offs)') -- as
    float64 (NBIN,), with the baseline (the median bin; None: none) removed.
    Config C4's portrait is this profile of the reference's B1855+09 template
    (DataProfile of it, tiled over the channels)."""
    _, sub, rec = read_psrfits(path)
    npol = int(sub.get("NPOL", 1))
    nchan = int(sub.get("NCHAN", 1))
    r = rec[subint]
    data = np.asarray(r["DATA"], dtype=np.float64).reshape(npol, nchan, -1)[pol, chan]
    scl = np.asarray(r["DAT_SCL"], dtype=np.float64).reshape(-1)[pol * nchan + chan]
    offs = np.asarray(r["DAT_OFFS"], dtype=np.float64).reshape(-1)[pol * nchan + chan]
    prof = data * scl + offs
    if baseline == "median":
        prof = prof - np.median(prof)
    return prof
