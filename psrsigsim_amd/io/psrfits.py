"""Fold-mode PSRFITS output (reference: psrsigsim/io/psrfits.py:305-424).

The reference writes PSRFITS by copying a template file's HDUs through
pdat/fitsio and rebuilds the POLYCO table with PINT; none of those are
available here, so this is a self-written FITS writer
producing the same data layout without a template:

* primary HDU: PSRFITS header cards the reference edits (OBSFREQ, OBSBW,
  OBSNCHAN, CHAN_DM, STT_IMJD/SMJD/OFFS from ``ref_MJD``, BE_DELAY, SRC_NAME,
  OBS_MODE = 'PSR', ...);
* SUBINT binary table, one row per subintegration: TSUBINT, OFFS_SUB
  (sublen/2 + i sublen, psrfits.py:213-217), DAT_FREQ, DAT_WTS = 1,
  DAT_OFFS = 0, DAT_SCL = 1 (``eq_wts``, psrfits.py:372-387) and DATA
  ``(NBIN, NCHAN, NPOL)`` int16 = ``signal.data[:, i nbin:(i+1) nbin]``
  truncated to '>i2' (psrfits.py:355-366); header NBIN, NCHAN, NPOL = 1,
  TBIN = P / nbin, CHAN_BW, DM, POL_TYPE = 'AA+BB', EPOCHS = 'MIDTIME'.

The SUBINT column set, order, TFORM codes and TDIM follow the reference's
template (``data/B1855+09.L-wide.PUPPI.11y.x.sum.sm``, whose SUBINT table the
reference copies, psrfits.py:487-509): the pointing/angle columns the
reference leaves at their draft value are written as zeros.

No POLYCO / PSRPARAM tables (PINT is absent): files are not phase-connected.
``read_fits`` parses any FITS file of binary tables (the reference's
template included, for config C4's portrait: :func:`template_profile`);
``read_psrfits`` returns the primary and SUBINT parts of it.
The device data is read back once (one D2H copy of the folded product; in a
multi-GPU run gather it first with ``psrsigsim_amd.shard.gather_channels``).
"""
import math

import numpy as np

from .._units import Quantity

__all__ = ["PSRFITS", "read_psrfits", "read_fits", "template_profile"]

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


class PSRFITS(object):
    """psrfits.py:22-424 subset: ``PSRFITS(path, obs_mode='PSR')``,
    ``save(signal, pulsar, ref_MJD=56000.0, inc_len=0.0, eq_wts=True)``."""

    def __init__(self, path=None, obs_mode="PSR", template=None, copy_template=False, fits_mode="new"):
        if template is not None or fits_mode == "copy":
            raise NotImplementedError("template-copy PSRFITS (pdat/fitsio) is not available; "
                                      "use fits_mode='new' without a template")
        if obs_mode not in ("PSR", "CAL"):
            raise NotImplementedError("only fold-mode (PSR) output is written")
        self._path = path
        self.obs_mode = obs_mode

    path = property(lambda self: self._path)

    def save(self, signal, pulsar, parfile=None, MJD_start=56000.0, segLength=60.0, inc_len=0.0,
             ref_MJD=56000.0, usePint=True, eq_wts=True, telescope="GBT"):
        if self.path is None:
            raise ValueError("no output path")
        nchan = int(signal.Nchan)
        npol = 1
        period = float(_val(pulsar.period))
        nbin = int(_val(signal.samprate) * 1e6 * period)          # samples per period, as make_pulses
        nsub = int(signal.nsub)
        sublen = float(_val(signal.sublen)) if signal.sublen is not None else float(_val(signal.tobs))
        data = signal.data
        stop = nbin * nsub
        if hasattr(data, "cpu"):
            import torch
            d16 = data[:, :stop].to(torch.int16).cpu().numpy()    # truncation toward zero, as astype
        else:
            d16 = np.asarray(data)[:, :stop].astype(np.int16)
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
