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

No POLYCO / PSRPARAM tables (PINT is absent): files are not phase-connected.
``read_psrfits`` parses what ``save`` writes (tests, and round trips).
The device data is read back once (one D2H copy of the folded product; in a
multi-GPU run gather it first with ``psrsigsim_amd.shard.gather_channels``).
"""
import math

import numpy as np

from .._units import Quantity

__all__ = ["PSRFITS", "read_psrfits"]

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
        cols = [("TSUBINT", "1D", None), ("OFFS_SUB", "1D", None), ("DAT_FREQ", "%dD" % nchan, None),
                ("DAT_WTS", "%dE" % nchan, None), ("DAT_OFFS", "%dE" % (nchan * npol), None),
                ("DAT_SCL", "%dE" % (nchan * npol), None),
                ("DATA", "%dI" % (nbin * nchan * npol), "(%d,%d,%d)" % (nbin, nchan, npol))]
        row = np.dtype([("TSUBINT", ">f8"), ("OFFS_SUB", ">f8"), ("DAT_FREQ", ">f8", (nchan,)),
                        ("DAT_WTS", ">f4", (nchan,)), ("DAT_OFFS", ">f4", (nchan * npol,)),
                        ("DAT_SCL", ">f4", (nchan * npol,)), ("DATA", ">i2", (npol, nchan, nbin))])
        tab = np.zeros(nsub, dtype=row)
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
    cards = {}
    order = []
    while True:
        block = buf[pos:pos + _BLOCK].decode("ascii")
        pos += _BLOCK
        done = False
        for i in range(0, _BLOCK, 80):
            c = block[i:i + 80]
            key = c[:8].strip()
            if key == "END":
                done = True
                break
            if c[8:10] == "= ":
                v = c[10:].split(" / ")[0].strip()
                if v.startswith("'"):
                    v = v[1:v.rindex("'")].rstrip().replace("''", "'")
                elif v in ("T", "F"):
                    v = v == "T"
                else:
                    v = float(v) if any(ch in v for ch in ".EeDd") else int(v)
                cards[key] = v
                order.append(key)
        if done:
            return cards, pos


def read_psrfits(path):
    """(primary header dict, SUBINT header dict, SUBINT records) of a file
    written by :meth:`PSRFITS.save`."""
    buf = open(path, "rb").read()
    prim, pos = _parse_header(buf, 0)
    sub, pos = _parse_header(buf, pos)
    fmt = {"D": ">f8", "E": ">f4", "I": ">i2", "J": ">i4"}
    fields = []
    for i in range(1, sub["TFIELDS"] + 1):
        form = sub["TFORM%d" % i]
        n, code = int(form[:-1] or 1), form[-1]
        shape = (n,) if n > 1 else ()
        dim = sub.get("TDIM%d" % i)
        if dim:
            shape = tuple(int(x) for x in dim.strip("()").split(","))[::-1]
        fields.append((sub["TTYPE%d" % i], fmt[code], shape))
    dt = np.dtype(fields)
    assert dt.itemsize == sub["NAXIS1"]
    rec = np.frombuffer(buf, dtype=dt, count=sub["NAXIS2"], offset=pos)
    return prim, sub, rec
