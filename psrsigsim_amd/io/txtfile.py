"""PSRCHIVE pdv text output (reference: psrsigsim/io/txtfile.py:10-182).

Host I/O after the device run: the signal's rows are read back once and
formatted exactly as the reference does, including its quirks (the RMS in the
header divides by the number of CHANNELS, ``len(signal.data)``; every subint
lists bins 0..nbin-1 of each channel; a file is written after every hundred
channel blocks, numbered floor(count / 100), with the count never reset)."""
import numpy as np

from .._units import Quantity
from ..utils import make_quant


def _val(q):
    return q.value if isinstance(q, Quantity) else q


class TxtFile(object):
    def __init__(self, path=None):
        self._path = path
        self.nchan = self.nbin = self.npol = self.nrows = None
        self._tbin = self._tsubint = self._chan_bw = self._obsbw = self._obsfreq = None

    path = property(lambda self: self._path)

    def save_psrchive_pdv(self, signal, pulsar):
        """txtfile.py:37-92."""
        self._get_signal_params(signal, pulsar)
        if self.path is None:
            self._path = "PsrSigSim_Simulated_Pulsar.ar"
        data = signal.data
        data = data.cpu().numpy() if hasattr(data, "cpu") else np.asarray(data)
        rms = np.sqrt((1.0 / len(data)) * np.sum(data.astype(np.float64) ** 2))
        header = "# File: %s Src: %s Nsub: %s Nch: %s Npol: %s Nbin: %s RMS: %s \n" % \
            (self.path, pulsar.name, str(self.nrows), str(self.nchan), str(self.npol), str(self.nbin), str(rms))
        lines = [header]
        dump_val = 0
        tsub_day = _val(self.tsubint) / 86400.0
        freqs = np.asarray(_val(signal.dat_freq), dtype=float)
        for ii in range(self.nrows):
            mjd_mid = 56000.0 + (ii + 1) * tsub_day / 2.0
            for ff in range(self.nchan):
                lines.append("# MJD(mid): %s Tsub: %s Freq: %s BW: %s \n"
                             % (mjd_mid, _val(self.tsubint), freqs[ff], _val(self.obsbw) / self.nchan))
                row = data[ff]
                lines.extend("%s %s %s %s \n" % (ii, ff, bb, row[bb]) for bb in range(self.nbin))
                dump_val += 1
            if dump_val >= 100:
                with open(self.path + "_%s.txt" % (str(int(np.floor(dump_val / 100)))), 'w') as f:
                    f.writelines(lines)
                lines = [header]
        with open(self.path + "_%s.txt" % (str(int(np.floor(dump_val / 100)))), 'w') as f:
            f.writelines(lines)

    def _get_signal_params(self, signal, pulsar):
        """txtfile.py:94-110."""
        self.nchan = signal.Nchan
        self._tbin = make_quant(1.0 / _val(signal.samprate), 'us')
        self.nbin = int(_val(signal.samprate) * 1e6 * _val(make_quant(pulsar.period, 's')))
        self.npol = signal.Npols
        self.nrows = signal.nsub
        self._obsfreq = signal.fcent
        self._obsbw = signal.bw
        self._chan_bw = make_quant(_val(signal.bw) / signal.Nchan, 'MHz')
        self._tsubint = make_quant(_val(signal.sublen), 'second')

    tbin = property(lambda self: self._tbin)
    obsfreq = property(lambda self: self._obsfreq)
    obsbw = property(lambda self: self._obsbw)
    chan_bw = property(lambda self: self._chan_bw)
    tsubint = property(lambda self: self._tsubint)
