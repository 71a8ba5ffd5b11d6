"""Signal base class -- mirrors ``psrsigsim/signal/signal.py``."""
import numpy as np

__all__ = ["Signal", "BaseSignal"]


class BaseSignal(object):
    """signal.py:11-165 (attributes and properties)."""
    _sigtype = "Signal"
    _Nchan = None
    _tobs = None
    _nsamp = None
    _draw_max = None
    _draw_norm = 1

    def __init__(self, fcent, bandwidth, sample_rate=None, dtype=np.float32, Npols=1):
        self._fcent = fcent
        self._bw = abs(bandwidth)
        self._samprate = sample_rate
        self._dtype = dtype
        if Npols != 1:
            raise ValueError("Only total intensity polarization is currently supported")
        self._Npols = 1
        self._delay = None
        self._dm = None

    def __repr__(self):
        return self.sigtype + "({0}, bw={1})".format(self.fcent, self.bw)

    def __add__(self, b):
        raise NotImplementedError()

    def _set_draw_norm(self):
        raise NotImplementedError()

    def to_RF(self):
        raise NotImplementedError()

    def to_Baseband(self):
        raise NotImplementedError()

    def to_FilterBank(self, Nsubband=512):
        raise NotImplementedError()

    @property
    def sigtype(self):
        return self._sigtype

    @property
    def Nchan(self):
        return self._Nchan

    @property
    def fcent(self):
        return self._fcent

    @property
    def bw(self):
        return self._bw

    @property
    def tobs(self):
        return self._tobs

    @property
    def samprate(self):
        return self._samprate

    @property
    def nsamp(self):
        return self._nsamp

    @property
    def dtype(self):
        return self._dtype

    @property
    def Npols(self):
        return self._Npols

    @property
    def dat_freq(self):
        return self._dat_freq

    @property
    def delay(self):
        return self._delay

    @property
    def dm(self):
        return self._dm

    @property
    def DM(self):
        return self._dm


def Signal():
    raise NotImplementedError()
