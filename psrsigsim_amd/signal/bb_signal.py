"""BasebandSignal -- mirrors ``psrsigsim/signal/bb_signal.py`` with a
device-resident (Nchan, nsamp) float32 buffer (Nchan = polarisation channels,
default 2).  Amplitude pulses (``Pulsar._make_amp_pulses``) and coherent
dispersion (``ISM._disperse_baseband``) run on the device through the same
C-ABI engine as the filterbank path; ``Telescope.observe`` rejects baseband
signals as the reference does (telescope.py:86-87)."""
import numpy as np

from .signal import BaseSignal
from .._units import make_quant, to_value
from .. import _engine

__all__ = ["BasebandSignal"]


class BasebandSignal(BaseSignal):
    """bb_signal.py:11-76."""
    _sigtype = "BasebandSignal"

    def __init__(self, fcent, bandwidth, sample_rate=None, dtype=np.float32, Nchan=2):
        self._fcent = make_quant(fcent, 'MHz')
        self._bw = make_quant(bandwidth, 'MHz')
        self._Nchan = Nchan
        self._Npols = 1
        f_Nyquist = 2 * self._bw
        if sample_rate is None:
            self._samprate = f_Nyquist
        else:
            self._samprate = make_quant(sample_rate, 'MHz')
            if self._samprate < f_Nyquist:
                print("Warning: specified sample rate {} < Nyquist frequency {}"
                      .format(self._samprate, f_Nyquist))
        self._dtype = dtype
        self._delay = None
        self._dm = None
        self._dat_freq = None
        # device state (the engine's view: every channel local, no null shadow)
        self._c0, self._c1 = 0, Nchan
        self._buf = None
        self._row0 = None
        self._track_row0 = False
        self._ncols = 0
        self._pending = None

    def to_RF(self):
        raise NotImplementedError()

    def to_Baseband(self):
        return self

    def to_FilterBank(self, Nsubband=512):
        raise NotImplementedError()

    # -- deferred execution (same contract as FilterBankSignal) ----------
    def _flush(self):
        pend = self._pending
        if pend is None or pend.empty():
            self._pending = None
            return
        _engine.execute(self, pend)
        self._pending = None

    @property
    def data(self):
        self._flush()
        return self._buf

    def data_numpy(self):
        return self.data.cpu().numpy().astype(np.float64)

    def _samprate_MHz(self):
        return float(to_value(self._samprate, 'MHz'))

    def _dt_s(self):
        """(1/samprate).to('us').to('s') (ism.py:84, 87)."""
        return float((1 / self._samprate).to('us').to('s').value)
