"""FilterBankSignal -- mirrors ``psrsigsim/signal/fb_signal.py`` with a
device-resident (Nchan, nsamp) float32 buffer.

``signal.data`` is a torch tensor on the current HIP device; reading it
executes any pending (deferred, fused) stages first.  The optional
keyword-only ``shard=(c0, c1)`` keeps only global channels [c0, c1) on this
process (multi-GPU channel sharding); every per-channel quantity and every
random draw is keyed by the GLOBAL channel, so a sharded run produces exactly
the rows of the unsharded one.  Keyword-only ``plan_group`` (a host process
group whose ranks hold a partition of the band) also splits the host
planning of the profile tables over those ranks (psrsigsim_amd.shard.RowSet).
"""
import numpy as np
from scipy import stats

from .signal import BaseSignal
from .._units import make_quant, Quantity, to_value
from .. import _engine

__all__ = ["FilterBankSignal"]


class FilterBankSignal(BaseSignal):
    """fb_signal.py:11-160."""
    _sigtype = "FilterBankSignal"
    _Nfold = None

    def __init__(self, fcent, bandwidth, Nsubband=512, sample_rate=None, sublen=None,
                 dtype=np.float32, fold=True, *, shard=None, plan_group=None):
        self._Npols = 1
        self._fcent = make_quant(fcent, 'MHz')
        if bandwidth < 0:
            self._bw = make_quant(np.abs(bandwidth), 'MHz')
        else:
            self._bw = make_quant(bandwidth, 'MHz')
        self._fold = fold
        if self.fold and sublen is not None:
            self._sublen = make_quant(sublen, 's')
        else:
            self._sublen = sublen
        f_Nyquist = 2 * self._bw
        if sample_rate is None:
            self._samprate = (1 / make_quant(20.48, 'us')).to('MHz')
        else:
            self._samprate = make_quant(sample_rate, 'MHz')
            if self._samprate < f_Nyquist:
                print("Warning: specified sample rate {} < Nyquist frequency {}"
                      .format(self._samprate, f_Nyquist))
        self._Nchan = Nsubband
        first = (self._fcent - self._bw / 2).to('MHz').value
        last = (self._fcent + self._bw / 2).to('MHz').value
        step = (self._bw / self._Nchan).to('MHz').value
        self._dat_freq = Quantity(np.arange(first, last, step), 'MHz')
        self._dtype = dtype
        self._set_draw_norm()
        self._delay = None
        self._dm = None
        # device state
        c0, c1 = (0, Nsubband) if shard is None else (int(shard[0]), int(shard[1]))
        if not (0 <= c0 < c1 <= Nsubband):
            raise ValueError("bad shard %r for %d channels" % (shard, Nsubband))
        self._c0, self._c1 = c0, c1
        # shard-local host planning (shard.RowSet): the ranks of plan_group
        # hold a partition of the band and plan their own profile rows
        self._rowset = None
        if plan_group is not None:
            from ..shard import RowSet
            self._rowset = RowSet(c0, c1, Nsubband, plan_group)
        self._buf = None
        self._row0 = None
        self._track_row0 = True
        self._ncols = 0
        self._pending = None

    def _set_draw_norm(self, df=1):
        """fb_signal.py:114-121 (identity tests on the dtype, as there)."""
        if self.dtype is np.float32:
            self._draw_max = 200
            self._draw_norm = 1
        if self.dtype is np.int8:
            limit = stats.chi2.ppf(0.999, float(df))
            self._draw_max = np.iinfo(np.int8).max
            self._draw_norm = self._draw_max / limit

    # -- deferred execution ----------------------------------------------
    def _flush(self):
        """Execute the pending stages (one fused device run)."""
        pend = self._pending
        if pend is None or pend.empty():
            self._pending = None
            return
        _engine.execute(self, pend)
        self._pending = None

    def _pend(self):
        """The pending pipeline to append a stage to (loads existing data when
        nothing is pending)."""
        if self._pending is None:
            if self._buf is None:
                raise ValueError("signal has no data: call Pulsar.make_pulses first")
            self._pending = _engine.Pending(None)
        return self._pending

    @property
    def data(self):
        self._flush()
        _engine.check_null_status(self)
        return self._buf

    def data_numpy(self):
        """Host copy of the (local) data as float64, like the reference's
        ``signal.data``."""
        return self.data.cpu().numpy().astype(np.float64)

    @property
    def shard(self):
        return (self._c0, self._c1)

    @property
    def local_dat_freq(self):
        return self._dat_freq[self._c0:self._c1]

    # -- properties --------------------------------------------------------
    @property
    def fold(self):
        return self._fold

    @property
    def sublen(self):
        return self._sublen

    @property
    def Nfold(self):
        return self._Nfold

    @property
    def nsub(self):
        return self._nsub

    def to_RF(self):
        raise NotImplementedError()

    def to_Baseband(self):
        raise NotImplementedError()

    def to_FilterBank(self, Nsubband=512):
        return self

    # -- helpers for the engine (float64 working units) -------------------
    def _samprate_MHz(self):
        return float(to_value(self._samprate, 'MHz'))

    def _dt_ms(self):
        """(1/samprate).to('ms') (ism.py:49)."""
        return float((1 / self._samprate).to('ms').value)

    def _freqs_MHz(self):
        return np.asarray(self._dat_freq.to('MHz').value, dtype=np.float64)
