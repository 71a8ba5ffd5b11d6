"""Backend -- mirrors ``psrsigsim/telescope/backend.py``."""
import torch

from .._units import make_quant, to_value
from .. import _engine, _lib

__all__ = ['Backend']


class Backend(object):
    def __init__(self, samprate=None, name=None):
        self._name = name
        self._samprate = make_quant(samprate, "MHz")

    def __repr__(self):
        return "Backend({:s})".format(self._name)

    @property
    def name(self):
        return self._name

    @property
    def samprate(self):
        return self._samprate

    def adc(self, signal):
        """backend.py:27-31 (unimplemented there too)."""

    def fold(self, signal, pulsar):
        """backend.py:34-49: Npbins = int(P * 2 * signal.samprate);
        sum over the N_fold blocks of Npbins//2 samples that follow the first
        Npbins samples.  As in the reference the reshape only succeeds when
        Nt - Npbins == N_fold * (Npbins//2), else ValueError."""
        data = signal.data
        Nf, Nt = data.shape
        P = float(to_value(pulsar.period, 's'))
        Npbins = int((P * 2 * signal._samprate_MHz()) * 1e6)
        N_fold = Nt // Npbins
        width = min(Nt, Npbins * (N_fold + 1)) - Npbins
        if width != N_fold * (Npbins // 2):
            raise ValueError("cannot reshape array of size %d into shape (%d,%d,%d)"
                             % (Nf * max(width, 0), Nf, N_fold, Npbins // 2))
        out = torch.empty((Nf, Npbins // 2), dtype=torch.float32, device=data.device)
        rc = _lib.lib().pss_fold(_engine.ptr(data), _engine.ptr(out), Nf, data.stride(0), Npbins,
                                 N_fold, _engine.stream_ptr())
        _lib.check(rc, "fold")
        return out

    def fold_periods(self, signal, pulsar, nbin=None):
        """Corrected fold (extension; the reference's ``fold`` above is only
        valid for exactly four periods): the sum of the signal over its whole
        periods of ``nbin`` samples (default ``int(P * samprate)``, the
        samples per period make_pulses uses), on the device.  Trailing samples
        of an incomplete period are dropped.  Returns [Nchan, nbin] float32."""
        data = signal.data
        Nf, Nt = data.shape
        if nbin is None:
            P = float(to_value(pulsar.period, 's'))
            nbin = int(P * signal._samprate_MHz() * 1e6)
        nbin = int(nbin)
        nper = Nt // nbin if nbin > 0 else 0
        if nbin < 1 or nper < 1:
            raise ValueError("fold_periods: %d samples hold no whole period of %d bins" % (Nt, nbin))
        out = torch.empty((Nf, nbin), dtype=torch.float32, device=data.device)
        rc = _lib.lib().pss_fold_periods(_engine.ptr(data), _engine.ptr(out), Nf, data.stride(0), nbin, nper,
                                         _engine.stream_ptr())
        _lib.check(rc, "fold_periods")
        return out
