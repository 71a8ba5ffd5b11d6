"""Receiver -- mirrors ``psrsigsim/telescope/receiver.py``.

radiometer_noise computes the noise scale on the host (receiver.py:140-172,
float64) and appends the noise stage; chi2 draws x scale are added on the GPU
in the epilogue of the fused run (full resolution, in place, unclipped).
"""
import numpy as np

from .._units import make_quant, to_value
from .. import _engine

__all__ = ['Receiver']


class Receiver(object):
    """receiver.py:12-80."""

    def __init__(self, response=None, fcent=None, bandwidth=None, Trec=35, name=None):
        if response is None:
            if fcent is None or bandwidth is None:
                raise ValueError("specify EITHER response OR fcent and bandwidth")
            self._response = _flat_response(fcent, bandwidth)
        else:
            if fcent is not None or bandwidth is not None:
                raise ValueError("specify EITHER response OR fcent and bandwidth")
            self._response = response
            raise NotImplementedError("Non-flat response not yet implemented.")
        self._Trec = make_quant(Trec, "K")
        self._name = name
        self._fcent = make_quant(fcent, "MHz")
        self._bandwidth = make_quant(bandwidth, "MHz")

    def __repr__(self):
        return "Receiver({:s})".format(self._name)

    @property
    def name(self):
        return self._name

    @property
    def Trec(self):
        return self._Trec

    @property
    def response(self):
        return self._response

    @property
    def fcent(self):
        return self._fcent

    @property
    def bandwidth(self):
        return self._bandwidth

    def radiometer_noise(self, signal, pulsar, gain=1, Tsys=None, Tenv=None):
        """receiver.py:82-121: Tsys = Tsys, or Tenv + Trec, or Trec."""
        Tsys_check = Tsys.value if hasattr(Tsys, 'value') else Tsys
        Tenv_check = Tenv.value if hasattr(Tenv, 'value') else Tenv
        if Tsys_check is None and Tenv_check is None:
            Tsys = self.Trec
        elif Tenv_check is not None:
            if Tsys_check is not None:
                raise ValueError("specify EITHER Tsys OR Tenv, not both")
            Tsys = make_quant(Tenv, 'K') + self.Trec
        gain = make_quant(gain, "K/Jy")
        if signal.sigtype in ["RFSignal", "BasebandSignal"]:
            raise NotImplementedError("amplitude noise is outside the filterbank path")
        elif signal.sigtype == "FilterBankSignal":
            self._make_pow_noise(signal, Tsys, gain, pulsar)
        else:
            raise NotImplementedError("no pulse method for signal: {}".format(signal.sigtype))

    def _make_amp_noise(self, signal, Tsys, gain, pulsar):
        raise NotImplementedError("amplitude noise is outside the filterbank path")

    @staticmethod
    def noise_norm(signal, pulsar, Tsys, gain):
        """receiver.py:143-169 scale: Tsys/gain/sqrt(2 dt bw/C) * draw_norm / Smax
        * nbins / sum(max_profile), in Jy-normalised units."""
        Tsys_K = float(to_value(make_quant(Tsys, 'K'), 'K'))
        gain_v = float(to_value(make_quant(gain, 'K/Jy'), 'K/Jy'))
        nbins = signal.nsamp / signal.nsub
        dt = float(to_value(signal.sublen, 's')) / nbins
        bw_per_chan = float(to_value(signal.bw, 'MHz')) / signal.Nchan
        sigS = Tsys_K / gain_v / np.sqrt(2 * dt * bw_per_chan) * 1e-3      # Jy
        U_scale = 1.0 / (np.sum(pulsar.Profiles._max_profile) / nbins)
        Smax = float(to_value(signal._Smax, 'Jy'))
        return (sigS * signal._draw_norm / Smax) * U_scale

    def _make_pow_noise(self, signal, Tsys, gain, pulsar):
        """receiver.py:140-172: data += norm * chi2(Nfold if fold else 1)."""
        norm = self.noise_norm(signal, pulsar, Tsys, gain)
        df = float(signal.Nfold) if signal.fold else 1.0
        pend = signal._pend()
        if pend.noise is not None:
            signal._flush()
            pend = signal._pend()
        pend.noise = {"norm": float(norm), "df": df, "call_id": _engine.next_call(),
                      "inj": _engine.take_injection("noise")}


def response_from_data(fs, values):
    raise NotImplementedError()


def _flat_response(fcent, bandwidth):
    """receiver.py:182-197."""
    fc = float(to_value(make_quant(fcent, 'MHz'), 'MHz'))
    bw = float(to_value(make_quant(bandwidth, 'MHz'), 'MHz'))
    fmin = fc - bw / 2
    fmax = fc + bw / 2
    return lambda f: np.heaviside(np.asarray(f) - fmin, 0) * np.heaviside(fmax - np.asarray(f), 0)
