"""Telescope -- mirrors ``psrsigsim/telescope/telescope.py``.

observe() decides the resampling branch exactly as the reference (float
comparisons of unit-converted dt's, telescope.py:94-126), attaches the
pre-noise ``out`` copy and the radiometer-noise stage to the signal's pending
pipeline and executes it as one fused device run.  On the down_sample /
rebin branches the run itself produces the resampled, clipped and cast
``out`` (telescope.py:108-125, 140-145): its epilogue adds every pre-noise
sample into float64 window sums and one small kernel divides, clips and casts
them (PssPipeline.out_len) -- no full-resolution copy, no separate resampling
or clip pass.
"""
import numpy as np
import torch

from .receiver import Receiver, _flat_response, response_from_data  # noqa: F401
from .backend import Backend
from .._units import make_quant
from .. import _engine, _lib
from ..utils.utils import rebin_edges

__all__ = ['Telescope', 'GBT', 'Arecibo']

_kB = make_quant(1.38064852e+03, "Jy*m^2/K")  # Boltzmann const in radio units


class Telescope(object):
    """telescope.py:14-162."""

    def __init__(self, aperture, area=None, Tsys=None, name=None):
        self._name = name
        self._aperture = make_quant(aperture, "m")
        self._systems = {}
        if area is None:
            self._area = np.pi * (self.aperture / 2) ** 2
        else:
            self._area = make_quant(area, "m^2")
        self._gain = self.area / (2 * _kB)
        if Tsys is None:
            self._Tsys = Tsys
        else:
            self._Tsys = make_quant(Tsys, "K")

    def __repr__(self):
        return "Telescope({:s}, {:f}m)".format(self._name, float(self._aperture.value))

    @property
    def name(self):
        return self._name

    @property
    def area(self):
        return self._area

    @property
    def gain(self):
        return self._gain

    @property
    def aperture(self):
        return self._aperture

    @property
    def systems(self):
        return self._systems

    @property
    def Tsys(self):
        return self._Tsys

    def add_system(self, name=None, receiver=None, backend=None):
        self._systems[name] = (receiver, backend)

    @staticmethod
    def resample_branch(signal, bak):
        """telescope.py:94-126 -> ('copy'|'down'|'rebin', arg)."""
        dt_tel = 1 / (2 * bak.samprate)
        if signal.sigtype == "FilterBankSignal" and signal.sublen is not None:
            dt_sig = signal.sublen / (signal.nsamp / signal.nsub)
        else:
            dt_sig = signal.tobs / signal.nsamp
        if bool(dt_sig == dt_tel):
            return "copy", None
        if bool((dt_tel % dt_sig) == 0):
            return "down", int(float(dt_tel // dt_sig))
        if bool(dt_tel > dt_sig):
            return "rebin", int(float(signal.tobs // dt_tel))
        return "copy", None

    def observe(self, signal, pulsar, system=None, noise=False, ret_resampsig=False):
        """telescope.py:72-149."""
        if signal.sigtype in ["RFSignal", "BasebandSignal"]:
            raise NotImplementedError
        rcvr, bak = self.systems[system][0], self.systems[system][1]
        kind, arg = self.resample_branch(signal, bak)
        # a pending noise stage belongs BEFORE this observe's pre-noise copy
        if signal._pending is not None and signal._pending.noise is not None:
            signal._flush()
        pend = signal._pend()
        rows, ncols = signal._c1 - signal._c0, signal._ncols
        dev = _engine.device()
        odt = torch.int8 if signal.dtype is np.int8 else torch.float32
        okind = _lib.OUT_I8 if signal.dtype is np.int8 else _lib.OUT_F32
        clip = float(signal._draw_max) if signal._draw_max is not None else float("inf")
        # The reference always builds `out` but only returns it on request;
        # here it is produced only when it is observable (ret_resampsig).
        out = None
        if ret_resampsig and kind == "copy":
            out = torch.empty((rows, ncols), dtype=odt, device=dev)
            pend.out = {"kind": okind, "tensor": out, "clip": clip}
        elif ret_resampsig:
            if kind == "down":
                # telescope.py:108-114 (down_sample: reshape(-1, fact).mean)
                new_Nt = int(signal.nsamp // arg)
                if ncols % arg or ncols // arg != new_Nt:
                    raise ValueError("could not broadcast input array from shape (%d,) into shape (%d,)"
                                     % (ncols // max(arg, 1), new_Nt))
                win = {"len": new_Nt, "lo": None, "hi": None, "step": float(arg)}
            else:
                # telescope.py:116-125 (rebin: ceil-edged windows, nanmean)
                new_Nt = int(arg)
                lo, hi = rebin_edges(ncols, new_Nt)
                step = float(np.linspace(0, ncols, new_Nt, endpoint=False)[1]) if new_Nt > 1 else float(ncols)
                win = {"len": new_Nt, "lo": _engine.to_dev(lo), "hi": _engine.to_dev(hi), "step": step}
            out = torch.empty((rows, new_Nt), dtype=odt, device=dev)
            win["acc"] = torch.empty((rows, new_Nt), dtype=torch.float64, device=dev)
            pend.out = {"kind": okind, "tensor": out, "clip": clip, "windows": win}
        if noise:
            rcvr.radiometer_noise(signal, pulsar, gain=self.gain, Tsys=self.Tsys)
        signal._flush()
        if ret_resampsig:
            # the returned copy is a read-out of the data: a null() whose
            # channel-0 maximum was not unique raises here, as the reference's
            # null() would have (pulsar.py:286); without ret_resampsig the
            # check stays deferred to the next read (no host sync per observe)
            _engine.check_null_status(signal)
            return out

    def apply_response(self, signal):
        raise NotImplementedError()

    def rfi(self):
        raise NotImplementedError()

    def init_signal(self, system):
        raise NotImplementedError()


def GBT():
    """telescope.py:186-206: the 100 m Green Bank Telescope."""
    g = Telescope(100.0, area=5500.0, Tsys=35.0, name="GBT")
    g.add_system(name="820_GUPPI", receiver=Receiver(fcent=820, bandwidth=180, name="820"),
                 backend=Backend(samprate=3.125, name="GUPPI"))
    g.add_system(name="Lband_GUPPI", receiver=Receiver(fcent=1400, bandwidth=800, name="Lband"),
                 backend=Backend(samprate=12.5, name="GUPPI"))
    g.add_system(name="800_GASP", receiver=Receiver(fcent=844, bandwidth=64, name="800"),
                 backend=Backend(samprate=0.25, name="GASP"))
    g.add_system(name="Lband_GASP", receiver=Receiver(fcent=1410, bandwidth=64, name="Lband"),
                 backend=Backend(samprate=0.25, name="GASP"))
    return g


def Arecibo():
    """telescope.py:209-239: the Arecibo 300 m Telescope."""
    a = Telescope(300.0, area=22000.0, Tsys=35.0, name="Arecibo")
    a.add_system(name="430_PUPPI", receiver=Receiver(fcent=430, bandwidth=100, name="430"),
                 backend=Backend(samprate=1.5625, name="PUPPI"))
    a.add_system(name="Lband_PUPPI", receiver=Receiver(fcent=1410, bandwidth=800, name="Lband"),
                 backend=Backend(samprate=12.5, name="PUPPI"))
    a.add_system(name="Sband_PUPPI", receiver=Receiver(fcent=2030, bandwidth=400, name="Sband"),
                 backend=Backend(samprate=12.5, name="PUPPI"))
    a.add_system(name="327_ASP", receiver=Receiver(fcent=327, bandwidth=64, name="327"),
                 backend=Backend(samprate=0.25, name="ASP"))
    a.add_system(name="430_ASP", receiver=Receiver(fcent=432, bandwidth=64, name="430"),
                 backend=Backend(samprate=0.25, name="ASP"))
    a.add_system(name="Lband_ASP", receiver=Receiver(fcent=1412, bandwidth=64, name="Lband"),
                 backend=Backend(samprate=0.25, name="ASP"))
    a.add_system(name="Sband_ASP", receiver=Receiver(fcent=2348, bandwidth=64, name="Sband"),
                 backend=Backend(samprate=0.25, name="ASP"))
    return a
