"""Simulation driver (reference: psrsigsim/simulate/simulate.py:18-510).

The natural caller of the synthesis path: parameter
plumbing around FilterBankSignal -> [scatter_broaden(convolve)] -> make_pulses
-> disperse -> Telescope.observe(noise=True), exactly in the reference's order
(simulate.py:292-326).  Nothing here computes: every stage records onto the
signal's pending device pipeline, so ``simulate()`` ends in ONE fused device
run (or none at all until ``signal.data`` is read).  With ``shard=(c0, c1)``
each rank of a multi-GPU run simulates its own channel block.
"""
import logging

import numpy as np

from ..signal import FilterBankSignal
from ..telescope import Telescope, Receiver, Backend
from ..telescope import telescope
from ..pulsar import Pulsar, GaussPortrait, UserPortrait, DataPortrait, DataProfile
from ..ism import ISM

log = logging.getLogger("psrsigsim_amd")

_PARAMS = ("fcent", "bandwidth", "sample_rate", "dtype", "Npols", "Nchan", "sublen", "fold", "period",
           "Smean", "profiles", "specidx", "ref_freq", "tobs", "name", "dm", "tau_d", "tau_d_ref_f",
           "aperture", "area", "Tsys", "tscope_name", "system_name", "rcvr_fcent", "rcvr_bw",
           "rcvr_name", "backend_samprate", "backend_name", "tempfile")


class Simulation(object):
    """simulate.py:18-186 (same parameters, defaults and precedence: manual
    values, then ``parfile`` (NotImplementedError, as there), then
    ``psrdict`` overriding them).  ``shard`` (keyword-only extension) keeps
    only global channels [c0, c1) on this process."""

    def __init__(self, fcent=None, bandwidth=None, sample_rate=None, dtype=np.float32, Npols=1,
                 Nchan=512, sublen=None, fold=True, period=None, Smean=None, profiles=None,
                 specidx=0.0, ref_freq=None, tobs=None, name=None, dm=None, tau_d=None,
                 tau_d_ref_f=None, aperture=None, area=None, Tsys=None, tscope_name=None,
                 system_name=None, rcvr_fcent=None, rcvr_bw=None, rcvr_name=None,
                 backend_samprate=None, backend_name=None, tempfile=None, parfile=None,
                 psrdict=None, *, shard=None):
        vals = locals()
        for k in _PARAMS:
            setattr(self, "_" + k, vals[k])
        self._shard = shard
        if parfile is not None:
            self.params_from_par(parfile)
        if psrdict is not None:
            self.params_from_dict(psrdict)

    def params_from_dict(self, psrdict):
        """simulate.py:188-193: every key becomes ``_<key>``."""
        for key in psrdict.keys():
            setattr(self, "_" + key, psrdict[key])

    def params_from_par(self, parfile):
        """simulate.py:195-199."""
        raise NotImplementedError()

    # -- stages (simulate.py:201-290) -----------------------------------------
    def init_signal(self, from_template=False):
        if from_template:
            # simulate.py:210-214 (note: the reference's simulate() never
            # passes from_template=True through)
            from ..io import PSRFITS
            pfit = PSRFITS(path="sim_fits.fits", template=self.tempfile, fits_mode='copy', obs_mode='PSR')
            self._signal = pfit.make_signal_from_psrfits()
            return
        self._signal = FilterBankSignal(fcent=self.fcent, bandwidth=self.bw, Nsubband=self.Nchan,
                                        sample_rate=self.samprate, fold=self.fold, sublen=self.sublen,
                                        dtype=self.dtype, shard=self._shard)

    def init_profile(self):
        proftypes = (GaussPortrait, UserPortrait, DataPortrait, DataProfile)
        if isinstance(self.profiles, proftypes):
            return
        if isinstance(self.profiles, (list, np.ndarray)):
            if len(self.profiles) == 3:
                prof = GaussPortrait(peak=self.profiles[0], width=self.profiles[1], amp=self.profiles[2])
            elif len(self.profiles) > 3:
                prof = DataProfile(self.profiles, phases=None, Nchan=self.Nchan)
            else:
                raise RuntimeError("Input profile array has too few values!")
        elif callable(self.profiles):
            raise NotImplementedError()
        else:
            log.warning("Unrecognized input profile type, defaulting to Gaussian.")
            prof = GaussPortrait()
        self._profiles = prof

    def init_pulsar(self):
        self._pulsar = Pulsar(period=self.period, Smean=self.Smean, profiles=self.profiles,
                              name=self.name, specidx=self.specidx, ref_freq=self.ref_freq)

    def init_ism(self):
        self._ism = ISM()

    def init_telescope(self):
        if self.tscope_name == 'GBT':
            tscope = telescope.GBT()
        elif self.tscope_name == 'Arecibo':
            tscope = telescope.Arecibo()
        else:
            tscope = Telescope(self.aperture, area=self.area, Tsys=self.Tsys, name=self.tscope_name)
        if type(self.rcvr_fcent) is list:
            n = len(self.rcvr_fcent)
            if not (len(self.system_name) == n == len(self.rcvr_bw) == len(self.rcvr_name)
                    == len(self.backend_samprate) == len(self.backend_name)):
                raise RuntimeError("Number of telescope system entries do not match!")
            for ii in range(n):
                tscope.add_system(name=self.system_name[ii],
                                  receiver=Receiver(fcent=self.rcvr_fcent[ii], bandwidth=self.rcvr_bw[ii],
                                                    name=self.rcvr_name[ii]),
                                  backend=Backend(samprate=self.backend_samprate[ii], name=self.backend_name[ii]))
        elif self.rcvr_fcent is not None:
            tscope.add_system(name=self.system_name,
                              receiver=Receiver(fcent=self.rcvr_fcent, bandwidth=self.rcvr_bw, name=self.rcvr_name),
                              backend=Backend(samprate=self.backend_samprate, name=self.backend_name))
        self._tscope = tscope

    def simulate(self, from_template=False):
        """simulate.py:292-326 (the reference passes from_template=False to
        init_signal regardless of the argument; so does this)."""
        self.init_signal(from_template=False)
        self.init_profile()
        self.init_pulsar()
        self.init_ism()
        if self.tau_d is not None:
            self.ism.scatter_broaden(self.signal, self.tau_d, self.tau_d_ref_f, convolve=True, pulsar=self.pulsar)
        self.pulsar.make_pulses(self.signal, tobs=self.tobs)
        self.ism.disperse(self.signal, self.dm)
        self.init_telescope()
        self.tscope.observe(self.signal, self.pulsar, system=self.system_name, noise=True)

    def save_simulation(self, outfile="simfits", out_format='psrfits', parfile=None, ref_MJD=56000.0,
                        MJD_start=55999.9861):
        """simulate.py:328-378.  'psrfits' copies the template file with the
        reference's edits (io.PSRFITS; the POLYCO table stays the template's:
        PINT is absent), 'pdv' writes the PSRCHIVE pdv text format
        (io.TxtFile)."""
        if out_format.lower() == 'psrfits':
            from ..io import PSRFITS
            from ..utils import make_par
            if outfile == 'simfits':
                outfile += ".fits"
            if self.tempfile is None:
                raise RuntimeError("No template PSRFITS file provided.")
            pfit = PSRFITS(path=outfile, template=self.tempfile, fits_mode='copy', obs_mode='PSR')
            pfit.get_signal_params(signal=self.signal)
            if parfile is None:
                log.warning("No par file provided, attempting to make one...")
                make_par(self.signal, self.pulsar, outpar="simpar.par")
                parfile = "simpar.par"
            pfit.save(self.signal, self.pulsar, parfile=parfile, MJD_start=MJD_start, segLength=60.0,
                      ref_MJD=ref_MJD, usePint=True)
        elif out_format.lower() == 'pdv':
            from ..io import TxtFile
            if outfile == 'simfits':
                outfile += ".ar"
            TxtFile(path=outfile).save_psrchive_pdv(self.signal, self.pulsar)
        else:
            raise RuntimeError("Unrecognized output file format: %s" % (out_format))

    # -- properties (simulate.py:380-510) -----------------------------------
    fold = property(lambda self: self._fold)
    sublen = property(lambda self: self._sublen)
    Nchan = property(lambda self: self._Nchan)
    fcent = property(lambda self: self._fcent)
    bw = property(lambda self: self._bandwidth)
    tobs = property(lambda self: self._tobs)
    samprate = property(lambda self: self._sample_rate)
    dtype = property(lambda self: self._dtype)
    Npols = property(lambda self: self._Npols)
    dm = property(lambda self: self._dm)
    tau_d = property(lambda self: self._tau_d)
    tau_d_ref_f = property(lambda self: self._tau_d_ref_f)
    profiles = property(lambda self: self._profiles)
    name = property(lambda self: self._name)
    period = property(lambda self: self._period)
    Smean = property(lambda self: self._Smean)
    specidx = property(lambda self: self._specidx)
    ref_freq = property(lambda self: self._ref_freq)
    tscope_name = property(lambda self: self._tscope_name)
    area = property(lambda self: self._area)
    aperture = property(lambda self: self._aperture)
    Tsys = property(lambda self: self._Tsys)
    system_name = property(lambda self: self._system_name)
    rcvr_fcent = property(lambda self: self._rcvr_fcent)
    rcvr_bw = property(lambda self: self._rcvr_bw)
    rcvr_name = property(lambda self: self._rcvr_name)
    backend_samprate = property(lambda self: self._backend_samprate)
    backend_name = property(lambda self: self._backend_name)
    tempfile = property(lambda self: self._tempfile)
    signal = property(lambda self: self._signal)
    pulsar = property(lambda self: self._pulsar)
    ism = property(lambda self: self._ism)
    tscope = property(lambda self: self._tscope)
