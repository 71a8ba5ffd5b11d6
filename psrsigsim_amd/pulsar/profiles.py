"""Pulse profiles -- mirrors ``psrsigsim/pulsar/profiles.py`` (host tables)."""
import logging

import numpy as np

from .portraits import PulsePortrait, GaussPortrait, DataPortrait, UserPortrait, tile_rows  # noqa: F401

log = logging.getLogger("psrsigsim_amd")

__all__ = ["PulseProfile", "GaussProfile", "UserProfile", "DataProfile"]


class PulseProfile(PulsePortrait):
    """profiles.py:10-65 (1-D profile base class)."""
    _profile = None

    def __call__(self, phases=None):
        if phases is None:
            if self._profile is None:
                print("Warning: base profile not generated, returning `None`")
            return self._profile
        return self.calc_profile(phases)

    def init_profile(self, Nphase):
        ph = np.arange(Nphase) / Nphase
        self._profile = self.calc_profile(ph)
        self._Amax = self._profile.max()
        self._profile = self._profile / self.Amax

    def calc_profile(self, phases):
        raise NotImplementedError()

    @property
    def profile(self):
        return self._profile


class GaussProfile(GaussPortrait):
    """profiles.py:68-115: a GaussPortrait tiled over channels."""

    def __init__(self, peak=0.5, width=0.05, amp=1):
        super().__init__(peak=peak, width=width, amp=amp)

    def set_Nchan(self, Nchan):
        raise NotImplementedError()


class UserProfile(PulseProfile):
    """profiles.py:118-153: profile from a callable."""

    def __init__(self, profile_func):
        self._generator = profile_func

    def calc_profile(self, phases):
        self._profile = self._generator(phases)
        self._Amax = self.Amax if hasattr(self, '_Amax') else np.max(self.profile)
        return self.profile / self.Amax


class DataProfile(DataPortrait):
    """profiles.py:155-205: a sampled 1-D profile tiled to ``Nchan`` rows
    (default 1).  Negative bins are zeroed through ``np.where(...)[0]`` as in
    the reference (for a 2-D input that zeroes whole rows)."""

    def __init__(self, profiles, phases=None, Nchan=None):
        profiles = np.array(profiles, dtype=float)
        if np.any(profiles < 0.0):
            log.warning("Some phase bins of input profile are negative, replacing them with zeros...")
            profiles[np.where(profiles < 0.0)[0]] = 0.0
        self._phases = phases
        if profiles.ndim == 1:
            if Nchan is None:
                Nchan = 1
            profiles = tile_rows(profiles, Nchan)     # np.tile, as a uniform (broadcast) table
        super().__init__(profiles=profiles, phases=phases)

    def set_Nchan(self, Nchan):
        raise NotImplementedError()
