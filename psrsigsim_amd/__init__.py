"""psrsigsim_amd -- MI355X-native engine for PsrSigSim's filterbank synthesis path.

Drop-in for ``psrsigsim.signal / pulsar / ism / telescope / utils`` on that
path (FilterBankSignal, Pulsar.make_pulses / null, ISM.disperse / FD_shift /
scatter_broaden, Telescope.observe, Receiver.radiometer_noise, Backend.fold,
utils.shift_t / down_sample / rebin).  ``signal.data`` is a device-resident
torch tensor produced by hand-written gfx950 HIP kernels (libpss_hip.so).

Randomness: ``psrsigsim_amd.seed(s)`` (counter-based Philox; the analogue of
``np.random.seed``).
"""
__version__ = "0.1.0"

from ._engine import seed, inject  # noqa: F401
from . import signal, pulsar, ism, telescope, utils  # noqa: F401
