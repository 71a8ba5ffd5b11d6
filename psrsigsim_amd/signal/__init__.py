from .signal import Signal, BaseSignal  # noqa: F401
from .fb_signal import FilterBankSignal  # noqa: F401
from .bb_signal import BasebandSignal  # noqa: F401
