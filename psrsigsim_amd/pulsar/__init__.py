from .pulsar import Pulsar  # noqa: F401
from .profiles import PulseProfile, GaussProfile, UserProfile, DataProfile  # noqa: F401
from .portraits import PulsePortrait, GaussPortrait, UserPortrait, DataPortrait  # noqa: F401
