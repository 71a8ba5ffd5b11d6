from .telescope import Telescope, GBT, Arecibo  # noqa: F401
from .receiver import Receiver, response_from_data  # noqa: F401
from .backend import Backend  # noqa: F401
from . import telescope  # noqa: F401
