from .txtfile import TxtFile  # noqa: F401
from .psrfits import PSRFITS, read_psrfits  # noqa: F401
