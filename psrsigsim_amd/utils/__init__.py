from .utils import make_quant, shift_t, down_sample, rebin, top_hat_width, make_par  # noqa: F401
from . import constants  # noqa: F401
