"""constants -- mirrors ``psrsigsim/utils/constants.py``."""
from .._units import Quantity

# PSRCHIVE-consistent dispersion constant (constants.py:13): 1/2.41e-4
DM_K_VALUE = 1.0 / 2.41e-4                       # MHz^2 s cm^3 / pc
DM_K = Quantity(DM_K_VALUE, 'MHz^2*s*cm^3/pc')
KOLMOGOROV_BETA = 11.0 / 3                       # (constants.py:16)
