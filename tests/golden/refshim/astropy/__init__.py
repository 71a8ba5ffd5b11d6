"""TEST-ONLY stand-in for the tiny subset of astropy that PsrSigSim's filterbank
path touches.  It exists so that tests/golden/make_golden.py can import the
unmodified reference in the survey container (astropy is not installed there)
and record golden vectors.  Nothing in psrsigsim_amd imports this package and it
never travels with the product; see DESIGN.md "Oracle"."""
from . import units  # noqa: F401
from . import log  # noqa: F401
from . import constants  # noqa: F401
