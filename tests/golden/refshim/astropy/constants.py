"""TEST-ONLY: astropy.constants stand-in (the reference imports it but the
filterbank path uses none of it)."""
