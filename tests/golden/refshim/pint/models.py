"""TEST-ONLY inert stand-in: PINT is imported by the reference at module import time but is not used on the filterbank path."""
