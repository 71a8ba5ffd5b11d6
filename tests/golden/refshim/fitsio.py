"""TEST-ONLY inert stand-in: fitsio is imported by psrsigsim.io, never used on the synthesis path."""
