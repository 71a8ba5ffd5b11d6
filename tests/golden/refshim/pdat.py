"""TEST-ONLY inert stand-in: pdat is imported by psrsigsim.io, never used on the synthesis path."""
