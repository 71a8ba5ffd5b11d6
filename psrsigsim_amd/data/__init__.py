"""Data files the reference ships and the BASELINE configs use.

* ``J1713+0747_profile.npy`` -- the reference's packaged 2048-bin J1713+0747
  profile (``psrsigsim/data/J1713+0747_profile.npy``; config C2's DataProfile).
* ``data/B1855+09.L-wide.PUPPI.11y.x.sum.sm`` (repository root, as in the
  reference's ``data/``) -- the PSRFITS template of config C4, read by
  :func:`psrsigsim_amd.io.psrfits.read_template`.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
B1855_TEMPLATE = os.path.join(ROOT, "data", "B1855+09.L-wide.PUPPI.11y.x.sum.sm")

__all__ = ["j1713_profile", "B1855_TEMPLATE"]


def j1713_profile():
    """float64 (2048,) J1713+0747 profile (plain .npy, no pickle)."""
    return np.load(os.path.join(HERE, "J1713+0747_profile.npy"), allow_pickle=False)
