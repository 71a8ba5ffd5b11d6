"""Split-cell device tables of portraits on NON-uniform phases
(DataPortrait.split_table): evaluated the way the kernels do (cell, u,
right cubic when u >= split), they reproduce the float64 piecewise cubic the
reference evaluates (PchipInterpolator over those knots) to fp32 rounding.
CPU only."""
import numpy as np
import pytest

from psrsigsim_amd.pulsar.portraits import DataPortrait, ppoly_eval


def _eval(tab, M, split, ph):
    pos = ph * M
    c = np.minimum(np.floor(pos).astype(np.int64), M - 1)
    u = (pos - c).astype(np.float32)
    t = tab.astype(np.float64)
    cc = np.where((u >= split[c])[None, :, None], t[:, c, 4:], t[:, c, :4])
    u = u.astype(np.float64)
    return ((cc[..., 0] * u + cc[..., 1]) * u + cc[..., 2]) * u + cc[..., 3]


@pytest.mark.parametrize("n,power,rows", [(96, 1.3, 1), (40, 0.7, 3), (300, 1.05, 2)])
def test_split_table_matches_pchip(n, power, rows):
    rng = np.random.default_rng(n)
    ph = (np.arange(n) / n) ** power
    vals = np.exp(-0.5 * ((ph - 0.45) / 0.05) ** 2)[None] * (1.0 + 0.1 * rng.random((rows, 1)))
    port = DataPortrait(vals, phases=ph)
    port.init_profiles(256, Nchan=rows)
    tab, M, third = port.device_table()
    assert np.ndim(third) == 1 and tab.shape == (rows, M, 8) and third.shape == (M,)
    x = np.sort(np.concatenate([rng.random(20000), ph, np.array([0.0])]))
    x = x[x < 1.0]
    got = _eval(tab, M, third, x)
    want = ppoly_eval(port._knots, port._coef, x) / port.Amax
    assert np.max(np.abs(got - want)) <= 2e-6 * np.max(np.abs(want))


def test_uniform_phases_keep_the_plain_table():
    n = 64
    port = DataPortrait(np.exp(-0.5 * ((np.arange(n) / n - 0.5) / 0.05) ** 2)[None], phases=np.arange(n) / n)
    port.init_profiles(128, Nchan=1)
    tab, M, nint = port.device_table()
    assert np.ndim(nint) == 0 and tab.shape[-1] == 4
