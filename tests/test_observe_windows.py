"""Host side of observe()'s fused resampled copy (PssPipeline.out_len):
the rebin window edges (utils.py:71-91) computed elementwise must equal the
reference's per-bin loop, and every window holding a sample n must be one of
the three candidates the device epilogue checks (pss_pipeline.hip
out_windows: floor(n / step) - 1 .. floor(n / step) + 1)."""
import numpy as np
import pytest

from psrsigsim_amd.utils.utils import rebin_edges


def _loop_edges(size, newlen):
    # the reference's loop (utils.py:77-89), restated for the check
    new_bins = np.linspace(0, size, newlen, endpoint=False)
    stride = new_bins[1] - new_bins[0]
    lo, hi = [], []
    for lbin in new_bins:
        rbin = int(np.ceil(lbin + stride))
        if rbin > size:
            rbin = size
        lo.append(int(np.ceil(lbin)))
        hi.append(rbin)
    return np.array(lo), np.array(hi), stride


@pytest.mark.parametrize("size,newlen", [(8192, 1097), (1 << 20, 143640), (30720, 4096), (1000, 3),
                                         (3125000, 99999), (4096, 4096), (16384, 2241)])
def test_rebin_edges_match_loop_and_candidates(size, newlen):
    lo, hi = rebin_edges(size, newlen)
    rlo, rhi, step = _loop_edges(size, newlen)
    np.testing.assert_array_equal(lo, rlo)
    np.testing.assert_array_equal(hi, rhi)
    # every (sample, window) membership lies within the device's candidates
    n = np.arange(size)
    c = np.floor(n / step).astype(np.int64)
    covered = np.zeros(size, dtype=np.int64)
    for j in range(newlen):
        m = np.arange(lo[j], hi[j])
        assert np.all((j >= c[m] - 1) & (j <= c[m] + 1)), j
        covered[m] += 1
    assert covered.max() <= 2
