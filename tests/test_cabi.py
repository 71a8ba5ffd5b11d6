"""CPU-side checks of the C ABI: the library loads, exports every function
include/pss_hip.h declares, and ctypes' PssPipeline has exactly the C layout
(offsets compared against a gcc build of the header)."""
import ctypes
import os
import re
import subprocess

import pytest

from psrsigsim_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "pss_hip.h")


def header_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pss_\w+)\s*\(", txt)))


def test_library_loads_and_exports_everything():
    L = _lib.load()
    names = header_functions()
    assert "pss_run" in names and len(names) >= 9
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib.EXPORTS, n
    assert L.pss_version() >= 100


def test_library_built_from_these_sources():
    """The binary that tests and benchmarks load is the one built from HEAD's
    sources: its embedded sha256 equals the hash of the sources in the tree
    (psrsigsim_amd/build.py; content, not mtimes)."""
    from psrsigsim_amd import build
    L = _lib.load()
    assert L.pss_build_hash().decode() == "PSS_BUILD_HASH=" + build.source_hash()
    assert build.embedded_hash() == build.source_hash()
    assert not build.stale()


def test_workspace_sizes():
    L = _lib.load()
    # [spill area, 256-B aligned regions][null mask row: nsamp floats]
    n = 1 << 20
    # pair mode: Yd ((nchan+2)//2 pairs, parity-aligned) + mask-table build (Mspec,
    # 6 node pair spills, 12 node rows, table bits/base, worst-case 16-float records,
    # misc) + per-channel null bits + row-pass pair ramp factors (2 x 64
    # complex per pair) + the null fix-up's word list (N/32 u32) + mask row -- no
    # per-channel mask spill
    table = n * 8 + 6 * n * 8 + 12 * n * 4 + (n // 32) * 8 + (n // 32) * 4 + n * 16 * 4 + 256
    wl = (n // 32) * 4
    pc = n * 4      # (round 6) the shared-profile pass A's per-run sample table
    assert L.pss_workspace_bytes(4, n) == 3 * n * 8 + table + 4 * n // 8 + 3 * 1024 + wl + pc + n * 4
    assert L.pss_workspace_bytes(3, n) == 2 * n * 8 + table + 3 * n // 8 + 2 * 1024 + wl + pc + n * 4
    a = lambda b: ((b + 255) // 256) * 256
    # even N <= 2^17 on the fallback paths: + the float64 null decisions'
    # e^{2 pi i n/N} [N] and box spectrum [N/2 + 1] (double2), row maxima [nchan]
    # (+ round 5: the box spectrum's 16 partial sums and the refine
    # candidate list -- 1/8 of the samples + 64 Ki entries of 8 B -- and its count)
    f64 = lambda n, nc: (a(n * 16) + a((n // 2 + 1) * 16) + a(nc * 4) + a(16 * (n // 2 + 1) * 16)
                         + a(min(nc * n, nc * n // 8 + 65536) * 8) + 256)
    # single-workgroup lengths (round 6): W1 [nchan][N] for the float64 null
    # refine of a delayed null, its buffers, the mask row
    assert L.pss_workspace_bytes(4, 4096) == a(4 * 4096 * 8) + f64(4096, 4) + 4096 * 4
    sp = 2 * 2 * 244 * 8 + 244 * 8                                   # fallback W1, W2, twiddles
    assert L.pss_workspace_bytes(2, 244) == a(sp) + f64(244, 2) + 1024   # row: 976 B, aligned
    # Bluestein fallback (N > 8192, 2 x 5003): W1 only (forward and inverse
    # DFT fused through Z) | chirp [N] | Bhat [M = 32768] | one batch row [M]
    # (nb = max(1, nchan N / M)) | mask row
    n = 10006
    assert L.pss_workspace_bytes(2, n) == a(2 * n * 8) + f64(n, 2) + a(n * 8) + 2 * a(32768 * 8) + a(n * 4)
    # 8 x (2^20 - 2): M = 2^21, nb = ceil(8 (2^20 - 2) / 2^21) = 4 (round 5:
    # ceil, so the last batch is not a near-empty one)
    n = (1 << 20) - 2
    M = 1 << 21
    assert L.pss_workspace_bytes(8, n) == a(8 * n * 8) + a(n * 8) + a(M * 8) + a(4 * M * 8) + a(n * 4)
    # the forced direct DFT keeps W1, W2 and the twiddles
    old = L.pss_set_flags(_lib.FLAG_DIRECT_DFT)
    try:
        n = 10006
        assert L.pss_workspace_bytes(2, n) == a(5 * n * 8) + f64(n, 2) + a(n * 8) + 2 * a(32768 * 8) + a(n * 4)
    finally:
        L.pss_set_flags(old)


def test_struct_layout_matches_header(tmp_path):
    fields = [f for f, _ in _lib.PssPipeline._fields_]
    src = ['#include <stdio.h>', '#include <stddef.h>', '#include "pss_hip.h"', 'int main(void){',
           'printf("%zu\\n", sizeof(PssPipeline));']
    src += ['printf("%%zu\\n", offsetof(PssPipeline, %s));' % f for f in fields]
    src += ['return 0;}']
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I" + os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(_lib.PssPipeline)
    for f, off in zip(fields, vals[1:]):
        assert getattr(_lib.PssPipeline, f).offset == off, f


def test_error_mapping():
    with pytest.raises(ValueError):
        _lib.check(_lib.PSS_EINVAL)
    with pytest.raises(NotImplementedError):
        _lib.check(_lib.PSS_EUNSUPPORTED)
    with pytest.raises(RuntimeError):
        _lib.check(_lib.PSS_EHIP)


def test_fold_rejects_out_of_row_geometry():
    """pss_fold validates its geometry at the C ABI (no GPU touched): the
    npbins + n_fold * npbins/2 samples it sums must lie inside the row."""
    L = _lib.load()
    assert L.pss_fold(None, None, 2, 100, 64, 3, None) == _lib.PSS_EINVAL     # 64 + 3*32 > 100
    assert L.pss_fold(None, None, 2, 100, 1, 3, None) == _lib.PSS_EINVAL      # npbins < 2
    assert L.pss_fold(None, None, 0, 100, 64, 1, None) == _lib.PSS_EINVAL     # no rows
    L.pss_fold(None, None, 2, 100, 64, 3, None)
    assert "exceed the row" in _lib.last_error()


def test_aux_entry_points_validate_arguments():
    """The resampling / cast / draw entry points reject NULL buffers and rows
    shorter than the data before any launch (no GPU touched)."""
    import ctypes
    L = _lib.load()
    host = (ctypes.c_float * 16)()
    p = ctypes.cast(host, ctypes.c_void_p)
    assert L.pss_down_sample(None, None, 2, 100, 100, 2, None) == _lib.PSS_EINVAL
    assert L.pss_down_sample(p, p, 2, 100, 50, 2, None) == _lib.PSS_EINVAL          # in_ld < in_len
    assert "in_ld < in_len" in _lib.last_error()
    assert L.pss_down_sample(p, p, 2, 100, 100, 3, None) == _lib.PSS_EINVAL         # 3 does not divide 100
    assert L.pss_rebin(None, None, 2, 100, 100, 10, None, None, None) == _lib.PSS_EINVAL
    assert L.pss_rebin(p, p, 2, 100, 50, 10, p, p, None) == _lib.PSS_EINVAL         # in_ld < in_len
    assert L.pss_clip_cast(None, None, 10, 200.0, _lib.OUT_F32, None) == _lib.PSS_EINVAL
    assert L.pss_chi2_fill(None, 2, 0, 16, 1.0, 1, 0, 0, None) == _lib.PSS_EINVAL
    assert L.pss_fold_periods(None, None, 2, 100, 10, 5, None) == _lib.PSS_EINVAL
