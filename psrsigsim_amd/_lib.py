"""ctypes binding of libpss_hip.so (include/pss_hip.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU
is visible, every compute call raises.  ``lib()`` loads the in-tree build
(``psrsigsim_amd/libpss_hip.so``, produced by ``__graft_entry__.build()`` /
``psrsigsim_amd/build.py``).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PSS_LIB_PATH") or os.path.join(_HERE, "libpss_hip.so")

PSS_OK, PSS_EINVAL, PSS_EUNSUPPORTED, PSS_EHIP = 0, -1, -2, -3
SRC_LOAD, SRC_SEARCH, SRC_FOLD = 0, 1, 2
NULL_NONE, NULL_UNDELAYED, NULL_DELAYED = 0, 1, 2
OUT_NONE, OUT_F32, OUT_I8 = 0, 1, 2
FLAG_NO_FAST = 1
FLAG_DIRECT_DFT = 2
FLAG_NULL_F32 = 4
FLAG_REFINE_PER_SAMPLE = 8
P_PULSE, P_BOX, P_REP, P_NOISE, P_TEST = 1, 2, 3, 4, 5
KERNEL_KINDS = ("elementwise", "single_pass", "fourstep_colA", "fourstep_row", "fourstep_colC",
                "fallback_dft", "null_fix")

c_i32, c_i64, c_u32, c_u64, c_f32, c_vp = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                                           ctypes.c_uint64, ctypes.c_float, ctypes.c_void_p)


class PssPipeline(ctypes.Structure):
    """Mirror of ``struct PssPipeline`` (include/pss_hip.h); field order and
    types must match exactly (checked by tests/test_cabi.py)."""
    _fields_ = [
        ("nchan", c_i32), ("chan0", c_i32), ("nsamp", c_i64), ("ld", c_i64),
        ("data", c_vp), ("work", c_vp),
        ("src", c_i32), ("prof_rows", c_i32), ("prof", c_vp), ("nint", c_i32), ("nph", c_i32),
        ("phase_step", c_u64), ("knot_m", c_u32), ("gen_df", c_f32), ("draw_norm", c_f32),
        ("shift", c_i32), ("data_in_fft", c_i32), ("ramp", c_vp), ("nyq_re", c_vp), ("nyq_im", c_vp),
        ("null_mode", c_i32), ("null_slots", c_i32), ("null_rank", c_vp), ("null_shift", c_i64),
        ("null_box_df", c_f32), ("null_box_scale", c_f32), ("null_rep_df", c_f32),
        ("null_rep_scale", c_f32),
        ("noise", c_i32), ("noise_df", c_f32), ("noise_norm", c_f32),
        ("out_kind", c_i32), ("out", c_vp), ("clip", c_f32),
        ("seed", c_u64), ("call_gen", c_u32), ("call_null", c_u32), ("call_noise", c_u32),
        ("inj_gen", c_vp), ("inj_box", c_vp), ("inj_rep", c_vp), ("inj_noise", c_vp),
        ("mask_ramp", c_vp),
        ("gen_amp", c_i32), ("prof_row0", c_i32), ("htab", c_vp), ("null_shift_dev", c_vp),
        ("tail_a", c_vp), ("prof_split", c_i32), ("out_len", c_i32), ("out_lo", c_vp), ("out_hi", c_vp),
        ("out_step", ctypes.c_double), ("out_acc", c_vp),
    ]


EXPORTS = {
    "pss_version": (ctypes.c_int, []),
    "pss_build_hash": (ctypes.c_char_p, []),
    "pss_set_flags": (ctypes.c_int, [ctypes.c_int]),
    "pss_last_error": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "pss_plan_collect": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "pss_workspace_bytes": (c_i64, [c_i32, c_i64]),
    "pss_timing_enable": (None, [ctypes.c_int]),
    "pss_timing_span_ms": (ctypes.c_double, []),
    "pss_timing_collect": (ctypes.c_int, [ctypes.POINTER(c_i32), ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(c_i64), ctypes.c_int]),
    "pss_run": (ctypes.c_int, [ctypes.POINTER(PssPipeline), c_vp]),
    "pss_shift_rows": (ctypes.c_int, [c_vp, c_i32, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "pss_filter_workspace_bytes": (c_i64, [c_i32, c_i64]),
    "pss_filter_rows": (ctypes.c_int, [c_vp, c_i32, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "pss_down_sample": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i64, c_i64, c_i32, c_vp]),
    "pss_rebin": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp]),
    "pss_clip_cast": (ctypes.c_int, [c_vp, c_vp, c_i64, c_f32, c_i32, c_vp]),
    "pss_fold": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i64, c_i64, c_i64, c_vp]),
    "pss_fold_periods": (ctypes.c_int, [c_vp, c_vp, c_i32, c_i64, c_i64, c_i64, c_vp]),
    "pss_null_shift": (ctypes.c_int, [c_vp, c_i64, c_vp, c_vp]),
    "pss_chi2_fill": (ctypes.c_int, [c_vp, c_i32, c_i32, c_i64, c_f32, c_u64, c_u32, c_u32, c_vp]),
    "pss_host_pchip_coef": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, ctypes.c_int]),
    "pss_host_ppoly_eval": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, ctypes.c_int]),
    "pss_host_pchip_eval": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, ctypes.c_double, c_vp,
                                           ctypes.c_int]),
    "pss_host_pchip_table": (ctypes.c_int, [c_vp, c_i64, c_vp, c_i64, ctypes.c_double, ctypes.c_double, c_vp,
                                            ctypes.c_int]),
    "pss_host_device_table": (ctypes.c_int, [c_vp, c_i64, c_i64, ctypes.c_double, ctypes.c_double,
                                             c_vp, ctypes.c_int]),
}

_LIB = None


class HipUnavailable(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load the shared library and declare every export (no GPU needed)."""
    global _LIB
    if _LIB is not None and path == LIB_PATH:
        return _LIB
    if not os.path.exists(path):
        raise HipUnavailable("libpss_hip.so not built at %s -- run `python -c 'import "
                             "__graft_entry__ as g; g.build()'`" % path)
    if path == LIB_PATH and not os.environ.get("PSS_LIB_PATH"):
        check_build_hash(path)
    L = ctypes.CDLL(path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if path == LIB_PATH:
        _LIB = L
    return L


def check_build_hash(path=LIB_PATH):
    """Refuse a library that was not built from the sources in this tree
    (the hash psrsigsim_amd/build.py compiles into it)."""
    from . import build as _b
    try:
        want = _b.source_hash()
        want_debug = _b.source_hash(["-DPSS_DEBUG=1"])   # the device-assert build (build --debug)
    except OSError:
        return          # sources not shipped: nothing to compare against
    got = _b.embedded_hash(path)
    if got not in (want, want_debug):
        raise HipUnavailable("%s was built from other sources (hash %s, tree %s) -- rebuild with "
                             "psrsigsim_amd/build.py" % (path, got, want))


def lib():
    """The library, for compute: also requires a visible HIP device."""
    L = load()
    import torch
    if not torch.cuda.is_available():
        raise HipUnavailable("psrsigsim_amd computes on an MI355X (HIP) device; none is visible")
    return L


def timing_collect(cap=4096):
    """[(kind_name, ms, channel_samples)] of the launches timed since enable."""
    k = (c_i32 * cap)()
    ms = (ctypes.c_double * cap)()
    u = (c_i64 * cap)()
    n = load().pss_timing_collect(k, ms, u, cap)
    return [(KERNEL_KINDS[k[i]], ms[i], u[i]) for i in range(n)]


def plan_collect():
    """The launch-plan lines of the pss_run calls since the last collect
    (pss_plan_collect: which kernels each run picked), and clear them."""
    buf = ctypes.create_string_buffer(16384)
    load().pss_plan_collect(buf, 16384)
    return [l for l in buf.value.decode(errors="replace").split("\n") if l]


def last_error():
    buf = ctypes.create_string_buffer(512)
    load().pss_last_error(buf, 512)
    return buf.value.decode(errors="replace")


def check(rc, what=""):
    if rc == PSS_OK:
        return
    msg = "%s: %s" % (what, last_error()) if what else last_error()
    if rc == PSS_EINVAL:
        raise ValueError(msg)
    if rc == PSS_EUNSUPPORTED:
        raise NotImplementedError(msg)
    raise RuntimeError(msg)


# ---------------------------------------------------------------------------
# native host planning (pss_host_*): float64 tables, bitwise equal to NumPy
# ---------------------------------------------------------------------------
def _tune_host_malloc():
    """Keep glibc from returning the planning tables' memory to the kernel
    between signals: (Nchan x Nph) float64 tables are 4-16 MB, above glibc's
    default mmap threshold, so every fresh table paid ~4k page faults (zeroing)
    -- most of the per-signal host planning time.  Heap-allocate up to 32 MB
    and trim only above 512 MB of free heap."""
    try:
        libc = ctypes.CDLL("libc.so.6")
        M_TRIM_THRESHOLD, M_MMAP_THRESHOLD = -1, -3
        libc.mallopt(M_MMAP_THRESHOLD, 32 << 20)
        libc.mallopt(M_TRIM_THRESHOLD, 512 << 20)
    except OSError:
        pass


if os.environ.get("PSS_NO_MALLOPT") is None:
    _tune_host_malloc()


_HOST_THREADS = []


def host_threads():
    if not _HOST_THREADS:
        n = os.environ.get("PSS_HOST_THREADS")
        _HOST_THREADS.append(max(1, int(n)) if n else max(1, min(8, os.cpu_count() or 1)))
    return _HOST_THREADS[0]


_POOL = []


def host_rows(rows, fn, min_rows=128):
    """fn(a, b) over row blocks [a, b) of ``rows`` rows on host_threads()
    threads (numpy / pocketfft release the GIL in their array loops); the
    blocks are disjoint, so the result does not depend on the split."""
    nt = min(host_threads(), max(1, rows // min_rows))
    if nt <= 1:
        fn(0, rows)
        return
    if not _POOL:
        from concurrent.futures import ThreadPoolExecutor
        _POOL.append(ThreadPoolExecutor(max_workers=host_threads(), thread_name_prefix="pss-plan"))
    futs = [_POOL[0].submit(fn, rows * t // nt, rows * (t + 1) // nt) for t in range(nt)]
    for f in futs:
        f.result()


def _dptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def host_pchip_coef(x, y):
    import numpy as np
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    rows, K = y.shape
    c = np.empty((rows, K - 1, 4))
    check(load().pss_host_pchip_coef(_dptr(x), K, _dptr(y), rows, _dptr(c), host_threads()),
          "pss_host_pchip_coef")
    return c


def host_ppoly_eval(x, c, ph):
    import numpy as np
    x = np.ascontiguousarray(x, dtype=np.float64)
    c = np.ascontiguousarray(c, dtype=np.float64)
    ph = np.ascontiguousarray(ph, dtype=np.float64).ravel()
    out = np.empty((c.shape[0], ph.size))
    check(load().pss_host_ppoly_eval(_dptr(x), x.size, _dptr(c), c.shape[0], _dptr(ph), ph.size,
                                     _dptr(out), host_threads()), "pss_host_ppoly_eval")
    return out


def host_pchip_eval(x, y, ph, div=1.0):
    """pchip_coefficients then ppoly_eval (then / div), fused per row."""
    import numpy as np
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    ph = np.ascontiguousarray(ph, dtype=np.float64).ravel()
    out = np.empty((y.shape[0], ph.size))
    check(load().pss_host_pchip_eval(_dptr(x), x.size, _dptr(y), y.shape[0], _dptr(ph), ph.size, float(div),
                                     _dptr(out), host_threads()), "pss_host_pchip_eval")
    return out


def host_pchip_table(x, y, h, amax, width=None):
    """pchip_coefficients then host_device_table, fused per row.  ``width``
    (> K - 1, one row): the table is allocated with that many intervals and
    the first K - 1 filled (the caller completes the rest in place)."""
    import numpy as np
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    n = x.size - 1
    if width is not None and width > n and y.shape[0] == 1:
        buf = np.empty((1, width, 4), dtype=np.float32)
        out = buf[:, :n]                   # (one row: contiguous)
    else:
        buf = out = np.empty((y.shape[0], n, 4), dtype=np.float32)
    check(load().pss_host_pchip_table(_dptr(x), x.size, _dptr(y), y.shape[0], float(h), float(amax),
                                      _dptr(out), host_threads()), "pss_host_pchip_table")
    return buf


def host_device_table(c, h, amax):
    import numpy as np
    c = np.ascontiguousarray(c, dtype=np.float64)
    out = np.empty(c.shape, dtype=np.float32)
    check(load().pss_host_device_table(_dptr(c), c.shape[0], c.shape[1], float(h), float(amax),
                                       _dptr(out), host_threads()), "pss_host_device_table")
    return out
