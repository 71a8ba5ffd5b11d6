"""Deferred, fused execution of the synthesis path on the GPU.

The reference mutates ``signal._data`` eagerly, one NumPy pass per call
(make_pulses, each shift_t loop, null, noise).  Here every call records a
*stage* on the signal's pending pipeline; the pipeline is executed -- as ONE
fused run of the HIP engine (pss_run) -- when the data is needed
(``signal.data``), when the next call cannot be appended (e.g. a delay after
noise), or by Telescope.observe.  Stage order is the reference's:

    source (make_pulses | existing data) -> delay stages* -> null -> noise

Results are identical to running the stages one by one: several delay stages
compose into a single ramp (phase = sum of delays, Nyquist factor = product of
the per-stage cos(pi s)), and the delayed-null mask rides through the same FFT
as the imaginary part of the transformed row.

Randomness: counter-based Philox keyed by (seed, call id, purpose, GLOBAL
channel, sample) -- see ``seed()``; exact replay of the reference's own draws
is available through ``inject()`` (tests).
"""
import ctypes
import os
import threading

import numpy as np
import torch

from . import _lib

# ---------------------------------------------------------------------------
# randomness
# ---------------------------------------------------------------------------
_state = {"seed": 0x5EED1776, "calls": 0}
_lock = threading.Lock()


def seed(s):
    """Seed the engine's Philox streams (the analogue of ``np.random.seed``).
    Resets the call counter so a seeded sequence of calls is reproducible."""
    with _lock:
        _state["seed"] = int(s) & 0xFFFFFFFFFFFFFFFF
        _state["calls"] = 0


def next_call():
    with _lock:
        _state["calls"] += 1
        return _state["calls"] & 0x0FFFFFFF


def host_rng(call_id):
    """numpy Generator for small host-side draws (null pulse choice), keyed
    like the device streams so every shard makes the same choice."""
    return np.random.Generator(np.random.Philox(key=[_state["seed"], call_id]))


# exact mode: draws to use instead of Philox, consumed by the next pipeline
# stage of that kind (tests replay the reference's recorded draws).
_inject = {}


def inject(**kw):
    """inject(gen=, box=, rep=, noise=, null_pulses=) -- host arrays (global
    channel x sample, or one row for `box`) used by the next stage of that
    kind instead of Philox draws."""
    for k, v in kw.items():
        if k not in ("gen", "box", "rep", "noise", "null_pulses"):
            raise KeyError(k)
        _inject[k] = v


class InjectedRowsMissing(KeyError):
    """Injected draws (a RowBlock) that do not cover the requested channels."""


class RowBlock(object):
    """Injected per-channel draws for global channels [c0, c0 + len(arr)) only
    (a shard's rows), instead of a full [Nchan, N] array."""

    def __init__(self, c0, arr):
        self.c0 = int(c0)
        self.arr = arr


def inj_rows(inj, gidx):
    """Rows ``gidx`` (global channel indices) of an injected draw array."""
    if isinstance(inj, RowBlock):
        rel = np.asarray(gidx) - inj.c0
        if rel.size and (rel.min() < 0 or rel.max() >= len(inj.arr)):
            raise InjectedRowsMissing("injected rows cover channels [%d, %d), not %s"
                           % (inj.c0, inj.c0 + len(inj.arr), list(np.asarray(gidx))))
        return np.asarray(inj.arr, dtype=np.float32)[rel]
    return np.asarray(inj, dtype=np.float32)[gidx]


def take_injection(kind):
    return _inject.pop(kind, None)


def clear_injections():
    _inject.clear()


# ---------------------------------------------------------------------------
# device helpers
# ---------------------------------------------------------------------------
def device():
    _lib.lib()
    return torch.device("cuda", torch.cuda.current_device())


def stream_ptr():
    """The launch stream for a library call; it first waits (on the device)
    for the uploads to_dev queued since the last call -- one event per call,
    not one per table."""
    st = torch.cuda.current_stream()
    if _upload_pending:
        idx = st.device.index
        if idx in _upload_pending:
            st.wait_stream(_upload[idx])
            _upload_pending.discard(idx)
    return ctypes.c_void_p(st.cuda_stream)


_ws = {}


def workspace(nbytes, role="main"):
    """Cached per-device workspace (grown on demand, never shrunk).  The
    channel-0 probe of null() has its own (``role="probe"``) so its small run
    does not resize the main one."""
    dev = device()
    key = (dev.index, role)
    buf = _ws.get(key)
    if nbytes <= 0:
        return None
    if buf is None or buf.numel() < nbytes:
        _ws.pop(key, None)
        buf = torch.empty(int(nbytes), dtype=torch.uint8, device=dev)
        _ws[key] = buf
    return buf


def release_workspace():
    _ws.clear()


_upload = {}
_upload_pending = set()
# "stream": every upload on the upload stream; "direct": on the launch stream;
# "auto": the upload stream after a large run (>= 2^27 channel-samples: what a
# stall would wait for is long), the launch stream after a small one (C4's
# 0.5-ms steps: the cross-stream event cost more than a stall, 0.565 vs 0.503
# ms/step; 256 x 2^22: 6.83 against 7.07 direct; tools/ab_upload.py)
UPLOAD_MODE = "auto"
_UPLOAD_STREAM_MIN = 1 << 27
_last_run = [0]


def to_dev(a, dtype=None):
    """Host array -> device tensor, stream-ordered and without blocking the
    host.  From pageable memory the copy would wait for the stream to drain
    (i.e. for the previous signal's fused run), so it goes through a pinned
    staging copy (torch's caching host allocator).  And it runs on an upload
    stream of its own, the launch stream waiting for it on the device: a
    small "asynchronous" copy on the launch stream itself still blocked the
    host until that stream drained, now and then (a whole step's kernels,
    ~7 ms at 256 channels x 2^22, during which the next step's planning could
    not run -- tools/host_stalls.py, tools/r5_hiptrace.sh).  The destination
    comes from the upload stream's pool, so it never aliases memory the
    launch stream still uses, and is recorded on the launch stream before it
    returns to the pool.  The launch stream waits for the upload stream at
    the next library call (stream_ptr), once for all of a run's tables."""
    t = torch.as_tensor(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    t = t.pin_memory()
    dev = device()
    main = torch.cuda.current_stream(dev)
    if UPLOAD_MODE == "direct" or (UPLOAD_MODE == "auto" and _last_run[0] < _UPLOAD_STREAM_MIN):
        return t.to(dev, non_blocking=True)
    up = _upload.get(dev.index)
    if up is None:
        up = _upload[dev.index] = torch.cuda.Stream(dev)
    with torch.cuda.stream(up):
        d = t.to(dev, non_blocking=True)
    d.record_stream(main)
    _upload_pending.add(dev.index)
    return d


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def ramp_words(samples, N):
    """frac(s/N) * 2^64 as uint64 (bin k gets exp(-2 pi i k s / N))."""
    x = np.asarray(samples, dtype=np.float64) / float(N)
    f = x - np.floor(x)
    w = np.ldexp(f, 64)
    w = np.where(w >= 2.0 ** 64, 0.0, w)
    hi = np.floor(w / 2.0 ** 32)
    lo = w - hi * 2.0 ** 32
    return (hi.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)


def u64_to_i64_tensor(u):
    return to_dev(np.asarray(u, dtype=np.uint64).view(np.int64))


# ---------------------------------------------------------------------------
# pending pipeline
# ---------------------------------------------------------------------------
class Source(object):
    """make_pulses stage (pulsar.py:185-244).  mode 'search' evaluates the
    PCHIP table at the pulse phase of every sample; 'fold' tiles an Nph-bin
    profile table.  Tables are global over channels (prof_rows == Nchan) or
    a single shared row."""

    def __init__(self, mode, table, df, draw_norm, call_id, nph=0, M=0, nint=0,
                 phase_step=0, inj=None, row_ids=None, split=None):
        self.mode = mode
        self.table = table            # np.float32, search [rows,nint,4] / fold [rows,nph]
        # global channel of each table row when the table holds only this
        # rank's channels (shard-local planning, shard.RowSet); None: row c is
        # channel c (or one shared row)
        self.row_ids = None if (row_ids is None or table.shape[0] == 1) else np.asarray(row_ids, dtype=np.int64)
        # non-uniform portrait phases: [M] split points after the [rows, M, 8]
        # split-cell table (PssPipeline.prof_split)
        self.split = split
        self.df = float(df)
        self.draw_norm = float(draw_norm)
        self.call_id = call_id
        self.nph = int(nph)
        self.M = int(M)
        self.nint = int(nint)
        self.phase_step = int(phase_step)
        self.inj = inj                # global [Nchan, N] draws or None
        self.amp = False              # amplitude pulses (baseband): sqrt(profile) x N(0,1)


class Pending(object):
    def __init__(self, source=None):
        self.source = source          # None -> load existing data
        self.shifts = []              # list of np.float64 [Nchan_global] (samples)
        self.tail = None              # np.float64 [Nchan_global] scattering-tail a (extension)
        self.null = None              # dict
        self.noise = None             # dict
        self.out = None               # dict(kind, tensor, clip)

    def empty(self):
        return (self.source is None and not self.shifts and self.tail is None and self.null is None
                and self.noise is None and self.out is None)


def plan_pipeline(sig, pend, rows, chan0):
    """Host-side plan of one fused run over global channels [chan0, chan0+rows):
    every scalar field of PssPipeline plus the per-row numpy arrays (ramp
    words, Nyquist factors, injected draws).  Pure host code (tested on CPU)."""
    N = sig._ncols
    gidx = np.arange(chan0, chan0 + rows)
    P = {"nchan": rows, "chan0": int(chan0), "nsamp": N, "seed": _state["seed"], "arrays": {}}
    A = P["arrays"]
    src = pend.source
    if src is None:
        P["src"] = _lib.SRC_LOAD
    else:
        P.update(src=_lib.SRC_SEARCH if src.mode == "search" else _lib.SRC_FOLD,
                 prof_rows=src.table.shape[0], nint=src.nint, nph=src.nph,
                 phase_step=src.phase_step, knot_m=src.M, gen_df=src.df,
                 draw_norm=src.draw_norm, call_gen=src.call_id,
                 gen_amp=(2 if src.amp == "gauss" else 1) if src.amp else 0,
                 prof_split=1 if getattr(src, "split", None) is not None else 0)
        if src.inj is not None:
            A["inj_gen"] = inj_rows(src.inj, gidx)
    nul = pend.null
    need_fft = bool(pend.shifts) or pend.tail is not None or (nul is not None and nul["mode"] == "delayed")
    if need_fft:
        if N % 2:
            raise ValueError("could not broadcast input array from shape (%d,) into shape (%d,)"
                             % (N - 1, N))
        P["shift"] = 1
        total = np.zeros(sig.Nchan)
        nyq_re = np.ones(sig.Nchan)
        for sh in pend.shifts:
            total = total + sh
            nyq_re = nyq_re * np.cos(np.pi * sh)
        if nul is not None and nul["mode"] == "delayed":
            mask_total = nul["mask_samples"]
            nyq_im = np.cos(np.pi * mask_total)
            A["mask_ramp"] = ramp_words(mask_total[gidx], N)
            if pend.shifts or pend.tail is not None:
                P["data_in_fft"], ramp_s = 1, total
            else:
                P["data_in_fft"], ramp_s = 0, mask_total
        else:
            P["data_in_fft"], ramp_s, nyq_im = 1, total, nyq_re
        A["ramp"] = ramp_words(ramp_s[gidx], N)
        A["nyq_re"] = nyq_re[gidx].astype(np.float32)
        A["nyq_im"] = nyq_im[gidx].astype(np.float32)
        if pend.tail is not None:
            A["tail_a"] = pend.tail[gidx].astype(np.float32)
    if nul is not None:
        P.update(null_mode=_lib.NULL_DELAYED if nul["mode"] == "delayed" else _lib.NULL_UNDELAYED,
                 null_slots=int(nul["rank"].size), null_shift=int(nul.get("shift_val", 0)),
                 nph=int(nul["nph"]), null_box_df=nul["box_df"], null_box_scale=nul["box_scale"],
                 null_rep_df=nul.get("rep_df", 1.0), null_rep_scale=nul.get("rep_scale", 0.0),
                 call_null=nul["call_id"])
        A["null_rank"] = nul["rank"].astype(np.int32)
        if nul.get("inj_box") is not None:
            A["inj_box"] = np.asarray(nul["inj_box"], dtype=np.float32)
        if nul.get("inj_rep") is not None:
            A["inj_rep"] = inj_rows(nul["inj_rep"], gidx)
    noi = pend.noise
    if noi is not None:
        P.update(noise=1, noise_df=noi["df"], noise_norm=noi["norm"], call_noise=noi["call_id"])
        if noi.get("inj") is not None:
            A["inj_noise"] = inj_rows(noi["inj"], gidx)
    return P


def build_pipeline(sig, pend, rows, chan0, data, out=None, ws_role="main"):
    """A PssPipeline (plus the device buffers it points at) for local rows
    [0, rows) of ``data`` holding global channels [chan0, chan0+rows)."""
    P = plan_pipeline(sig, pend, rows, chan0)
    p = _lib.PssPipeline()
    keep = []
    for k, v in P.items():
        if k != "arrays":
            setattr(p, k, v)
    p.ld = data.stride(0)
    p.data = ptr(data)
    src = pend.source
    if src is not None:
        # rows are indexed by GLOBAL channel inside the kernel (or row 0 when
        # the table is shared); the device copy is cached on the stage.
        if getattr(src, "dev_table", None) is None:
            flat = np.ascontiguousarray(src.table, dtype=np.float32).ravel()
            if getattr(src, "split", None) is not None:
                flat = np.concatenate([flat, np.asarray(src.split, dtype=np.float32)])
            src.dev_table = to_dev(flat)
        p.prof = ptr(src.dev_table)
        if src.row_ids is not None:
            # a channel window: point at the row of global channel chan0
            i = int(np.searchsorted(src.row_ids, chan0))
            if not np.array_equal(src.row_ids[i:i + rows], np.arange(chan0, chan0 + rows)):
                raise RuntimeError("profile table holds no rows for channels [%d, %d)" % (chan0, chan0 + rows))
            p.prof = ctypes.c_void_p(src.dev_table.data_ptr() + i * int(src.table[0].size) * 4)
            p.prof_rows = src.table.shape[0] - i
            p.prof_row0 = int(chan0)
    if P["arrays"]:
        # every per-run array in ONE host->device copy (a pinned staging
        # buffer, 256-B aligned slots): each separate upload costs ~20-40 us of
        # host time (pinning, a copy launch), which the short runs of the
        # reference's own shapes (tutorial 2: 64 x 40 960) feel
        slots, off = [], 0
        for name, arr in P["arrays"].items():
            a = np.ascontiguousarray(np.asarray(arr, dtype=np.uint64).view(np.int64)
                                     if name in ("ramp", "mask_ramp") else arr)
            slots.append((name, off, a))
            off += (a.nbytes + 255) & ~255
        host = np.zeros(max(off, 256), dtype=np.uint8)
        for _, o, a in slots:
            host[o:o + a.nbytes] = a.view(np.uint8).ravel()
        t = to_dev(host)
        keep.append(t)
        base = t.data_ptr()
        for name, o, _ in slots:
            setattr(p, name, ctypes.c_void_p(base + o))
    if P.get("shift"):
        ws = workspace(_lib.load().pss_workspace_bytes(rows, sig._ncols), ws_role)
        p.work = ptr(ws) if ws is not None else None
    nul = pend.null
    if nul is not None and nul.get("shift_dev") is not None:
        p.null_shift_dev = ptr(nul["shift_dev"])
    if out is not None:
        p.out_kind = out["kind"]
        p.out = ptr(out["tensor"])
        p.clip = out["clip"]
        win = out.get("windows")
        if win is not None:
            # observe()'s resampled copy, produced by the run (PssPipeline.out_len)
            p.out_len = int(win["len"])
            p.out_lo = ptr(win["lo"])
            p.out_hi = ptr(win["hi"])
            p.out_step = float(win["step"])
            p.out_acc = ptr(win["acc"])
    return p, keep


def run(p, keep):
    rc = _lib.lib().pss_run(ctypes.byref(p), stream_ptr())
    _lib.check(rc, "pss_run")
    # (to_dev's upload-stream choice: the size of the recent runs, decaying
    # by half per smaller run, so null()'s 2-channel probe between two band
    # runs does not count as "small")
    _last_run[0] = max(int(p.nchan) * int(p.nsamp), _last_run[0] // 2)
    return keep


def execute(sig, pend):
    """Run ``pend`` over the signal's local rows (allocating the buffer when
    the source generates it) and over the shadow of global channel 0."""
    N = sig._ncols
    rows = sig._c1 - sig._c0
    if sig._buf is None or tuple(sig._buf.shape) != (rows, N):
        if pend.source is None:
            raise RuntimeError("signal has no data")
        sig._buf = torch.empty((rows, N), dtype=torch.float32, device=device())
    out = pend.out
    if (sig._c0 > 0 or sig._c1 < min(2, sig.Nchan)) and sig._track_row0:
        # shadow of global channels 0..1 (shard-invariant null()): same stages,
        # same (0, 1) channel pairing as the shard that owns channel 0
        nrow = min(2, sig.Nchan)
        if sig._row0 is None or tuple(sig._row0.shape) != (nrow, N):
            if pend.source is None:
                raise RuntimeError("channel-0 shadow lost")
            sig._row0 = torch.empty((nrow, N), dtype=torch.float32, device=device())
        try:
            p0, k0 = build_pipeline(sig, pend, nrow, 0, sig._row0)
        except InjectedRowsMissing:
            # exact mode with draws injected for this shard's rows only: no
            # shadow (a later null() on this shard then needs the draws of
            # channels 0..1, and raises without them)
            sig._row0 = None
        else:
            run(p0, k0)
    p, keep = build_pipeline(sig, pend, rows, sig._c0, sig._buf, out=out)
    run(p, keep)


def filter_rows(sig, htab):
    """rows <- irfft(rfft(row) * H) on the device for every local row of
    ``sig`` (baseband coherent dispersion, ism.py:76-98); ``htab`` is the
    complex transfer function on the N/2 + 1 rfft bins."""
    data = sig.data                                   # flushes pending stages
    rows, N = data.shape
    h = to_dev(np.ascontiguousarray(np.asarray(htab, dtype=np.complex64)).view(np.float32))
    L = _lib.load()
    ws = workspace(L.pss_filter_workspace_bytes(rows, N))
    rc = _lib.lib().pss_filter_rows(ptr(data), rows, N, data.stride(0), ptr(h), ptr(ws), stream_ptr())
    _lib.check(rc, "filter_rows")


def null_shift_device(sig, pend, count):
    """Pulsar.null's shift_val (pulsar.py:285-288: count//2 - argmax of the
    first ``count`` samples of GLOBAL channel 0 after ``pend``, without
    noise) computed on the device, stream-ordered, with no host round trip:
    returns a device int64 tensor [shift_val, status] (pss_null_shift) that
    the fused run reads through PssPipeline.null_shift_dev.  Channel 0 is
    replayed for global channels 0..1 (the pairing the full run uses, so the
    values are bit-identical to the final channel 0) from the source when it
    is generated, else taken from the local buffer or the channel-0 shadow --
    on any shard, without communication."""
    N = sig._ncols
    nrow = min(2, sig.Nchan)
    if sig._c0 == 0 and sig._c1 >= nrow and sig._buf is not None:
        base = sig._buf[0:nrow]
    else:
        base = sig._row0
    if pend.empty():
        if base is None:
            raise RuntimeError("no data for channel 0")
        row = base[0]
    else:
        scratch = torch.empty((nrow, N), dtype=torch.float32, device=device())
        if pend.source is None:
            if base is None:
                raise RuntimeError("no data for channel 0")
            scratch.copy_(base)
        probe = Pending(pend.source)
        probe.shifts = list(pend.shifts)
        probe.tail = pend.tail
        probe.null = pend.null
        p, keep = build_pipeline(sig, probe, nrow, 0, scratch, ws_role="probe")
        run(p, keep)
        row = scratch[0]
    out = torch.empty(2, dtype=torch.int64, device=device())
    rc = _lib.lib().pss_null_shift(ptr(row), int(count), ptr(out), stream_ptr())
    _lib.check(rc, "null_shift")
    return out


def check_null_status(sig):
    """Raise the reference's error for a null() whose channel-0 maximum was
    not unique (pulsar.py:286-288: the broadcast of a shift_val of size != 1
    fails).  Deferred to the first read of the data: the value is on the
    device, and reading it at null() time would stall the host.  A failed
    check is sticky: the data then holds a null the reference never made, so
    every later read-out raises the same error (not only the first)."""
    err = getattr(sig, "_null_error", None)
    if err is not None:
        raise ValueError(err)
    checks = getattr(sig, "_null_checks", None)
    if not checks:
        return
    sig._null_checks = []
    for t, nph in checks:
        st = int(t[1].item())
        if st != 0:
            sig._null_error = ("operands could not be broadcast together with shapes (%d,) (%s,)"
                               % (nph, "0" if st == 2 else "2+"))
            raise ValueError(sig._null_error)


