"""Replay the golden cases (tests/golden/make_golden.py) through
psrsigsim_amd on the GPU with the reference's own recorded draws injected,
and compare every stage with the reference outputs stored in the fixtures.

A case is a small script of API calls; the same script is interpreted by the
CPU oracle (to derive the injected box / replacement rows and the null
bookkeeping) and by the product.  ``fused=True`` reads the data only at the
end (every stage runs inside one fused device run where possible);
``fused=False`` reads ``signal.data`` after every call (each stage flushed on
its own).  Returns {stage: normwise error} with the error defined per channel
as max|gpu - ref| / max|ref| (SURVEY.md §8(d) parity gate, 1e-5).
"""
import os

import numpy as np

from oracle import pss_cpu as O
from tests.fixtures_util import load

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fixtures")
AMBIG = 1e-3   # |shifted null mask - 1| below which the threshold decision is fp32-ambiguous
# ... or, at least, the fp32 tolerance (1e-5, north_star) of the transform that
# carries the mask: paths that pack the mask with the channel's data in one
# complex row (direct / Bluestein) have an error relative to the larger of the
# two (a fold-mode channel peaks at ~5000 against a ~120 mask)
AMBIG_REL = 1e-5
# Four-step lengths (N = 2^m >= 2^14) decide the threshold from the mask
# table, whose fp32 error is relative to the mask alone (its Chebyshev
# interpolant and node FFTs), not to the channel's data: band 2e-6 x the mask
# scale (+ AMBIG absolute).
AMBIG_REL_TABLE = 2e-6
# The exclusion may only hide a small, bounded set: the fraction of the
# compared samples inside the ambiguity band is bounded per path (the packed
# direct / Bluestein rows of fold-mode signals, whose data peak at ~10^4 next
# to a threshold of 1, have a wide band: ~2 % measured at config C4), and of
# those at most TOL (as a fraction of all samples) may actually come out on
# the other side of the threshold (FLIP_MAX_FRAC; both reported in STATS).
# (Round 3 measured the alternative of transforming the mask alone on these
# paths, tools/null_band.py, profiles/r03/nullband/: fold-mode boxes are
# chi2(Nfold ~ 1e4) values themselves, so the band relative to the mask is
# the same 1.9 % and the flips went 4.9e-5 -> 9.8e-5 (Gaussian portrait) and
# 1.1e-4 -> 1.6e-5 (B1855 template): the ambiguity is the fp32 transform's
# ~2e-6 relative error on a row of ~1e4 values thresholded at 1, not the
# packing -- kept packed.)
# Packed lengths whose decisions the device re-evaluates in float64
# (`k_null_refine`: even N <= 2^17 on the direct / Bluestein paths and, since
# round 6, the single-workgroup 2^m <= 8192 kernel; no scattering tail): what is left
# is the rounding of the fp32 box values the device starts from, <= 6e-8 x
# sum_j |box_j K(n - j)| (K the shift's interpolation kernel, L1 norm ~5 at
# these N): band 5e-7 x the mask scale (+ AMBIG absolute).
AMBIG_REL_P64 = 5e-7
REFINE_MAX_N = 1 << 17
REFINED = True      # False while the device runs with PSS_FLAG_NULL_F32 (tools)


def packed64(n, case):
    """Mirrors the device dispatch (pss_run / refine_null): every even N <=
    2^17 off the mask-table four-step (2^m >= 2^14) is decided in float64 --
    the single-workgroup kernel's 2^m <= 8192 (round 6) and N = 2 .. 32
    (direct DFT) included -- unless a scattering tail rides on the transform."""
    pow2 = n & (n - 1) == 0
    return (REFINED and n % 2 == 0 and n <= REFINE_MAX_N and not (pow2 and n >= 16384)
            and not any(op[0] == "scatter_tail" for op in case["ops"]))


# "packed": the float64-decided packed lengths (C4's fold-mode geometry with a
# delayed null: band 9.3e-4, no flips, against 1.9 % and up to 1.1e-4 flipped
# with the fp32 decisions, tools/null_band_r4.py, profiles/r04/null_band.txt);
# "packed_f32": the packed lengths the device still decides in fp32 (N >
# 2^17 off the four-step, the scattering tail; until round 6 also the
# single-workgroup 2^m <= 8192 kernel) -- on
# the search-mode cases that reach them (golden northstar_mini: 8192 samples;
# Bluestein 100002) the measured band is 3.05e-5 / 3.5e-5 with no flip
# (profiles/r04/null_band.txt), so the bounds sit ~10x above that (VERDICT r04
# item 3; they were 3e-2 / 3e-4, sized for fold-mode rows, which now take the
# float64 path)
AMBIG_MAX_FRAC = {"table": 2e-3, "packed": 2e-3, "packed_f32": 3e-4}
FLIP_MAX_FRAC = {"table": 1e-5, "packed": 1e-5, "packed_f32": 1e-5}


def _prof():
    return np.load(os.path.join(FIX, "j1713_search.npz"))["input_profile"]


CASES = {
    "tutorial1": dict(
        sig=dict(fcent=1400, bw=400, nchan=2), psr=dict(period=0.005, Smean=10, prof=("gauss", 0.5, 0.05, 1)),
        ops=[("make_pulses", 1.0, "pulses"), ("disperse", 10, "disperse"),
             ("observe", "Arecibo", "Lband_PUPPI", True, "noise")]),
    "northstar_mini": dict(
        sig=dict(fcent=1400, bw=400, nchan=4, fold=False), psr=dict(period=0.005, Smean=1.0, prof=("gauss", 0.5, 0.05, 1)),
        ops=[("scatter_conv", 1e-4, 1400, None), ("make_pulses", 8192 * 20.48e-6, "pulses"),
             ("disperse", 100, "disperse"), ("fd", [2e-4, -3e-5], "fd"),
             ("scatter_shift", 3e-4, 1400, "scatter"), ("null", 0.1, "null"),
             ("observe", "Arecibo", "Lband_PUPPI", True, "noise")]),
    "j1713_search": dict(
        sig=dict(fcent=1500, bw=800, nchan=4, samprate=0.048828125, fold=False),
        psr=dict(period=1.0 / 218.8118437960826270, Smean=0.009, prof=("data", 4)),
        ops=[("make_pulses", 4096 * 20.48e-6, "pulses"), ("disperse", 15.917131, "disperse"),
             ("observe", "GBT", "Lband_GUPPI", True, "noise")]),
    "fold_sublen": dict(
        sig=dict(fcent=1400, bw=400, nchan=2, samprate=1.0 * 2048 * 10 ** -6, sublen=0.5),
        psr=dict(period=1.0, Smean=1.0, prof=("data", 2)),
        ops=[("make_pulses", 2.0, "pulses"), ("disperse", 10.0, "disperse"), ("null", 0.34, "null"),
             ("observe", "GBT", "Lband_GUPPI", True, "noise")]),
    "null_undelayed": dict(
        sig=dict(fcent=1400, bw=400, nchan=3, fold=False), psr=dict(period=0.005, Smean=2.0, prof=("gauss", 0.45, 0.03, 1)),
        ops=[("make_pulses", 4096 * 20.48e-6, "pulses"), ("null", 0.3, "null"), ("disperse", 5, "disperse"),
             ("observe", "Arecibo", "Lband_PUPPI", False, None)]),
    "specidx_int8": dict(
        sig=dict(fcent=1400, bw=400, nchan=4, dtype=np.int8),
        psr=dict(period=0.005, Smean=1.0, prof=("gaussarr",), specidx=-1.6, ref_freq=1300),
        ops=[("make_pulses", 1.0, "pulses"), ("disperse", 20, "disperse"),
             ("observe", "Arecibo", "Lband_PUPPI", True, "noise")]),
}
for _tag, _dt in (("eq", 4.8828125e-06), ("down", 9.765625e-06), ("rebin", 7.5e-06)):
    CASES["observe_" + _tag] = dict(
        sig=dict(fcent=1400, bw=400, nchan=2, fold=False, samprate=(1.0 / 0.005) * 2048 * 10 ** -6),
        psr=dict(period=0.005, Smean=10, prof=("gauss", 0.5, 0.05, 1)),
        ops=[("make_pulses", 0.02, "pulses"), ("observe", ("custom", _dt), "T", True, "noise")])


# ---------------------------------------------------------------------------
# oracle interpretation (derives the injections)
# ---------------------------------------------------------------------------
def b1855():
    """Config C4's portrait: the reference template's profile (io/psrfits.py
    reader; DATA * DAT_SCL + DAT_OFFS, median baseline removed)."""
    from psrsigsim_amd.io.psrfits import template_profile
    from psrsigsim_amd.data import B1855_TEMPLATE
    return template_profile(B1855_TEMPLATE)


def nonuniform_portrait(nchan, n=96):
    """A 1-D Gaussian sampled on NON-uniform phases (u^1.3 of a uniform grid),
    tiled over ``nchan`` rows: (values [nchan, n], phases [n])."""
    ph = (np.arange(n) / n) ** 1.3
    prof = np.exp(-0.5 * ((ph - 0.45) / 0.04) ** 2) + 0.3 * np.exp(-0.5 * ((ph - 0.6) / 0.02) ** 2)
    return np.tile(prof, (nchan, 1)), ph


def _oracle_profile(spec):
    kind = spec[0]
    if kind == "b1855":
        return O.DataProfile(b1855(), nchan=spec[1])
    if kind == "dataph":
        vals, ph = nonuniform_portrait(spec[1])
        return O.DataPortrait(vals, phases=ph)
    if kind == "gauss":
        return O.GaussPortrait(*spec[1:])
    if kind == "gaussarr":
        return O.GaussPortrait(np.array([0.3, 0.6]), np.array([0.02, 0.05]), np.array([0.5, 1.0]))
    return O.DataProfile(_prof(), nchan=spec[1])


def oracle_exec(case, d):
    """Run ``case`` through the oracle with draw provider ``d``; returns
    (stage arrays like the fixtures', injections for the product)."""
    sg = case["sig"]
    sig = O.Signal(sg["fcent"], sg["bw"], nchan=sg["nchan"], samprate=sg.get("samprate"),
                   sublen=sg.get("sublen"), dtype=sg.get("dtype", np.float32), fold=sg.get("fold", True))
    if sg.get("chans") is not None:
        # only global channels [c0, c1) of the Nchan-channel band (a shard):
        # their frequencies, and bw/Nchan kept for the radiometer noise
        c0, c1 = sg["chans"]
        assert c0 == 0 or not any(op[0] == "null" for op in case["ops"]), \
            "null's shift_val comes from global channel 0"
        sig.dat_freq = sig.dat_freq[c0:c1]
        sig.bw = sig.bw * (c1 - c0) / sig.nchan
        sig.nchan = c1 - c0
    ps = case["psr"]
    pspec = ps["prof"]
    if sg.get("chans") is not None and pspec[0] in ("data", "b1855"):
        pspec = ("data", sig.nchan)     # the same 1-D template on the shard's rows
    psr = O.Pulsar(ps["period"], ps["Smean"], profiles=_oracle_profile(pspec),
                   specidx=ps.get("specidx", 0.0), ref_freq=ps.get("ref_freq"))
    inj, A = {}, {}

    def last_chi2():
        return d.log[-1][2] if hasattr(d, "log") else d.draws[d.i - 1][2]

    for op in case["ops"]:
        k = op[0]
        if k == "make_pulses":
            O.make_pulses(sig, psr, op[1], d)
            inj["gen"] = last_chi2()
        elif k == "disperse":
            O.disperse(sig, op[1])
        elif k == "fd":
            O.FD_shift(sig, op[1])
        elif k == "scatter_shift":
            O.scatter_broaden(sig, op[1], op[2], convolve=False)
        elif k == "scatter_conv":
            O.scatter_broaden(sig, op[1], op[2], convolve=True, pulsar=psr)
        elif k == "scatter_tail":
            # EXTENSION (no reference counterpart): the
            # float64 restatement of scatter_broaden(tail=True) -- every row
            # circularly convolved with (1 - a) a^n, a = exp(-dt / tau_c),
            # tau_c = tau_d (f_c / f_ref)^(-22/5); a filter, not a delay, so
            # signal.delay (and the null mask) are untouched
            x = np.asarray(sig.data, dtype=np.float64)
            n = x.shape[1]
            f = np.asarray(sig.dat_freq, dtype=np.float64)
            tau_ms = op[1] * 1e3 * (f / op[2]) ** (-22.0 / 5.0)
            a = np.exp(-(1e-3 / sig.samprate) / tau_ms)[:, None]          # dt in ms (samprate in MHz)
            kk = np.arange(n // 2 + 1)[None, :]
            H = (1 - a) / (1 - a * np.exp(-2j * np.pi * kk / n))
            sig.data = np.fft.irfft(np.fft.rfft(x, axis=1) * H, n=n, axis=1)
        elif k == "null":
            pre_max = np.max(np.abs(np.asarray(sig.data, dtype=np.float64)), axis=1)
            info = O.null(sig, psr, op[1], d)
            inj["null_pulses"] = info["pulses"]
            inj["box"] = info["box_row"]
            inj["rep"] = info["rep_dense"]
            inj["shift_val"] = int(np.asarray(info["shift_val"])[0])
            if info["mask_shifted"] is not None:
                # samples whose shifted mask is within fp32 reach of the > 1
                # threshold may legitimately land on either side of it
                ms = np.asarray(info["mask_shifted"], dtype=np.float64)
                n = ms.shape[1]
                if n >= (1 << 14) and n & (n - 1) == 0:
                    inj["ambig_path"] = "table"
                    band = AMBIG_REL_TABLE * np.max(np.abs(ms), axis=1)[:, None]
                elif packed64(n, case):
                    inj["ambig_path"] = "packed"
                    band = AMBIG_REL_P64 * np.max(np.abs(ms), axis=1)[:, None]
                else:
                    inj["ambig_path"] = "packed_f32"
                    band = AMBIG_REL * np.maximum(pre_max, np.max(np.abs(ms), axis=1))[:, None]
                inj["ambiguous"] = np.abs(ms - 1.0) < np.maximum(AMBIG, band)
        elif k == "observe":
            tel_spec, system, noise = op[1], op[2], op[3]
            if tel_spec == "Arecibo":
                tel = O.Arecibo()
            elif tel_spec == "GBT":
                tel = O.GBT()
            else:
                tel = O.Telescope(20.0, area=None, Tsys=25.0)
                tel.systems["T"] = O.System(35.0, 1.0 / tel_spec[1], samprate_scale=1.0)
            A["out"] = O.observe(sig, psr, tel, system, d, noise=noise)
            if noise:
                inj["noise"] = last_chi2()
        if op[-1] is not None and k != "scatter_conv":
            A["data_" + op[-1]] = np.array(sig.data)
    return A, inj


def oracle_run(name):
    meta, A, draws = load(name)
    _, inj = oracle_exec(CASES[name], O.InjectedDraws(draws))
    return meta, A, inj


# ---------------------------------------------------------------------------
# product interpretation
# ---------------------------------------------------------------------------
_AMB = {"band": 0, "flipped": 0, "total": 0}


def _err(gpu, ref, exclude=None, scale_ref=None):
    """Per-channel max|gpu - ref| / max|ref|.  ``scale_ref`` (same shape)
    supplies the magnitude instead: observe's ``out`` is min(data, draw_max)
    -- the clip is exact and |min(a, c) - min(b, c)| <= |a - b|, so its fp32
    error is that of the un-clipped data and is measured on that scale (a
    fold-mode C4 channel peaks at ~5000 and is clipped to 200)."""
    gpu = np.asarray(gpu, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    if gpu.shape != ref.shape:
        return float("inf")
    ref2 = ref.reshape(ref.shape[0], -1) if ref.ndim > 1 else ref[None]
    mag = ref2
    if scale_ref is not None and np.shape(scale_ref) == ref.shape:
        mag = np.maximum(np.abs(ref2), np.abs(np.asarray(scale_ref, dtype=np.float64).reshape(ref2.shape)))
    scale = np.maximum(np.max(np.abs(mag), axis=1), 1e-30)
    if exclude is not None and exclude.shape == ref.shape and exclude.any():
        # count what the exclusion hides: samples in the band, and those whose
        # null decision actually differs from the reference's
        off = np.abs(gpu.reshape(ref2.shape) - ref2) > 1e-5 * scale[:, None]
        _AMB["band"] += int(exclude.sum())
        _AMB["flipped"] += int((exclude.reshape(ref2.shape) & off).sum())
        _AMB["total"] += int(ref.size)
        gpu = np.where(exclude, ref, gpu)
    gpu2 = gpu.reshape(ref2.shape)
    return float(np.max(np.max(np.abs(gpu2 - ref2), axis=1) / scale))


def assert_plan(lines, nchan, nsamp, tokens, absent=()):
    """The last pss_run of an nchan x nsamp run in a launch-plan log
    (psrsigsim_amd._lib.plan_collect) picked every kernel named in
    ``tokens`` ("fourstep", "1024x4096", "A:fast", "R:pair_row", "C:fast",
    "N:fix_list", ...) and none in ``absent``: the parity tests name the
    kernels whose bits they check, so a dispatch change cannot move them
    onto other kernels unnoticed."""
    pref = "%dx%d:" % (nchan, nsamp)
    runs = [l for l in lines if l.startswith(pref)]
    assert runs, ("no %s run in the plan log" % pref, lines)
    got = set(runs[-1][len(pref):].split())
    missing = set(tokens) - got
    extra = set(absent) & got
    assert not missing and not extra, ("kernel plan %r: missing %s, unexpected %s" % (runs[-1], sorted(missing),
                                                                                     sorted(extra)))
    return runs[-1]


def run_case(name, fused=True, case=None, seed=None):
    """Replay a golden case (``name``) -- or, with ``case``/``seed``, any case
    script against the oracle run with legacy RandomState(seed) draws."""
    import psrsigsim_amd as pss
    import psrsigsim_amd._engine  # noqa: F401
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile, DataProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    from psrsigsim_amd.telescope import Telescope, Receiver, Backend
    from psrsigsim_amd._units import Quantity

    if case is None:
        meta, A, inj = oracle_run(name)
        case = CASES[name]
    else:
        A, inj = oracle_exec(case, O.LegacyDraws(seed))
    sg = case["sig"]
    chans = sg.get("chans")
    sig = FilterBankSignal(sg["fcent"], sg["bw"], Nsubband=sg["nchan"], sample_rate=sg.get("samprate"),
                           sublen=sg.get("sublen"), dtype=sg.get("dtype", np.float32),
                           fold=sg.get("fold", True), shard=chans)

    def rows(a):
        # a shard's injected draws: the oracle computed only its channels
        return pss._engine.RowBlock(chans[0], a) if (chans is not None and a is not None) else a
    for _AMB_k in _AMB:
        _AMB[_AMB_k] = 0
    ps = case["psr"]
    spec = ps["prof"]
    if spec[0] == "gauss":
        prof = GaussProfile(*spec[1:])
    elif spec[0] == "gaussarr":
        prof = GaussProfile(np.array([0.3, 0.6]), np.array([0.02, 0.05]), np.array([0.5, 1.0]))
    elif spec[0] == "b1855":
        prof = DataProfile(b1855(), Nchan=spec[1])
    elif spec[0] == "dataph":
        from psrsigsim_amd.pulsar.portraits import DataPortrait
        vals, ph = nonuniform_portrait(spec[1])
        prof = DataPortrait(vals, phases=ph)
    else:
        prof = DataProfile(_prof(), Nchan=spec[1])
    psr = Pulsar(ps["period"], ps["Smean"], profiles=prof, specidx=ps.get("specidx", 0.0),
                 ref_freq=ps.get("ref_freq"))
    ism = ISM()
    errs = {}
    pss.seed(1)

    amb = {"mask": None}

    seen = []

    def snap(tag):
        if tag is not None:
            seen.append(tag)
        if tag is not None and not fused:
            errs[tag] = _err(sig.data.cpu().numpy(), A["data_" + tag], amb["mask"])

    for op in case["ops"]:
        k = op[0]
        if k == "make_pulses":
            pss.inject(gen=rows(inj["gen"]))
            psr.make_pulses(sig, op[1])
            snap(op[2])
        elif k == "disperse":
            ism.disperse(sig, op[1])
            snap(op[2])
        elif k == "fd":
            ism.FD_shift(sig, op[1])
            snap(op[2])
        elif k == "scatter_shift":
            ism.scatter_broaden(sig, op[1], op[2], convolve=False)
            snap(op[3])
        elif k == "scatter_conv":
            ism.scatter_broaden(sig, op[1], op[2], convolve=True, pulsar=psr)
        elif k == "scatter_tail":
            ism.scatter_broaden(sig, op[1], op[2], tail=True)
            snap(op[3])
        elif k == "null":
            pss.inject(null_pulses=inj["null_pulses"], box=inj["box"])
            if inj["rep"] is not None:
                pss.inject(rep=rows(inj["rep"]))
            psr.null(sig, op[1])
            amb["mask"] = inj.get("ambiguous")
            snap(op[2])
        elif k == "observe":
            tel_spec, system, noise, tag = op[1], op[2], op[3], op[4]
            if tel_spec == "Arecibo":
                tel = T.Arecibo()
            elif tel_spec == "GBT":
                tel = T.GBT()
            else:
                tel = Telescope(20.0, area=None, Tsys=25.0, name="Twenty_Meter")
                tel.add_system(name="T", receiver=Receiver(fcent=1400, bandwidth=400, name="Lband"),
                               backend=Backend(samprate=1.0 / Quantity(tel_spec[1], "s"), name="Cyborg"))
            if noise:
                pss.inject(noise=rows(inj["noise"]))
            pre = A.get("data_" + seen[-1]) if seen else None
            out = tel.observe(sig, psr, system=system, noise=noise, ret_resampsig=True)
            errs["out"] = _err(out.cpu().numpy().astype(np.float64), A["out"], amb["mask"], scale_ref=pre)
            if tag is not None:
                errs[tag] = _err(sig.data.cpu().numpy(), A["data_" + tag], amb["mask"])
    # the final state is always compared
    last = [op for op in case["ops"] if op[-1] is not None and op[0] != "observe"]
    if fused and case["ops"][-1][0] != "observe" and last:
        errs[last[-1][-1]] = _err(sig.data.cpu().numpy(), A["data_" + last[-1][-1]], amb["mask"])
    if _AMB["total"]:
        band = _AMB["band"] / _AMB["total"]
        path = inj.get("ambig_path", "packed_f32")
        flipped = _AMB["flipped"] / _AMB["total"]
        STATS["null_flipped_frac"] = flipped
        STATS["ambiguous_band_frac"] = band
        STATS["ambiguous_path"] = path
        assert band <= AMBIG_MAX_FRAC[path], "null threshold ambiguity band (%s path) holds %.3g of the samples" % (
            path, band)
        assert flipped <= FLIP_MAX_FRAC[path], "%.3g of the samples flipped their null decision (%s path)" % (
            flipped, path)
    return errs


STATS = {}
