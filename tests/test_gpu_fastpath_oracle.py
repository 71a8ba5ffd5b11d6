"""The headline (fast-path) kernels against the oracle directly (VERDICT r02
item 8): a C3-geometry run -- global channels 0..3 of the 2048-channel band,
2^22 samples, scatter_broaden(convolve) + disperse(100) + delayed null(0.1)
+ Arecibo radiometer noise, observe() without a returned copy -- so
k_pairA_fast / k_pair_row / k_pairC_fast / k_null_fix_list run with their
own Philox draws, not injected ones.  And the C5 geometry (VERDICT r04 item
3): global channels 0..3 of the 8192-channel band, 2^24 samples, DM 500,
noise -- without a null (BASELINE C5: the 1024 x 16384 split, C3's
k_pairA_fast / k_pairC_fast and the 16384-point k_pair_row_seq) and with a
delayed null(0.1) (the 2048 x 8192 split: k_pairA_fast on 2048-point
columns, the 8192-point k_pair_row_seq, k_pairC_fast32, k_null_fix_list).
Each run asserts through the launch-plan log (pss_plan_collect) that these
kernels, and no generic pass, produced the bits it checks.  The draws are then recovered with
pss_chi2_fill (the same counter-based keys: seed, call id, purpose, global
channel, sample) and replayed through the CPU oracle in the reference's
draw order (pulses, null pulse choice, box values, replacements, noise).
Tolerance: per-channel max|d| / max|ref| <= 1e-5 (north_star), null
threshold decisions within fp32 reach of the threshold excluded as in
tests/replay.py."""
import numpy as np
import pytest
import torch

from oracle import pss_cpu as O
from tests import replay

pytestmark = pytest.mark.gpu
TOL = 1e-5
P_PULSE, P_BOX, P_REP, P_NOISE = 1, 2, 3, 4


def _fill(rows, chan0, n, df, seed, call, purpose):
    from psrsigsim_amd import _lib, _engine
    out = torch.empty((rows, n), dtype=torch.float32, device="cuda")
    _lib.check(_lib.lib().pss_chi2_fill(_engine.ptr(out), rows, chan0, n, float(df), seed, call, purpose,
                                        _engine.stream_ptr()))
    return out.cpu().numpy().astype(np.float64)


class _PhiloxReplay(object):
    """Oracle draw provider serving the device's Philox draws in the
    reference's call order; replacement draws are taken at the positions the
    oracle's own mask selects (oracle.null's chi2_at hook)."""

    def __init__(self, gen, pulses, boxes, rep, noise):
        self.queue = [("chi2", gen), ("choice", pulses)] + [("box", b) for b in boxes] + [("chi2", noise)]
        self.rep = rep
        self.log = []

    def _pop(self, kind):
        k, a = self.queue.pop(0)
        assert k == kind, (k, kind)
        return a

    def chi2(self, df, size):
        if self.queue and self.queue[0][0] == "box":
            a = self._pop("box")[:int(size)]
        else:
            a = self._pop("chi2")
            assert a.shape == tuple(np.atleast_1d(size)), (a.shape, size)
        self.log.append(("chi2", float(df), a))
        return a

    def choice(self, n, k):
        a = self._pop("choice")
        assert len(a) == k
        return a

    def chi2_at(self, df, hit):
        a = self.rep[hit]
        self.log.append(("chi2", float(df), a))
        return a


# (name, log2 N, band channels, scatter_broaden(convolve), DM, null)
GEOMS = {"c3": (22, 2048, True, 100, True), "c5": (24, 8192, False, 500, False),
         "c5_null": (24, 8192, False, 500, True)}
# the kernels each geometry must run (pss_plan_collect tokens)
PLANS = {"c3": ("fourstep", "1024x4096", "A:fast", "R:pair_row", "C:fast", "N:table", "N:fix_list"),
         "c5": ("fourstep", "1024x16384", "A:fast_shared", "R:pair_row_seq", "C:fast"),
         "c5_null": ("fourstep", "2048x8192", "A:fast_shared", "R:pair_row_seq", "C:fast32", "N:table",
                     "N:fix_list")}


@pytest.mark.parametrize("geom", sorted(GEOMS))
def test_fast_path_channels_vs_oracle(geom, hip_lib):
    import psrsigsim_amd as pss
    from psrsigsim_amd import _engine, _lib
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    log2n, band, scatter, dm, null = GEOMS[geom]
    N, C, seed = 1 << log2n, 4, 0x5EED0003 + log2n
    pss.seed(seed)
    sig = FilterBankSignal(1400, 400, Nsubband=band, fold=False, shard=(0, C))
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    ism = ISM()
    if scatter:
        ism.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    psr.make_pulses(sig, tobs=N * 20.48e-6)                 # call 1
    ism.disperse(sig, dm)
    if null:
        psr.null(sig, 0.1)                                  # call 2
    _lib.plan_collect()
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)   # call 3 / 2 (no copy: fast epilogue)
    got = sig.data.cpu().numpy().astype(np.float64)
    replay.assert_plan(_lib.plan_collect(), C, N, PLANS[geom], absent=("A:generic", "C:generic"))
    # the device's draws, recovered by key
    gen = _fill(C, 0, N, 1.0, seed, 1, P_PULSE)
    if null:
        nsub = int(sig.nsub)
        npulse = int(np.round(nsub * 0.1))
        pulses = _engine.host_rng(2).choice(nsub, npulse, replace=False)
        nph = int(psr._nph(sig))
        rep = _fill(C, 0, N, 1.0, seed, 2, P_REP)
        boxrows = _fill(npulse, 0, nph, 100.0, seed, 2, P_BOX)   # row = rank in the choice list, column = bin
    noise = _fill(C, 0, N, 1.0, seed, 3 if null else 2, P_NOISE)
    ops = [("scatter_conv", 1e-4, 1400, None)] if scatter else []
    ops += [("make_pulses", N * 20.48e-6, "pulses"), ("disperse", dm, "disperse")]
    ops += [("null", 0.1, "null")] if null else []
    ops += [("observe", "Arecibo", "Lband_PUPPI", True, "noise")]
    case = dict(sig=dict(fcent=1400, bw=400, nchan=band, fold=False, chans=(0, C)),
                psr=dict(period=0.005, Smean=1.0, prof=("gauss", 0.5, 0.05, 1)), ops=ops)
    if null:
        d = _PhiloxReplay(gen, pulses, [boxrows[r] for r in range(npulse)], rep, noise)
    else:
        d = _PhiloxReplay(gen, None, [], None, noise)
        d.queue = [q for q in d.queue if q[0] != "choice"]
    A, inj = replay.oracle_exec(case, d)
    assert not d.queue, "draws left over: the oracle's call order diverged"
    err = replay._err(got, A["data_noise"], inj.get("ambiguous"))
    assert err <= TOL, err
    if null:
        amb = inj["ambiguous"]
        assert amb.mean() <= replay.AMBIG_MAX_FRAC["table"]
