#!/usr/bin/env python
"""Benchmark of the filterbank synthesis path (BASELINE.json metric).

One *step* = one pass of the north-star pipeline (config C3) over a freshly
made signal, through the drop-in API exactly as Simulation.simulate strings it
(simulate/simulate.py:292-326) plus the C3 null:

    FilterBankSignal(1400, 400, Nsubband=2048, fold=False)       (20.48 us)
    ISM.scatter_broaden(tau_d=1e-4 s, 1400 MHz, convolve=True)   (profile level)
    Pulsar(5 ms, GaussProfile(0.5, 0.05, 1)).make_pulses(tobs = 2^22 * 20.48 us)
    ISM.disperse(DM=100)
    Pulsar.null(0.1)                       (delayed branch: mask through the FFT)
    Arecibo().observe('Lband_PUPPI', noise=True)

= 2048 x 2^22 channel-samples per GPU, synthetic (Philox) data, fp32 compute.
Host planning, the channel-0 probe for null's shift_val (on the device, no
host round trip) and the fused device run are all inside the timed region.

Multi-GPU: one process per GPU over torch.distributed (RCCL).  Under a
launcher (torchrun / torch.distributed.run: WORLD_SIZE set) every rank runs
its channel block; invoked directly with --gpus N > 1, bench.py launches the
N ranks itself (torch.distributed.run as a child process, before anything in
this process touches the GPU) and exits with their status.
  --scaling strong (default for C3/C2/C4): the BASELINE C3 definition -- ONE
                   2048-channel signal split into N contiguous channel blocks
                   (shard.channel_block): 2048/N channels per rank;
  --scaling weak   (default for C5, whose BASELINE config IS per GPU: 1024 of
                   8192 channels each): every rank owns its own --nchan block.
No collective on the data path (shard-invariant RNG keyed by global channel);
the timing barrier and the max-over-ranks reduction are the only RCCL calls
(the C4 workload adds the gather of the folded product).

Reports (one JSON line on rank 0): value = channel-samples/s over all ranks,
the roofline of the dominant kernel (HIP events on the launch stream, inside
the timed region) and of the whole step (roofline.pipeline_frac: algorithmic
bytes of every kernel of a step / ms_per_step / 8 TB/s), and the CPU oracle
timed on a bounded channel sample; next
to them the first and steady step spans (step_ms_first / step_ms_steady: the
first timed step starts on an idle GPU and carries its host planning) and the
GPU's socket power and gfx clock through the timed steps (gpu_power).
Defaults: 20 timed steps after 2 warm-up steps, N = 1.
"""
import argparse
import contextlib
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "channel-samples/sec (node) at 2048ch x 2^22 samp; % HBM roofline; speedup vs CPU"
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md chip table (spec)
NCHAN = 2048
LOG2N = 22
TOBS_PER_SAMPLE = 20.48e-6

# algorithmic HBM bytes per channel-sample of each kernel in the C3 run
# (DESIGN.md "Roofline"): the four-step spill holds two channels per complex64
# value (pair mode), i.e. 4 B per channel-sample per spill pass; the null mask
# is a once-per-run table (no per-channel bytes).
#   colA: write spill 4 | row: read 4 + write 4 | colC: read spill 4 + write fp32 4
#   null_fix: rewrite the nulled samples, 4 B each.  C3's null(0.1) nulls
#   round(0.1 nsub) whole periods, and the reference thresholds the FFT-shifted
#   chi2(100) box mask at > 1 (pulsar.py:306-330), whose Gibbs ringing crosses
#   the threshold next to the boxes too: 10.1-10.9 % of a channel's samples
#   end up nulled (the oracle's shifted mask at C3's parameters, 8 channels
#   across the band, two seeds; DESIGN.md "Roofline accounting").  PMC writes
#   of the fix-up: 3.91 GB per launch = 0.455 B per channel-sample, 1.08x the
#   4 x 0.105 booked here (profiles/r03/pmc_traffic.json; round 2's 5.5 GB
#   was partial-line write amplification, removed by the lane-major entries)
NULL_FRAC_C3 = 0.105
ALG_BYTES = {"fourstep_colA": 4.0, "fourstep_row": 8.0, "fourstep_colC": 8.0, "null_fix": 4.0 * NULL_FRAC_C3,
             "single_pass": 4.0, "elementwise": 8.0, "fallback_dft": 28.0}


def c3_step(pss, nchan_total, shard, nsamp_log2, ret_out=False, plan_group=None):
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    sig = FilterBankSignal(1400, 400, Nsubband=nchan_total, fold=False, shard=shard, plan_group=plan_group)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    ism = ISM()
    ism.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    psr.make_pulses(sig, tobs=(1 << nsamp_log2) * TOBS_PER_SAMPLE)
    ism.disperse(sig, 100)
    psr.null(sig, 0.1)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True, ret_resampsig=ret_out)
    return sig


F0_B1855 = 186.4940812499314404
_B1855 = {}


def b1855_profile():
    """Config C4's template profile (read once per process)."""
    if "p" not in _B1855:
        from psrsigsim_amd.io.psrfits import template_profile
        from psrsigsim_amd.data import B1855_TEMPLATE
        _B1855["p"] = template_profile(B1855_TEMPLATE)
    return _B1855["p"]


def c4_step(pss, nchan_total, shard, gather, plan_group=None):
    """BASELINE config C4: fold mode, 30 subints x 1024 bins over 30 min
    (30720 samples per channel: the mixed-radix 30 x 1024 four-step), DM 13.3,
    Arecibo radiometer noise; the folded filterbank is gathered to rank 0 over
    RCCL (psrsigsim_amd.shard) inside the step.  Portrait: the B1855+09
    template's profile (DATA * DAT_SCL + DAT_OFFS of the reference's
    data/B1855+09.L-wide.PUPPI.11y.x.sum.sm, median baseline removed; read once
    by the FITS reader, outside the timed region) as a DataProfile tiled over
    the channels."""
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, DataProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    sig = FilterBankSignal(1400, 400, Nsubband=nchan_total, sample_rate=F0_B1855 * 1024 * 1e-6, sublen=60.0,
                           fold=True, shard=shard, plan_group=plan_group)
    psr = Pulsar(1.0 / F0_B1855, 0.005, profiles=DataProfile(b1855_profile(), Nchan=nchan_total))
    psr.make_pulses(sig, tobs=1800.0)
    ISM().disperse(sig, 13.299393)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
    if gather:
        from psrsigsim_amd.shard import gather_channels
        gather_channels(sig.data, nchan_total)
    return sig


def c5_step(pss, nchan_total, shard, nsamp_log2, plan_group=None):
    """BASELINE config C5 per GPU: search mode, 2^24 samples, DM 500 (delays
    up to ~7x10^4 samples), Arecibo radiometer noise."""
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    sig = FilterBankSignal(1400, 400, Nsubband=nchan_total, fold=False, shard=shard, plan_group=plan_group)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, tobs=(1 << nsamp_log2) * TOBS_PER_SAMPLE)
    ISM().disperse(sig, 500)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
    return sig


def c2_step(pss, nchan_total, shard, nsamp_log2, plan_group=None):
    """BASELINE config C2: NANOGrav L-band search mode, 512 channels x 2^20
    samples at 20.48 us, J1713+0747 (P = 1/218.81 Hz from the par file, the
    reference's packaged 2048-bin DataProfile), disperse(DM = 15.917131),
    GBT Lband_GUPPI radiometer noise."""
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, DataProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    from psrsigsim_amd.data import j1713_profile
    sig = FilterBankSignal(1500, 800, Nsubband=nchan_total, sample_rate=0.048828125, fold=False, shard=shard,
                           plan_group=plan_group)
    psr = Pulsar(1.0 / 218.8118437960826270, 0.009, profiles=DataProfile(j1713_profile(), Nchan=nchan_total))
    psr.make_pulses(sig, tobs=(1 << nsamp_log2) * TOBS_PER_SAMPLE)
    ISM().disperse(sig, 15.917131)
    T.GBT().observe(sig, psr, system="Lband_GUPPI", noise=True)
    return sig


def s5_step(pss, nchan_total, shard, plan_group=None):
    """The 5-smooth length 3 125 000 = 2^3 5^8 (the sample count of the
    reference's own simulate fixture, tests/test_simulate.py:47-56): 256
    channels by default (one rank's share of the C3 band at 8 GPUs; 64
    channels leave ~7 % of the step to per-step host work), GaussProfile
    P = 5 ms, disperse(DM=100) + Arecibo noise, through the radix-5
    four-step (1250 x 2500)."""
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    sig = FilterBankSignal(1400, 400, Nsubband=nchan_total, fold=False, shard=shard, plan_group=plan_group)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    psr.make_pulses(sig, tobs=S5_NSAMP * TOBS_PER_SAMPLE)
    ISM().disperse(sig, 100)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
    return sig


S5_NSAMP = 3125000

# The reference's only published timings: the
# dispersion loop's progress line in its tutorials -- disperse stage only,
# hardware unstated.  (shape, ch-samp/s, source)
PUBLISHED = {
    "t1": {"value": 8.8e6, "chans": 126, "nsamp": 97656, "seconds": 1.399, "source": "docs/tutorial_1.rst:178",
           "stage": "ISM.disperse (search mode, 126 of 128 channels at the 98% progress line)"},
    "t2": {"value": 1.84e7, "chans": 63, "nsamp": 40960, "seconds": 0.140, "source": "docs/tutorial_2.rst:150",
           "stage": "ISM.disperse (fold mode, 63 of 64 channels at the 98% progress line)"},
}
T1_NSAMP, T2_NSAMP = 97656, 40960


def tutorial_signal(workload, nchan_total, shard, plan_group=None):
    """The tutorials' signals (BASELINE.md section 1's published shapes):
    t1 = docs/tutorial_1.rst (FilterBankSignal(820, 200, Nsubband=128,
    fold=False) at the default 0.048828125 MHz, GaussProfile(0.5, 0.05, 1),
    Pulsar(1 s, 10 Jy), 2 s -> 97 656 samples = 2^3 3 13 313: the Bluestein
    path; DM 40; GBT 820_GUPPI); t2 = docs/tutorial_2.rst (FilterBankSignal(
    1500, 800, Nsubband=64, sample_rate=2048 / 10 ms, sublen=60, fold=True),
    Pulsar(10 ms, 5 mJy, specidx=-1.6, ref_freq=1400), 20 min -> 20 x 2048 =
    40 960 samples: the mixed-radix 10 x 4096 split; DM 40; GBT
    Lband_GUPPI).  Returns (signal, pulsar, dm, telescope, system) with the
    pulses made."""
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.telescope import telescope as T
    prof = GaussProfile(peak=0.5, width=0.05, amp=1.0)
    if workload == "t1":
        sig = FilterBankSignal(820, 200.0, Nsubband=nchan_total, fold=False, shard=shard, plan_group=plan_group)
        psr = Pulsar(1.0, 10.0, profiles=prof, name="J0000+0000")
        psr.make_pulses(sig, tobs=2.0)
        return sig, psr, 40.0, T.GBT(), "820_GUPPI"
    sig = FilterBankSignal(1500, 800.0, Nsubband=nchan_total, sample_rate=(1.0 / 0.010) * 2048 * 10 ** -6,
                           sublen=60.0, fold=True, shard=shard, plan_group=plan_group)
    psr = Pulsar(0.010, 0.005, profiles=prof, name="J0000+0000", specidx=-1.6, ref_freq=1400.0)
    psr.make_pulses(sig, tobs=60.0 * 20)
    return sig, psr, 40.0, T.GBT(), "Lband_GUPPI"


def tutorial_step(pss, workload, nchan_total, shard, plan_group=None):
    """One pass of the tutorial's pipeline: make_pulses, disperse, observe
    with radiometer noise."""
    from psrsigsim_amd.ism import ISM
    sig, psr, dm, tel, system = tutorial_signal(workload, nchan_total, shard, plan_group)
    ISM().disperse(sig, dm)
    tel.observe(sig, psr, system=system, noise=True)
    return sig


def tutorial_disperse_only(pss, workload, nchan, steps):
    """The published stage alone: ISM.disperse on a materialised pulse signal
    of the tutorial's shape (device-resident, the pulses made and read out
    before the clock starts), K timed calls -> ch-samp/s."""
    import torch
    from psrsigsim_amd.ism import ISM
    sigs = []
    for _ in range(steps + 1):
        sig, psr, dm, _, _ = tutorial_signal(workload, nchan, (0, nchan))
        _ = sig.data                                # pulses materialised (not timed)
        sigs.append((sig, dm))
    sig, dm = sigs[0]
    ISM().disperse(sig, dm)                         # warm-up
    _ = sig.data
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for sig, dm in sigs[1:]:
        ISM().disperse(sig, dm)
        _ = sig.data                                # the delay stage runs here
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    n = int(sigs[0][0].data.shape[1])
    return nchan * n / dt, dt


def cpu_tutorial(workload, nchan):
    """The oracle on the tutorial shape: the disperse stage alone (what the
    published line times: per-channel rfft -> ramp -> irfft in float64) and
    the whole pipeline, single process."""
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from oracle import pss_cpu as O
    d = O.LegacyDraws(1776)
    if workload == "t1":
        sig = O.Signal(820, 200.0, nchan=nchan, fold=False)
        psr = O.Pulsar(1.0, 10.0, profiles=O.GaussPortrait(0.5, 0.05, 1.0))
        tobs, tel, system = 2.0, O.GBT(), "820_GUPPI"
    else:
        sig = O.Signal(1500, 800.0, nchan=nchan, samprate=(1.0 / 0.010) * 2048 * 10 ** -6, sublen=60.0, fold=True)
        psr = O.Pulsar(0.010, 0.005, profiles=O.GaussPortrait(0.5, 0.05, 1.0), specidx=-1.6, ref_freq=1400.0)
        tobs, tel, system = 60.0 * 20, O.GBT(), "Lband_GUPPI"
    t0 = time.perf_counter()
    O.make_pulses(sig, psr, tobs, d)
    t1 = time.perf_counter()
    O.disperse(sig, 40.0)
    t2 = time.perf_counter()
    O.observe(sig, psr, tel, system, d, noise=True)
    t3 = time.perf_counter()
    n = np.asarray(sig.data).shape[1]
    return {"disperse": nchan * n / (t2 - t1), "disperse_s": t2 - t1, "pipeline": nchan * n / (t3 - t0),
            "pipeline_s": t3 - t0, "nsamp": n}


WORKLOADS = {
    "c2": "C2: NANOGrav L-band search mode 512 ch x 2^20 samp, J1713+0747 DataProfile (P=1/218.81 Hz), "
          "disperse(DM=15.917131) + GBT Lband_GUPPI radiometer noise",
    "c3": "C3 north-star: FilterBankSignal 2048 ch x 2^22 samp (strong: one signal channel-sharded over the "
          "GPUs), GaussProfile P=5 ms, "
          "scatter_broaden(1e-4 s, convolve) + disperse(DM=100) + null(0.1) + Arecibo Lband_PUPPI radiometer noise",
    "c4": "C4: fold mode 2048 ch x (30 subints x 1024 bins), P=1/186.49 Hz, B1855+09 template "
          "DataProfile, disperse(DM=13.3) + Arecibo noise, RCCL gather of the folded filterbank to rank 0",
    "c5": "C5 per GPU: 1024 ch x 2^24 samp (8192 ch over 8 GPUs), GaussProfile P=5 ms, disperse(DM=500) + "
          "Arecibo noise",
    "s5": "5-smooth length: 256 ch x 3 125 000 samp (= 2^3 5^8, the reference simulate fixture's sample count), "
          "GaussProfile P=5 ms, disperse(DM=100) + Arecibo noise (radix-5 four-step 1250 x 2500)",
    "t1": "tutorial_1 (the reference's published search-mode shape): 128 ch x 97 656 samp (2 s at 48.8 kHz, "
          "2^3 3 13 313: Bluestein), GaussProfile, P=1 s, disperse(DM=40) + GBT 820_GUPPI noise",
    "t2": "tutorial_2 (the reference's published fold-mode shape): 64 ch x 40 960 samp (20 subints x 2048 bins, "
          "10 x 4096 mixed radix), P=10 ms, specidx -1.6, disperse(DM=40) + GBT Lband_GUPPI noise",
}


def dry_step(pss, nchan_total, shard, nsamp_log2, plan_group=None):
    """--dry-run: the C3 calls up to the fused run's host plan (no device)."""
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd import _engine
    sig = FilterBankSignal(1400, 400, Nsubband=nchan_total, fold=False, shard=shard, plan_group=plan_group)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    ism = ISM()
    ism.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    psr.make_pulses(sig, tobs=((1 << nsamp_log2) if nsamp_log2 else S5_NSAMP) * TOBS_PER_SAMPLE)
    ism.disperse(sig, 100)
    _engine.plan_pipeline(sig, sig._pending, shard[1] - shard[0], shard[0])
    return sig


def usable_cores():
    """CPUs this process may use: its affinity set, capped by the cgroup's
    CPU quota (cgroup v2 cpu.max "quota period", or v1 cfs_quota/period) --
    the box's share of a many-core host is a quota, not an affinity mask --
    next to os.cpu_count() (the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            a, b = f.read().split()[:2]
            if a != "max":
                q = float(a) / float(b)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                a = float(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                b = float(f.read())
            if a > 0:
                q = a / b
        except (OSError, ValueError):
            pass
    if q is not None:
        n = min(n, max(1, int(round(q))))
    return n


def cpu_baseline(nch, nsamp_log2):
    """The oracle (NumPy restatement with the reference's call structure:
    per-channel rfft/irfft, legacy RandomState chi2, scipy PCHIP), single
    process, on `nch` channels of the same pipeline."""
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from oracle import pss_cpu as O
    d = O.LegacyDraws(1776)
    t0 = time.perf_counter()
    sig = O.Signal(1400, 400, nchan=nch, fold=False)
    psr = O.Pulsar(0.005, 1.0, profiles=O.GaussPortrait(0.5, 0.05, 1))
    O.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    O.make_pulses(sig, psr, (1 << nsamp_log2) * TOBS_PER_SAMPLE, d)
    O.disperse(sig, 100)
    O.null(sig, psr, 0.1, d)
    O.observe(sig, psr, O.Arecibo(), "Lband_PUPPI", d, noise=True)
    dt = time.perf_counter() - t0
    return nch * (1 << nsamp_log2) / dt, dt


# one all-core worker: bench.cpu_baseline's pipeline on its own channel block
# (bench.py is not imported there: that would import torch in every worker)
_ALLCORE_WORKER = r'''
import sys, time
sys.path.insert(0, sys.argv[1])
from oracle import pss_cpu as O
nch, log2n, seed = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
d = O.LegacyDraws(seed)
t0 = time.perf_counter()
sig = O.Signal(1400, 400, nchan=nch, fold=False)
psr = O.Pulsar(0.005, 1.0, profiles=O.GaussPortrait(0.5, 0.05, 1))
O.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
O.make_pulses(sig, psr, (1 << log2n) * 20.48e-6, d)
O.disperse(sig, 100)
O.null(sig, psr, 0.1, d)
O.observe(sig, psr, O.Arecibo(), "Lband_PUPPI", d, noise=True)
print(time.perf_counter() - t0)
'''


def cpu_baseline_allcore(workers, nch_each, nsamp_log2):
    """The same oracle pipeline in ``workers`` concurrent single-threaded
    processes (one per core, channel blocks of ``nch_each``; the honest
    all-core CPU figure SURVEY §8(d) asks for next to the single-core one).
    Child processes (no exec of this GPU process): each times its own
    pipeline, the job time is the slowest worker."""
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    env.pop("HIP_VISIBLE_DEVICES", None)
    procs = [subprocess.Popen([sys.executable, "-c", _ALLCORE_WORKER, ROOT, str(nch_each),
                               str(nsamp_log2), str(1776 + w)], stdout=subprocess.PIPE, env=env)
             for w in range(workers)]
    times = []
    for pr in procs:
        out, _ = pr.communicate(timeout=600)
        if pr.returncode != 0:
            raise RuntimeError("all-core CPU worker failed")
        times.append(float(out.decode().split()[-1]))
    dt = max(times)
    return workers * nch_each * (1 << nsamp_log2) / dt, dt


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


@contextlib.contextmanager
def _stdout_to_stderr():
    """fd-level redirect of stdout to stderr: gloo's C++ layer prints its
    connection messages on stdout, which must carry only the JSON line."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def _free_port():
    import socket
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    return port


class PowerSampler:
    """Socket power and gfx clock of this rank's GPU (amdsmi), sampled by a
    daemon thread every `period` s through the timed region: the C3 step runs
    at the power limit with sclk held near 2.1 GHz.  Any
    failure (no amdsmi, no matching device) leaves the bench line's field null."""

    def __init__(self, dev, period=0.05):
        import threading
        self.samples = []
        self.limit_w = None
        self._stop = threading.Event()
        self._ready = threading.Event()
        self._thread = None
        try:
            import amdsmi
            import torch
            amdsmi.amdsmi_init()
            bus = torch.cuda.get_device_properties(dev).pci_bus_id
            self._smi = amdsmi
            self._h = None
            for h in amdsmi.amdsmi_get_processor_handles():
                try:
                    if int(amdsmi.amdsmi_get_gpu_device_bdf(h).split(":")[1], 16) == bus:
                        self._h = h
                except Exception:
                    continue
            if self._h is None:
                return
            lim = amdsmi.amdsmi_get_power_info(self._h).get("power_limit")
            self.limit_w = lim / 1e6 if isinstance(lim, (int, float)) else None
            self._thread = threading.Thread(target=self._run, args=(period,), daemon=True)
        except Exception:
            self._thread = None

    def _sample(self):
        try:
            w = self._smi.amdsmi_get_power_info(self._h).get("current_socket_power")
            c = self._smi.amdsmi_get_clock_info(self._h, self._smi.AmdSmiClkType.GFX).get("clk")
            if isinstance(w, (int, float)) and isinstance(c, (int, float)):
                self.samples.append((float(w), float(c)))
            return True
        except Exception:
            return False

    def _run(self, period):
        self._ready.set()
        while not self._stop.wait(period):
            if not self._sample():
                return

    def start(self):
        """A sample every `period` s on the thread, the first one `period`
        after the start; returns once the thread waits for it.  amdsmi calls
        slow the host work of the next ~2 ms (C4's first timed step: 1.9-2.1
        ms after amdsmi_init or a sample right before it, 1.1-1.2 without;
        profiles/r05/power_sampler.txt), so the sampler is built before the
        warm-up and takes no sample at the start of the timed region."""
        if self._thread is not None:
            self._thread.start()
            self._ready.wait(1.0)

    def stop(self):
        if self._thread is not None:
            self._stop.set()
            self._thread.join(timeout=2.0)

    def report(self):
        if len(self.samples) < 3:
            return None
        w = np.array([a for a, _ in self.samples])
        c = np.array([b for _, b in self.samples])
        return {"socket_w_median": round(float(np.median(w)), 1), "socket_w_max": round(float(w.max()), 1),
                "power_limit_w": self.limit_w, "sclk_mhz_median": round(float(np.median(c)), 1),
                "samples": len(self.samples), "source": "amdsmi, every 50 ms through the timed steps"}


def launch_ranks(n):
    """Start one rank per GPU (torch.distributed.run, 127.0.0.1) as a child
    process running this same command line, and return its exit status.
    Called before this process imports anything that touches the GPU."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
           "--master-addr=127.0.0.1", "--master-port=%d" % _free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None,
                    help="strong (default; c5: weak): --nchan channels in total, split over the GPUs; "
                         "weak: --nchan channels per GPU")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU-only check of the launcher / JSON contract: host planning only, gloo, no GPU")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nchan", type=int, default=NCHAN,
                    help="channels in total (strong scaling) or per GPU (weak)")
    ap.add_argument("--log2n", type=int, default=LOG2N)
    ap.add_argument("--cpu-chans", type=int, default=32, help="oracle sample size (channels; BASELINE.md §3: 32)")
    ap.add_argument("--cpu-workers", type=int, default=16,
                    help="all-core CPU baseline: concurrent single-threaded oracle processes (0: skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="N > 1 process group (nccl = RCCL over xGMI; gloo only to rehearse on one GPU)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a one-GPU box: every rank on cuda:0 (with --backend gloo)")
    ap.add_argument("--whole-band-plan", action="store_true",
                    help="N > 1: every rank plans the whole band's profile tables (no plan group)")
    ap.add_argument("--verbose", action="store_true", help="per-step wall times on stderr")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3",
                    help="BASELINE config (default: the north-star C3; c4/c5 are extra measurements)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if args.workload == "c2":
        if args.nchan == NCHAN:
            args.nchan = 512
        if args.log2n == LOG2N:
            args.log2n = 20
    if args.workload == "c5":
        if args.nchan == NCHAN:
            args.nchan = 1024
        if args.log2n == LOG2N:
            args.log2n = 24
    if args.workload == "c4":
        args.log2n = None
        args.no_cpu = True
    if args.workload == "s5":
        if args.nchan == NCHAN:
            args.nchan = 256
        args.log2n = None
        args.no_cpu = True
    if args.workload in ("t1", "t2"):
        if args.nchan == NCHAN:
            args.nchan = 128 if args.workload == "t1" else 64
        args.log2n = None
    if args.scaling is None:
        args.scaling = "weak" if args.workload == "c5" else "strong"

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        print("bench.py: --gpus %d but the launcher started %d ranks; measuring %d" % (args.gpus, world, world),
              file=sys.stderr)
    if args.dry_run:
        if world > 1:
            with _stdout_to_stderr():
                dist.init_process_group("gloo")
                dist.barrier()
    elif world > 1:
        dev = 0 if args.same_device else local
        torch.cuda.set_device(dev)
        with _stdout_to_stderr():
            if args.backend == "gloo":
                dist.init_process_group("gloo")
                dist.barrier()
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    ranks = dist.get_world_size() if world > 1 else 1
    import psrsigsim_amd as pss
    from psrsigsim_amd import _lib
    from psrsigsim_amd.shard import channel_block
    if not args.dry_run:
        _lib.lib()
    pss.seed(1776)

    if args.scaling == "strong":
        total = args.nchan
        shard = channel_block(total, rank, world)
    else:
        total = args.nchan * world
        shard = (rank * args.nchan, (rank + 1) * args.nchan)
    C = shard[1] - shard[0]

    def sync():
        if not args.dry_run:
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()
        sync()

    nsamp = {"c4": 30720, "s5": S5_NSAMP, "t1": T1_NSAMP, "t2": T2_NSAMP}.get(args.workload) or (1 << args.log2n)

    def step():
        # the API prints the reference's user warnings (e.g. C4's "sample
        # rate < Nyquist"); stdout carries only the JSON line
        with contextlib.redirect_stdout(sys.stderr):
            return _step()

    # host planning of the profile tables split over the ranks (shard.RowSet):
    # a gloo group next to the RCCL one, so the planning reductions stay on
    # the host and never wait for the device
    pg = None
    if world > 1 and not args.whole_band_plan:
        if args.dry_run or args.backend == "gloo":
            pg = dist.group.WORLD
        else:
            with _stdout_to_stderr():
                pg = dist.new_group(backend="gloo")
                dist.barrier(group=pg)

    def _step():
        if args.dry_run:
            return dry_step(pss, total, shard, args.log2n, plan_group=pg)
        if args.workload == "c4":
            return c4_step(pss, total, shard, gather=world > 1, plan_group=pg)
        if args.workload == "c5":
            return c5_step(pss, total, shard, args.log2n, plan_group=pg)
        if args.workload == "c2":
            return c2_step(pss, total, shard, args.log2n, plan_group=pg)
        if args.workload == "s5":
            return s5_step(pss, total, shard, plan_group=pg)
        if args.workload in ("t1", "t2"):
            return tutorial_step(pss, args.workload, total, shard, plan_group=pg)
        return c3_step(pss, total, shard, args.log2n, plan_group=pg)

    power = None if args.dry_run else PowerSampler(torch.cuda.current_device())
    for _ in range(args.warmup):
        s = step()
        del s
    # stream-ordered step boundaries (the engine launches on the current
    # stream): the first step's span includes its host planning on an idle
    # GPU, the later ones are the steady state.  These events and the
    # library's per-launch timing events are created (first record) before
    # the barrier, so the timed steps pay no event creation.
    evs = []
    if not args.dry_run:
        _lib.load().pss_timing_enable(1)
        _lib.timing_collect()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        for e in evs:
            e.record()
    if power is not None:
        power.start()
    barrier()
    t0 = time.perf_counter()
    if evs:
        evs[0].record()
    marks = []
    for i in range(args.steps):
        s = step()
        if args.workload == "c4":
            _ = s.data          # fold-mode output is small: materialise it (the gather did when N > 1)
        del s
        if evs:
            evs[i + 1].record()
        marks.append(time.perf_counter())
    sync()
    t1 = time.perf_counter()
    if power is not None:
        power.stop()
    spans = [a.elapsed_time(b) for a, b in zip(evs, evs[1:])]
    if args.verbose:
        prev = t0
        for i, m in enumerate(marks):
            print("step %d host-return %.2f ms" % (i, (m - prev) * 1e3), file=sys.stderr)
            prev = m
        print("final sync %.2f ms" % ((t1 - marks[-1]) * 1e3), file=sys.stderr)
    barrier()
    launches = []
    if not args.dry_run:
        _lib.load().pss_timing_enable(0)
        launches = _lib.timing_collect()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cpu" if (args.dry_run or args.backend == "gloo") else "cuda",
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    per_step = elapsed / args.steps
    n_devices = 1 if args.same_device else world
    units = float(total) * nsamp
    value = units / per_step

    # dominant kernel of the full-size launches
    full = C * nsamp
    agg = {}
    for kind, ms, u in launches:
        if u != full:
            continue
        a = agg.setdefault(kind, [0.0, 0])
        a[0] += ms
        a[1] += 1
    gpu_ms = sum(v[0] for v in agg.values()) / max(args.steps, 1)
    dom = max(agg, key=lambda k: agg[k][0]) if agg else None
    roof = None
    kernels = {}
    for k, (ms, n) in agg.items():
        avg = ms / n
        b = ALG_BYTES.get(k, 0.0) * full
        kernels[k] = {"avg_ms": round(avg, 4), "launches": n, "alg_bytes": b,
                      "GBps": round(b / (avg * 1e-3) / 1e9, 1)}
    # the whole step against the HBM roofline: every kernel's algorithmic
    # bytes of one step (all ranks) over the wall time per step
    step_bytes = sum(ALG_BYTES.get(k, 0.0) * full * n for k, (ms, n) in agg.items()) / max(args.steps, 1) \
        * (float(total) / C)
    if dom is not None:
        avg_ms = agg[dom][0] / agg[dom][1]
        bytes_launch = ALG_BYTES[dom] * full
        ach = bytes_launch / (avg_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "kernel": dom,
                "avg_launch_ms": round(avg_ms, 4), "alg_bytes_per_launch": bytes_launch,
                "pipeline_alg_bytes_per_step": step_bytes,
                "pipeline_achieved": round(step_bytes / per_step / 1e9, 1),
                # (--same-device rehearsals: every rank on one card, one HBM)
                "pipeline_frac": round(step_bytes / per_step / 1e9 / (HBM_PEAK_GBS * n_devices), 4),
                "pipeline_frac_basis": "all kernels' algorithmic bytes per step (ALG_BYTES x channel-samples) "
                                       "/ ms_per_step / (8 TB/s x n_devices)"}
        # measured HBM bytes per launch of this kernel (rocprofv3 PMC passes,
        # tools/pmc_round.sh + tools/pmc_traffic.py; C3 size only)
        # the rocprofv3 kernel trace of the same C3 run (tools/prof_summary.py
        # --json, full-size launches): which kernel dominates there and its
        # fraction, reported next to this run's HIP-event figures (the two
        # rankings can differ box to box)
        for rnd in ("r06", "r05", "r04"):
            kj = os.path.join(ROOT, "profiles", rnd, "kernel_profile.json")
            if args.workload == "c3" and C == NCHAN and nsamp == (1 << LOG2N) and os.path.exists(kj):
                kp = json.load(open(kj))
                kp = {k: v for k, v in kp.items() if k in ALG_BYTES}
                if kp:
                    pd = max(kp, key=lambda k: kp[k]["avg_ms"])
                    fr = {k: round(ALG_BYTES[k] * full / (v["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                          for k, v in kp.items()}
                    roof["frac_profile"] = fr[pd]
                    roof["kernel_profile"] = pd
                    roof["avg_launch_ms_profile"] = kp[pd]["avg_ms"]
                    roof["frac_profile_same_kernel"] = fr.get(dom)
                    roof["frac_profile_source"] = "profiles/%s/kernel_profile.json (rocprofv3 kernel trace, " \
                                                  "full-size launches)" % rnd
                break
        for rnd in ("r06", "r05", "r04", "r03", "r02"):
            tj = os.path.join(ROOT, "profiles", rnd, "pmc_traffic.json")
            if args.workload == "c3" and C == NCHAN and nsamp == (1 << LOG2N) and os.path.exists(tj):
                t = json.load(open(tj)).get(dom)
                if t:
                    roof["traffic"] = round(t["traffic_bytes"] / 1e9, 3)
                    roof["traffic_unit"] = "GB per launch (PMC, profiles/%s/pmc_traffic.json)" % rnd
                break                           # the newest round's passes only

    cpu = None
    cpu_all = None
    # CPU baseline: rank 0 at N=1 only, on the C3 pipeline (the metric's workload)
    if rank == 0 and world == 1 and not args.no_cpu and not args.dry_run and args.workload == "c3":
        v, dt = cpu_baseline(args.cpu_chans, args.log2n)
        if args.cpu_workers > 0:
            va, dta = cpu_baseline_allcore(args.cpu_workers, 2, args.log2n)
            cpu_all = {"value": round(va, 1), "unit": "channel-samples/s", "cores": args.cpu_workers,
                       "cpu_count": os.cpu_count(), "usable_cores": usable_cores(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "kind": "port",
                       "sample": "%d concurrent single-threaded processes x 2 ch x 2^%d samp of the same C3 "
                                 "pipeline (oracle/pss_cpu.py), slowest worker %.1f s" % (args.cpu_workers,
                                                                                         args.log2n, dta)}
        cpu = {"value": round(v, 1), "unit": "channel-samples/s", "cores": 1, "cpu_count": os.cpu_count(),
               "usable_cores": usable_cores(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "kind": "port",
               "sample": "%d ch x 2^%d samp of the same C3 pipeline, oracle/pss_cpu.py (float64 NumPy, "
                         "reference call structure; like the reference it also builds observe's pre-noise "
                         "out copy, ~2%% of its time, which the GPU run elides when ret_resampsig=False), "
                         "single process, %.1f s on %s" % (args.cpu_chans, args.log2n, dt, cpu_model())}
    tut = None
    if rank == 0 and world == 1 and not args.dry_run and args.workload in ("t1", "t2"):
        # the published stage (disperse alone) next to the reference's own
        # number and the oracle's on this host, same shape
        pub = PUBLISHED[args.workload]
        gv, gdt = tutorial_disperse_only(pss, args.workload, total, max(args.steps, 5))
        tut = {"published_disperse": dict(pub, unit="channel-samples/s", hardware="unstated (the tutorial's "
                                          "run; BASELINE.md section 1)"),
               "gpu_disperse_only": {"value": round(gv, 1), "ms": round(gdt * 1e3, 4),
                                     "vs_published": round(gv / pub["value"], 1)}}
        if not args.no_cpu:
            c = cpu_tutorial(args.workload, total)
            tut["cpu_oracle"] = {"disperse_only": round(c["disperse"], 1), "disperse_s": round(c["disperse_s"], 3),
                                 "pipeline": round(c["pipeline"], 1), "pipeline_s": round(c["pipeline_s"], 3),
                                 "cores": 1, "cpu_count": os.cpu_count(), "usable_cores": usable_cores(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
                                 "kind": "port", "host": cpu_model()}
            tut["gpu_disperse_only"]["vs_cpu_oracle"] = round(gv / c["disperse"], 1)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "channel-samples/s",
            "n_gpus": world, "n_devices": n_devices, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(per_step * 1e3, 3), "higher_is_better": True, "scaling": args.scaling,
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (Philox chi2 pulses/noise)",
            "config": {"workload": WORKLOADS[args.workload], "nchan_total": total,
                       "nchan_per_gpu": C, "nsamp": nsamp, "parallelism": "channel-shard x%d" % world},
            "ranks": ranks,
            "gpu_kernel_ms_per_step": round(gpu_ms, 3),
            "step_ms_first": round(spans[0], 3) if spans else None,
            "step_ms_steady": round(float(np.median(spans[1:])), 3) if len(spans) > 1 else None,
            "step_ms_first_minus_steady": (round(spans[0] - float(np.median(spans[1:])), 3)
                                           if len(spans) > 1 else None),
            "gpu_power": power.report() if power is not None else None,
            "kernels": kernels,
            "roofline": roof,
            "cpu_baseline": cpu,
            "speedup_vs_cpu": round(value / cpu["value"], 1) if cpu else None,
            "cpu_baseline_allcore": cpu_all,
            "speedup_vs_cpu_allcore": round(value / cpu_all["value"], 1) if cpu_all else None,
        }
        if tut is not None:
            line["published_shape"] = tut
        if args.dry_run:
            line["dry_run"] = "host planning only (CPU, gloo): launcher / JSON contract check, not a measurement"
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
