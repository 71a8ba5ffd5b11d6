"""Multi-process (gloo, CPU) checks of the channel-sharded path: every rank
plans its block of a sharded signal exactly like the same rows of the
unsharded signal (tables, ramp words, Nyquist factors, RNG keys), so the
device runs are bit-identical per row (the GPU side of that claim is
tests/test_gpu_stats.py::test_shard_invariance_bitwise)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _plan(nchan, shard, plan_group=None, specidx=0.0, ret_psr=False):
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd import _engine
    pss.seed(99)
    sig = FilterBankSignal(1400, 400, Nsubband=nchan, fold=False, shard=shard, plan_group=plan_group)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1), specidx=specidx, ref_freq=1300)
    ism = ISM()
    ism.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    psr.make_pulses(sig, tobs=(1 << 16) * 20.48e-6)
    ism.disperse(sig, 100)
    ism.FD_shift(sig, [1e-4, 2e-5])
    c0, c1 = sig.shard
    P = _engine.plan_pipeline(sig, sig._pending, c1 - c0, c0)
    if ret_psr:
        return sig, P, psr
    return sig, P


def _plan_group_worker(rank, world, port, nchan, q):
    """Shard-local planning (plan_group): each rank's profile tables hold
    only its channels + the channel-0 pair, bitwise the rows of the
    whole-band plan, and the band-wide scalars match."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from psrsigsim_amd.shard import channel_block
    c0, c1 = channel_block(nchan, rank, world)
    ok = True
    for specidx in (0.0, -1.6):
        sig, P, psr = _plan(nchan, (c0, c1), plan_group=dist.group.WORLD, specidx=specidx, ret_psr=True)
        fsig, F, fpsr = _plan(nchan, None, specidx=specidx, ret_psr=True)
        src, fsrc = sig._pending.source, fsig._pending.source
        ids = src.row_ids
        want = sorted(set([0, 1]) | set(range(c0, c1)))
        ok &= ids is not None and list(ids) == want
        ok &= src.table.shape[0] == len(want)
        ok &= np.array_equal(src.table, fsrc.table[want])
        ok &= float(sig._Smax.value) == float(fsig._Smax.value)
        ok &= psr.Profiles.Amax == fpsr.Profiles.Amax
        ok &= np.array_equal(psr.Profiles._max_profile, fpsr.Profiles._max_profile)
        ok &= np.array_equal(psr.Profiles._calcOffpulseWindow(Nphase=244),
                             fpsr.Profiles._calcOffpulseWindow(Nphase=244))
        for k in ("ramp", "nyq_re", "nyq_im"):
            ok &= np.array_equal(P["arrays"][k], F["arrays"][k][c0:c1])
        for k in ("seed", "call_gen", "phase_step", "knot_m", "nint", "draw_norm", "src"):
            ok &= P[k] == F[k]
    flag = torch.tensor([1 if ok else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        q.put(int(flag.item()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,nchan", [(2, 16), (3, 10)])
def test_shard_local_planning_gloo(world, nchan):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_group_worker, args=(r, world, port, nchan, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    assert q.get(timeout=10) == 1


def _worker(rank, world, port, nchan, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    per = nchan // world
    sig, P = _plan(nchan, (rank * per, (rank + 1) * per))
    full_sig, F = _plan(nchan, None)
    ok = True
    sl = slice(rank * per, (rank + 1) * per)
    for k in ("ramp", "nyq_re", "nyq_im"):
        ok &= np.array_equal(P["arrays"][k], F["arrays"][k][sl])
    for k in ("seed", "call_gen", "phase_step", "knot_m", "nint", "prof_rows", "draw_norm", "src"):
        ok &= P[k] == F[k]
    ok &= np.array_equal(sig._pending.source.table, full_sig._pending.source.table)
    ok &= P["chan0"] == rank * per and P["nchan"] == per
    # gather the shard plans on every rank: they tile the full plan exactly
    t = torch.tensor(P["arrays"]["ramp"].view(np.int64))
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    whole = torch.cat(parts).numpy().view(np.uint64)
    ok &= np.array_equal(whole, F["arrays"]["ramp"])
    flag = torch.tensor([1 if ok else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        q.put(int(flag.item()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_plans_tile_the_unsharded_plan(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 16, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) == 1


def test_shard_validation():
    from psrsigsim_amd.signal import FilterBankSignal
    with pytest.raises(ValueError):
        FilterBankSignal(1400, 400, Nsubband=8, shard=(4, 12))


def test_channel_block_tiles():
    from psrsigsim_amd.shard import channel_block
    for nchan in (1, 7, 16, 2048, 2049):
        for world in (1, 2, 3, 8):
            blocks = [channel_block(nchan, r, world) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == nchan
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in blocks]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        channel_block(8, 2, 2)


def _gather_worker(rank, world, port, nchan, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from psrsigsim_amd.shard import channel_block, gather_channels
    c0, c1 = channel_block(nchan, rank, world)
    # a folded product: [channels, bins] (+ a trailing axis to check shapes)
    full = torch.arange(nchan * 12, dtype=torch.float32).reshape(nchan, 6, 2) * 0.5 - 3.0
    got = gather_channels(full[c0:c1].clone(), nchan, dst=world - 1)
    ok = (got is None) if rank != world - 1 else bool(torch.equal(got, full))
    flag = torch.tensor([1 if ok else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        q.put(int(flag.item()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,nchan", [(2, 16), (3, 10)])
def test_gather_channels_gloo(world, nchan):
    """The folded/down-sampled product's gather (RCCL on the GPU path) on
    gloo: uneven channel blocks, non-zero destination rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, nchan, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(timeout=10) == 1


def test_bench_self_launch_world2():
    """bench.py --gpus 2 started directly launches its two ranks itself
    (torch.distributed.run child process, 127.0.0.1) and rank 0 prints one
    JSON line reporting both ranks -- here in --dry-run (gloo, host planning
    only), the same launcher path the GPU run takes with RCCL."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for scaling in ("weak", "strong", None):
        flag = ["--scaling", scaling] if scaling else []
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1",
                            "--warmup", "0", "--dry-run", "--log2n", "14", "--nchan", "8"] + flag,
                           capture_output=True, text=True, timeout=300, cwd=root)
        scaling = scaling or "strong"      # the C3 default: one signal split over the GPUs (BASELINE C3)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [l for l in r.stdout.splitlines() if l.strip()]
        assert len(lines) == 1 and lines[0].startswith("{"), r.stdout   # stdout carries only the JSON line
        line = json.loads(lines[0])
        assert line["n_gpus"] == 2 and line["ranks"] == 2
        assert line["scaling"] == scaling
        assert line["config"]["nchan_total"] == (16 if scaling == "weak" else 8)
        assert line["config"]["nchan_per_gpu"] == (8 if scaling == "weak" else 4)
        assert line["value"] > 0


def test_rowset_requires_host_backend(monkeypatch):
    """shard.RowSet reduces CPU tensors: an NCCL/RCCL plan_group is refused
    with a clear error instead of failing or hanging inside a collective."""
    from psrsigsim_amd import shard
    monkeypatch.setattr(shard.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(shard.dist, "get_backend", lambda group=None: "nccl")
    with pytest.raises(ValueError, match="gloo"):
        shard.RowSet(0, 4, 4, object())


def test_rowset_uninitialised_and_mixed_backend(monkeypatch):
    """Without an initialised process group RowSet raises a ValueError
    naming the fix; a mixed-device group ('cpu:gloo,cuda:nccl') is accepted
    (its gloo part reduces the CPU tensors)."""
    from psrsigsim_amd import shard
    monkeypatch.setattr(shard.dist, "is_initialized", lambda: False)
    with pytest.raises(ValueError, match="init_process_group"):
        shard.RowSet(0, 4, 4, None)
    monkeypatch.setattr(shard.dist, "is_initialized", lambda: True)
    monkeypatch.setattr(shard.dist, "get_backend", lambda group=None: "cpu:gloo,cuda:nccl")
    monkeypatch.setattr(shard, "_COVERED", {(id(None), 0, 4, 4)})
    rs = shard.RowSet(0, 4, 4, None)
    assert rs.c0 == 0 and rs.c1 == 4
