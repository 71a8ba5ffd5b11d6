"""Shard-local host planning on the GPU (plan_group, psrsigsim_amd.shard.RowSet):
two ranks (processes sharing the one GPU, gloo plan group) each plan and run
their channel block with profile tables holding only their own rows + the
channel-0 pair (PssPipeline.prof_row0 windows); their rows must be bitwise
the rows of the whole-band run (C3's calls: scatter convolution, delays,
delayed null, radiometer noise)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _c3(nchan, shard, plan_group, log2n):
    import psrsigsim_amd as pss
    from psrsigsim_amd.signal import FilterBankSignal
    from psrsigsim_amd.pulsar import Pulsar, GaussProfile
    from psrsigsim_amd.ism import ISM
    from psrsigsim_amd.telescope import telescope as T
    pss.seed(5)
    sig = FilterBankSignal(1400, 400, Nsubband=nchan, fold=False, shard=shard, plan_group=plan_group)
    psr = Pulsar(0.005, 1.0, profiles=GaussProfile(0.5, 0.05, 1))
    ism = ISM()
    ism.scatter_broaden(sig, 1e-4, 1400, convolve=True, pulsar=psr)
    psr.make_pulses(sig, tobs=(1 << log2n) * 20.48e-6)
    ism.disperse(sig, 100)
    psr.null(sig, 0.1)
    T.Arecibo().observe(sig, psr, system="Lband_PUPPI", noise=True)
    return sig.data.cpu().numpy(), sig._pending


def _rank(rank, world, port, nchan, log2n, out):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from psrsigsim_amd.shard import channel_block
    c0, c1 = channel_block(nchan, rank, world)
    data, _ = _c3(nchan, (c0, c1), dist.group.WORLD, log2n)
    np.save(os.path.join(out, "rank%d.npy" % rank), data)
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("nchan,log2n", [(7, 16), (12, 22)])
def test_plan_group_rows_bitwise(nchan, log2n, hip_lib, tmp_path):
    from psrsigsim_amd.shard import channel_block
    world = 2
    ctx = mp.get_context("spawn")
    port = _port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, nchan, log2n, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    full, _ = _c3(nchan, None, None, log2n)
    for r in range(world):
        c0, c1 = channel_block(nchan, r, world)
        got = np.load(os.path.join(str(tmp_path), "rank%d.npy" % r))
        np.testing.assert_array_equal(got, full[c0:c1])
