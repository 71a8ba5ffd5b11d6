"""Channel shards across the GPUs of one node.

Frequency channels are independent on this path, so a multi-GPU run gives
every rank (one process per GPU, ``torch.distributed``) a contiguous block of
global channels -- ``FilterBankSignal(..., shard=channel_block(...))`` -- and
nothing is exchanged while the signal is synthesised: every table row, delay
and random draw is keyed by the GLOBAL channel, so a rank's rows are bitwise
the rows of the unsharded run.

The one collective of the path is the last step: the small folded or
down-sampled product (``Backend.fold``, ``Telescope.observe(...,
ret_resampsig=True)`` after down-sampling) is gathered to one rank before
PSRFITS I/O -- over RCCL/xGMI when the process group is ``nccl`` (device
tensors), over gloo for host tensors (the CPU tests).  Full-resolution
filterbanks (34 GB per GPU at the north-star size) stay on their rank.
"""
import torch
import torch.distributed as dist

__all__ = ["channel_block", "gather_channels"]


def channel_block(nchan, rank, world):
    """Contiguous global channel block ``(c0, c1)`` of ``rank`` out of
    ``world`` (the first ``nchan % world`` ranks hold one channel more)."""
    nchan, rank, world = int(nchan), int(rank), int(world)
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank %d of %d" % (rank, world))
    base, extra = divmod(nchan, world)
    c0 = rank * base + min(rank, extra)
    return c0, c0 + base + (1 if rank < extra else 0)


def gather_channels(block, nchan, dst=0, group=None):
    """Gather every rank's channel block (``[c1 - c0, ...]`` rows of the
    blocks laid out by :func:`channel_block`) into the full ``[nchan, ...]``
    array on rank ``dst``; other ranks get ``None``.

    One ``gather`` of equal-size (row-padded) blocks: on the ``nccl`` backend
    RCCL moves them device to device over xGMI, and rank ``dst`` receives
    ``world`` contiguous slabs that are trimmed and concatenated in place.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:
        return block
    rows = [channel_block(nchan, r, world) for r in range(world)]
    c0, c1 = rows[rank]
    if block.shape[0] != c1 - c0:
        raise ValueError("rank %d holds %d rows, its channel block is %d" % (rank, block.shape[0], c1 - c0))
    pad = max(b - a for a, b in rows)
    send = block.contiguous()
    if send.shape[0] < pad:
        send = torch.cat([send, send.new_zeros((pad - send.shape[0],) + tuple(send.shape[1:]))])
    recv = None
    if rank == dst:
        recv = [torch.empty_like(send) for _ in range(world)]
    dist.gather(send, gather_list=recv, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([recv[r][:b - a] for r, (a, b) in enumerate(rows)])
