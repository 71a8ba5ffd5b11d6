"""Channel shards across the GPUs of one node.

Frequency channels are independent on this path, so a multi-GPU run gives
every rank (one process per GPU, ``torch.distributed``) a contiguous block of
global channels -- ``FilterBankSignal(..., shard=channel_block(...))`` -- and
nothing is exchanged while the signal is synthesised: every table row, delay
and random draw is keyed by the GLOBAL channel, so a rank's rows are bitwise
the rows of the unsharded run.

Host planning can be split the same way (``FilterBankSignal(..., shard=...,
plan_group=group)``, :class:`RowSet`): each rank then builds the per-channel
profile tables (scatter-broadening convolutions, PCHIP coefficients, device
tables) only for its own channels plus the channel-0 pair its ``null()``
probe needs, and the portrait-wide quantities the reference derives from
every channel -- the normalisation ``Amax``, the first row that peaks at 1
(``_max_profile``: ``Smax`` and the off-pulse window), the periodic-closure
test -- are exact reductions over ``group`` (a host process group, e.g.
gloo).  Without ``plan_group`` every rank plans the whole band.

The one collective of the data path is the last step: the small folded or
down-sampled product (``Backend.fold``, ``Telescope.observe(...,
ret_resampsig=True)`` after down-sampling) is gathered to one rank before
PSRFITS I/O -- over RCCL/xGMI when the process group is ``nccl`` (device
tensors), over gloo for host tensors (the CPU tests).  Full-resolution
filterbanks (34 GB per GPU at the north-star size) stay on their rank.
"""
import torch
import torch.distributed as dist

__all__ = ["channel_block", "gather_channels", "RowSet"]


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


_COVERED = set()


class RowSet(object):
    """The global channels whose profile rows this rank computes -- its shard
    [c0, c1) plus channels 0 and 1 (the pair of the channel-0 probe) -- and
    the host process group whose ranks together hold every channel.

    Reductions are exact (max / min / or / one row copied from an owner), so
    a rank's tables and the portrait-wide scalars are bitwise those of a
    whole-band plan.  Every rank of the group must make the same API calls
    (the reductions are collective)."""

    def __init__(self, c0, c1, nglobal, group):
        import numpy as np
        # the reductions run on CPU tensors: the group needs a host backend
        # (an NCCL/RCCL group would fail or hang here; bench.py makes a gloo
        # group next to the RCCL one)
        if not dist.is_available() or not dist.is_initialized():
            raise ValueError("plan_group needs an initialised torch.distributed process group (gloo): call "
                             "torch.distributed.init_process_group first")
        backend = str(dist.get_backend(group)).lower()
        # a mixed-device group ('cpu:gloo,cuda:nccl') reduces CPU tensors on its gloo part
        if not any(b in backend for b in ("gloo", "mpi")):
            raise ValueError("plan_group must be a CPU (gloo) process group, got backend %r: create one with "
                             "torch.distributed.new_group(backend='gloo')" % backend)
        self.c0, self.c1, self.nglobal, self.group = int(c0), int(c1), int(nglobal), group
        head = [c for c in (0, 1) if c < self.nglobal and not c0 <= c < c1]
        self.gids = np.array(sorted(set(head) | set(range(self.c0, self.c1))), dtype=np.int64)
        # the ranks must cover every channel (else a portrait-wide max would
        # silently miss rows): the shards, gathered once per (group, shard)
        key = (id(group), self.c0, self.c1, self.nglobal)
        if key not in _COVERED:
            t = torch.tensor([self.c0, self.c1], dtype=torch.int64)
            parts = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
            dist.all_gather(parts, t, group=group)
            spans = sorted((int(a), int(b)) for a, b in (x.tolist() for x in parts))
            ok = spans[0][0] == 0 and spans[-1][1] == self.nglobal and all(
                spans[i][1] == spans[i + 1][0] for i in range(len(spans) - 1))
            if not ok:
                raise ValueError("plan_group shards %r do not partition the %d channels" % (spans, self.nglobal))
            _COVERED.add(key)

    def _reduce(self, vals, ops):
        out = []
        for v, op in zip(vals, ops):
            t = torch.tensor([v], dtype=torch.float64)
            dist.all_reduce(t, op=op, group=self.group)
            out.append(float(t.item()))
        return out

    def max(self, local_max):
        return self._reduce([float(local_max)], [dist.ReduceOp.MAX])[0]

    def any(self, flag):
        return self._reduce([1.0 if flag else 0.0], [dist.ReduceOp.MAX])[0] > 0.0

    def first_row(self, local_hits, local_rows):
        """The row of the smallest GLOBAL channel whose local flag is set (over
        every rank), copied from a rank that holds it; None when no rank has
        one.  ``local_hits``: bool per local row; ``local_rows``: [len(gids), K]."""
        import numpy as np
        hit = np.flatnonzero(np.asarray(local_hits))
        me, world = dist.get_rank(self.group), dist.get_world_size(self.group)
        # (smallest channel, then smallest rank holding it) in one MIN: g W + rank
        g = int(self.gids[hit[0]]) if hit.size else self.nglobal
        key = self._reduce([float(g * world + me)], [dist.ReduceOp.MIN])[0]
        gmin, owner = divmod(int(key), world)
        if gmin >= self.nglobal:
            return None
        K = np.asarray(local_rows).shape[1]
        buf = torch.zeros(K, dtype=torch.float64)
        if int(owner) == me:
            i = int(np.flatnonzero(self.gids == int(gmin))[0])
            buf.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(local_rows)[i], dtype=np.float64)))
        src = dist.get_global_rank(self.group, int(owner)) if self.group is not None else int(owner)
        dist.broadcast(buf, src=src, group=self.group)
        return buf.numpy()
