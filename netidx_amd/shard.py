"""Sharding over ranks (one process per GPU): the record / byte split and the torch.distributed
transport that plugs into the library's own multi-rank protocols (nxg_multi.cpp) where RCCL
cannot serve -- gloo on CPU hosts, ranks sharing one GPU (RCCL refuses two ranks on a device).

The protocols themselves (config 5: every rank's shard encoded straight into its place and
delivered to every rank, nxg_encode_allgather; one frame decoded in byte ranges whose summaries
are linked, nxg_decode_sharded) live only in the library; this module hands them a transport
through nxg_comm_init_ops (Comm.with_ops): an all-gather of small host buffers and the grouped
send/recv of shards at their offsets.
"""
import numpy as np


def shard_range(total, world, rank):
    """[begin, end) of the records rank `rank` owns when `total` records go to `world` ranks
    (contiguous, balanced: sizes differ by at most one). Byte ranges of a frame use the same
    split."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of world {world}")
    return total * rank // world, total * (rank + 1) // world


def max_over_ranks(x, world, device="cpu"):
    """The maximum of a per-rank float (the job's time is its slowest rank's)."""
    if world == 1:
        return float(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allgather_at_offsets(out, off, rank, world):
    """`out` holds this rank's shard at [off[rank], off[rank+1]); afterwards it holds every
    shard at its offset (grouped send/recv, the same pattern as nxg_encode_allgather)."""
    import torch.distributed as dist
    ops = []
    mine = out[int(off[rank]):int(off[rank + 1])]
    for p in range(world):
        if p == rank:
            continue
        if len(mine):
            ops.append(dist.P2POp(dist.isend, mine, p))
        theirs = out[int(off[p]):int(off[p + 1])]
        if len(theirs):
            ops.append(dist.P2POp(dist.irecv, theirs, p))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return out


def gloo_comm(codec, world, rank, buffers):
    """Comm.with_ops over torch.distributed (gloo, already initialised): the library's protocols
    with this transport. `buffers`: the device tensors the protocols may all-gather shards of
    (the encode's output frame); they are staged through host memory."""
    import torch
    import torch.distributed as dist
    from .codec import Comm

    def allgather(mine):
        t = torch.frombuffer(bytearray(mine), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return b"".join(x.numpy().tobytes() for x in out)

    def allgatherv(buf_ptr, off, n, r):
        dev = [b for b in buffers if b.data_ptr() == buf_ptr]
        if not dev:
            raise ValueError("all-gather of a buffer the transport was not given")
        d = dev[0]
        torch.cuda.synchronize()
        host = d[: off[-1]].cpu()
        allgather_at_offsets(host, off, r, n)
        d[: off[-1]].copy_(host)
        torch.cuda.synchronize()

    return Comm.with_ops(codec, world, rank, allgather, allgatherv)
