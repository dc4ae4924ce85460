"""Sharding over ranks (one process per GPU): torch.distributed mirrors of the library's RCCL
calls (include/nxg_codec.h: nxg_encode_allgather, nxg_decode_sharded), for gloo on CPU (the
multi-rank tests), for ranks that share one GPU (rehearsals: RCCL refuses two ranks on a
device), and as bench.py's fallback when librccl cannot be opened.

- Encode (BASELINE configs[4]): shards are encoded in rank order; after one all-gather of the
  shard sizes, every rank places its shard at its final byte offset and grouped point-to-point
  transfers deliver every shard to the same offsets on every rank. No padding, no compaction, one
  host read of the sizes. A netidx frame payload is a plain sequence of
  length-wrapped messages (netidx/src/channel.rs:177-202), so the shards in rank order are the
  batch's payload.
- Decode: one frame, cut into contiguous byte ranges. Each rank decodes the
  messages that START in its range (reading past its end); the ranges' summaries (entry, exit,
  rows) are all-gathered and linked by nxg_range_link; a range whose guessed entry is off the
  chain decodes again from its predecessor's exit (a true message start).
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


def shard_offsets(length, world, device="cpu"):
    """All-gather of the per-rank shard lengths; returns the byte offsets (world + 1 entries)."""
    import torch
    import torch.distributed as dist
    mine = torch.tensor([int(length)], dtype=torch.int64, device=device)
    lens = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(lens, mine) if device != "cpu" else \
        dist.all_gather(list(lens.split(1)), mine)
    off = np.zeros(world + 1, np.int64)
    off[1:] = np.cumsum(lens.cpu().numpy())
    return off


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


def link_ranges(mine, world):
    """All-gather of the ranges' summaries (NxgRange tuples) and nxg_range_link over them.
    Returns (row offsets, None) or (None, index of the first range off the chain)."""
    import torch.distributed as dist
    from . import codec
    allr = [None] * world
    dist.all_gather_object(allr, tuple(int(x) for x in mine))
    offs, bad = codec.range_link(allr, allr[-1][1])
    return offs, bad, allr


def decode_sharded(decode_range, frame_len, rank, world):
    """The byte-range decode protocol of nxg_decode_sharded over torch.distributed.

    decode_range(begin, end) decodes the messages that start in [begin, end) and returns its
    summary (NxgRange or a tuple: begin, end, entry, exit, n_rows, ok, err_kind). Returns
    (this rank's first global row, its final summary)."""
    def summary(r):
        return tuple(int(x) for x in (r.tuple() if hasattr(r, "tuple") else r))

    b, e = shard_range(frame_len, world, rank)
    mine = summary(decode_range(b, e))
    for _ in range(world + 1):
        offs, bad, allr = link_ranges(mine, world)
        if offs is not None:
            return int(offs[rank]), mine
        if any(r[5] == 0 for r in allr):
            raise RuntimeError("a range is not a homogeneous-f64 range: decode the whole frame")
        if bad == rank:
            if rank == 0:
                raise RuntimeError("the frame does not start with a message")
            at = 0
            for r in allr[:rank]:
                if r[0] != r[1]:
                    at = r[3]
            if at >= e:  # no message starts in this range: the chain passes through
                mine = (b, e, at, at, 0, 1, 0)
            else:
                mine = (b, e) + summary(decode_range(at, e))[2:]
    raise RuntimeError("the byte ranges of the frame do not link into one chain")
