"""Sharding of a batch over ranks (one process per GPU), for bench.py and the multi-rank tests.

The decode path shards with no data-path collective: each rank owns a contiguous range of the
records (a frame of its own, ids disjoint) and decodes it alone ("weak" scaling). The only
exchange is config 5's: each rank encodes its shard and an all-gather assembles the full frame
on every rank. A netidx frame payload is a plain sequence of length-wrapped messages
(netidx/src/channel.rs:177-202 writes them back to back), so the concatenation of the shards'
payloads in rank order is the payload of the whole batch.

Everything here is device-agnostic torch.distributed code: RCCL ("nccl") with GPU tensors in
bench.py, gloo with CPU tensors in tests/test_multirank_cpu.py.
"""


def shard_range(total, world, rank):
    """[begin, end) of the records rank `rank` owns when `total` records go to `world` ranks
    (contiguous, balanced: sizes differ by at most one)."""
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


def gather_frames(local, length, world):
    """All-gather of per-rank frame payloads of different lengths.

    `local` is a uint8 tensor holding this rank's payload in its first `length` bytes (it may
    be longer). Returns (full, lengths): `full` is a uint8 tensor on local's device with the
    payloads of ranks 0..world-1 back to back, `lengths` the per-rank byte counts. The payloads
    travel padded to the longest one, in one all-gather."""
    import torch
    import torch.distributed as dist
    dev = local.device
    mine = torch.tensor([int(length)], dtype=torch.int64, device=dev)
    lens = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(lens, mine)
    lengths = [int(t.item()) for t in lens]
    mx = max(lengths)
    send = torch.zeros(mx, dtype=torch.uint8, device=dev)
    send[:length] = local[:length]
    parts = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(parts, send)
    full = torch.cat([p[:n] for p, n in zip(parts, lengths)])
    return full, lengths
