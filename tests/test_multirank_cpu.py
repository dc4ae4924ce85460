"""Multi-rank protocols on the CPU: gloo, world size 2 and 3, one process per rank.

bench.py --gpus N runs one process per GPU; the library's RCCL calls (nxg_encode_allgather,
nxg_decode_sharded) and their torch.distributed mirrors in netidx_amd/shard.py follow the same
protocols, checked here over gloo with the oracle standing in for the per-rank GPU kernels:

- config 5's encode: shards encoded in rank order, one all-gather of their sizes, every shard
  delivered at its final byte offset by grouped send/recv; every rank ends with exactly the whole
  batch's frame (the oracle decodes it: every id and value in order);
- one frame decoded in byte ranges: each rank takes the messages that start in its range,
  nxg_range_link (the product's host code) links the ranges' summaries and numbers their rows,
  including cuts inside records and a rank whose first guess at its entry is off the chain (it
  decodes again from its predecessor's exit);
- the timing reduction takes the slowest rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import nxo
from netidx_amd import shard, synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _rank_encode(rank, world, port, total, outdir):
    _init(rank, world, port)
    try:
        b, e = shard.shard_range(total, world, rank)
        ids, vals = synth.f64_columns(e - b, synth.SEED_8GPU, id_offset=b)
        wire = nxo.encode_f64(ids, vals)
        off = shard.shard_offsets(len(wire), world)
        out = torch.zeros(int(off[-1]), dtype=torch.uint8)
        out[int(off[rank]):int(off[rank + 1])] = torch.from_numpy(wire)  # the shard in place
        shard.allgather_at_offsets(out, off, rank, world)
        slowest = shard.max_over_ranks(0.25 + rank, world)
        np.save(os.path.join(outdir, f"full{rank}.npy"), out.numpy())
        np.save(os.path.join(outdir, f"meta{rank}.npy"),
                np.array([b, e, len(wire), slowest] + list(np.diff(off)), dtype=np.float64))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 20_011), (3, 9_999)])
def test_encode_allgather_at_offsets_rebuilds_the_whole_batch(tmp_path, world, total):
    mp.spawn(_rank_encode, args=(world, _free_port(), total, str(tmp_path)), nprocs=world,
             join=True)
    ids, vals = synth.f64_columns(total, synth.SEED_8GPU)
    want = nxo.encode_f64(ids, vals)
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    assert [int(m[0]) for m in metas] == [shard.shard_range(total, world, r)[0]
                                          for r in range(world)]
    assert int(metas[0][0]) == 0 and int(metas[-1][1]) == total
    for r in range(world):
        full = np.load(tmp_path / f"full{r}.npy")
        assert full.tobytes() == want.tobytes()  # every rank: the single-process frame
        assert float(metas[r][3]) == 0.25 + (world - 1)  # max over ranks
        assert [int(x) for x in metas[r][4:]] == [int(m[2]) for m in metas]
    d = nxo.decode(want, cap_rows=total + 1, cap_children=1, cap_ctl=1)
    assert d.s.err_kind == 0 and d.s.n_rows == total
    t = d.trim()
    assert np.array_equal(t["id"], ids) and np.array_equal(t["fixed"], vals)


def _starts(wire):
    """Message start offsets of a frame (the oracle's chain: each length prefix is the message
    length, netidx-core/src/pack.rs:537-555; f64 records are < 128 bytes: one-byte prefixes)."""
    st, p = [], 0
    while p < len(wire):
        st.append(p)
        p += int(wire[p])
    return np.array(st, np.int64)


def _rank_decode(rank, world, port, total, seed, liar, outdir):
    _init(rank, world, port)
    try:
        ids, vals = synth.f64_columns(total, seed)
        wire = nxo.encode_f64(ids, vals)
        W = len(wire)
        starts = _starts(wire)
        calls = []

        def decode_range(b, e):
            """The GPU range decode's contract, restated from the oracle's chain: messages that
            start in [b, e); entry = first start >= b, exit = first start >= e (or W). Rank
            `liar` first guesses an entry inside a record (as a false record header would)."""
            i0 = int(np.searchsorted(starts, b))
            i1 = int(np.searchsorted(starts, e))
            entry = int(starts[i0]) if i0 < len(starts) else W
            exit_ = int(starts[i1]) if i1 < len(starts) else W
            rows = i1 - i0
            if rank == liar and not calls:
                entry, exit_, rows = entry + 3, exit_ + 5, rows - 1
            calls.append((b, e))
            o = nxo.decode(wire[entry:exit_] if rank != liar or len(calls) > 1 else wire[:0],
                           cap_children=1, cap_ctl=1).trim()
            np.save(os.path.join(outdir, f"rows{rank}.npy"), o["fixed"])
            return (b, e, entry, exit_, rows, 1, 0)

        off, mine = shard.decode_sharded(decode_range, W, rank, world)
        np.save(os.path.join(outdir, f"dec{rank}.npy"),
                np.array([off, len(calls)] + list(mine), dtype=np.int64))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,liar", [(2, 30_001, -1), (3, 20_000, 1), (2, 5000, 1)])
def test_decode_byte_ranges_link_and_number_rows(tmp_path, world, total, liar):
    mp.spawn(_rank_decode, args=(world, _free_port(), total, 91, liar, str(tmp_path)),
             nprocs=world, join=True)
    ids, vals = synth.f64_columns(total, 91)
    W = len(nxo.encode_f64(ids, vals))
    got = []
    for r in range(world):
        d = np.load(tmp_path / f"dec{r}.npy")
        off, ncalls, rng = int(d[0]), int(d[1]), d[2:]
        b, e = shard.shard_range(W, world, r)
        assert (int(rng[0]), int(rng[1])) == (b, e)
        assert ncalls == (2 if r == liar else 1)  # the liar decoded again, from the true chain
        rows = np.load(tmp_path / f"rows{r}.npy")
        assert off == len(got) and len(rows) == int(rng[4])
        got.extend(rows.tolist())
    assert np.array_equal(np.array(got, np.uint64), vals)  # every record once, in order


def test_shard_range_partitions():
    for total in (0, 1, 7, 10_000_000, 100_000_000):
        for world in (1, 2, 3, 4, 8):
            spans = [shard.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1
            assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_max_over_ranks_single_process():
    assert shard.max_over_ranks(3.5, 1) == 3.5
