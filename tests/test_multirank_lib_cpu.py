"""The library's own multi-rank protocols (nxg_multi.cpp: nxg_encode_allgather,
nxg_decode_sharded) on the CPU, world size 2 and 3, one process per rank.

The communicator is nxg_comm_init_ops: the transport is gloo (torch.distributed) behind the
NxgCommOps callbacks, and the local codec -- on a GPU node the ctx's kernels -- is the oracle
(the checker) behind the codec hooks, because this container has no GPU. Everything between the
callbacks is the product's C++: the size exchange and offsets, the capacity check, the agreed
failures, the range summaries, nxg_range_link, the re-decode of a range whose first entry is off
the chain (the "liar"), and the row numbering.

The failure cases check the fix for a protocol that used to return on one rank only: every rank
must return false at the same step (a hang fails the test by its timeout).
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import nxo
from netidx_amd import shard, synth

pytestmark = pytest.mark.timeout(240)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def gloo_allgather(world):
    def allgather(mine):
        t = torch.frombuffer(bytearray(mine), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        return b"".join(x.numpy().tobytes() for x in out)
    return allgather


def host_view(ptr, n):
    return torch.from_numpy(np.ctypeslib.as_array((C.c_uint8 * max(n, 1)).from_address(ptr)))[:n]


def gloo_allgatherv(buf_ptr, off, n, r):
    shard.allgather_at_offsets(host_view(buf_ptr, off[-1]), off, r, n)


def _starts(wire):
    st, p = [], 0
    while p < len(wire):
        st.append(p)
        p += int(wire[p])
    return np.array(st, np.int64)


def _rank_encode(rank, world, port, total, fail_rank, small_cap_rank, outdir):
    import netidx_amd
    from netidx_amd.codec import NxgColumns
    _init(rank, world, port)
    try:
        b, e = shard.shard_range(total, world, rank)
        ids, vals = synth.f64_columns(e - b, synth.SEED_8GPU, id_offset=b)
        wire = nxo.encode_f64(ids, vals)

        def encoded_len(cols):
            if rank == fail_rank:
                raise RuntimeError("this rank cannot size its shard")
            return len(wire)

        def encode(cols, out_ptr, cap):
            assert cap >= len(wire)
            C.memmove(out_ptr, wire.ctypes.data, len(wire))
            return len(wire)

        comm = netidx_amd.Comm.with_ops(None, world, rank, gloo_allgather(world), gloo_allgatherv,
                                        encoded_len, encode, lambda *a: None)
        cap = 16 * total + 64
        if rank == small_cap_rank:
            cap = 10
        out = np.zeros(cap, np.uint8)
        try:
            W, offs = comm.encode_allgather(NxgColumns(), None, out.ctypes.data, cap)
            np.save(os.path.join(outdir, f"full{rank}.npy"), out[:W])
            np.save(os.path.join(outdir, f"offs{rank}.npy"), np.array(offs, np.int64))
        except netidx_amd.CodecError as ex:
            with open(os.path.join(outdir, f"err{rank}.txt"), "w") as f:
                f.write(str(ex))
        comm.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 20_011), (3, 9_999)])
def test_library_encode_allgather(tmp_path, world, total):
    mp.spawn(_rank_encode, args=(world, _free_port(), total, -1, -1, str(tmp_path)),
             nprocs=world, join=True)
    ids, vals = synth.f64_columns(total, synth.SEED_8GPU)
    want = nxo.encode_f64(ids, vals)
    sizes = [len(nxo.encode_f64(*synth.f64_columns(e - b, synth.SEED_8GPU, id_offset=b)))
             for b, e in (shard.shard_range(total, world, r) for r in range(world))]
    for r in range(world):
        assert not (tmp_path / f"err{r}.txt").exists()
        assert np.load(tmp_path / f"full{r}.npy").tobytes() == want.tobytes()
        assert list(np.load(tmp_path / f"offs{r}.npy")) == list(np.cumsum([0] + sizes[:-1]))


@pytest.mark.parametrize("world,fail_rank,small_cap_rank", [(2, 1, -1), (3, 0, -1), (3, -1, 2)])
def test_library_encode_allgather_fails_on_every_rank(tmp_path, world, fail_rank,
                                                      small_cap_rank):
    mp.spawn(_rank_encode, args=(world, _free_port(), 3001, fail_rank, small_cap_rank,
                                 str(tmp_path)), nprocs=world, join=True)
    culprit = fail_rank if fail_rank >= 0 else small_cap_rank
    for r in range(world):
        msg = (tmp_path / f"err{r}.txt").read_text()
        assert not (tmp_path / f"full{r}.npy").exists()
        if r != culprit:
            assert f"rank {culprit} failed" in msg


def _rank_decode(rank, world, port, total, seed, liar, fail_rank, outdir):
    import netidx_amd
    from netidx_amd.codec import NxgColumns
    _init(rank, world, port)
    try:
        ids, vals = synth.f64_columns(total, seed)
        wire = nxo.encode_f64(ids, vals)
        W = len(wire)
        starts = _starts(wire)
        calls = []

        def decode_range(frame_ptr, flen, b, e, cols):
            """The GPU range decode's contract restated from the oracle's chain; rank `liar`
            first guesses an entry inside a record."""
            assert flen == W and frame_ptr == wire.ctypes.data
            if rank == fail_rank:
                raise RuntimeError("this rank's range decode failed")
            i0 = int(np.searchsorted(starts, b))
            i1 = int(np.searchsorted(starts, e))
            entry = int(starts[i0]) if i0 < len(starts) else W
            exit_ = int(starts[i1]) if i1 < len(starts) else W
            rows = i1 - i0
            if rank == liar and not calls:
                entry, exit_, rows = entry + 3, exit_ + 5, rows - 1
            calls.append((b, e))
            o = nxo.decode(wire[entry:exit_], cap_children=1, cap_ctl=1).trim()
            np.save(os.path.join(outdir, f"rows{rank}.npy"), o["fixed"])
            return (b, e, entry, exit_, rows, 1, 0)

        comm = netidx_amd.Comm.with_ops(None, world, rank, gloo_allgather(world), gloo_allgatherv,
                                        lambda c: 0, lambda c, p, n: 0, decode_range)
        try:
            off, rng = comm.decode_sharded(wire.ctypes.data, W, NxgColumns())
            np.save(os.path.join(outdir, f"dec{rank}.npy"),
                    np.array([off, len(calls)] + list(rng.tuple()), dtype=np.int64))
        except netidx_amd.CodecError as ex:
            with open(os.path.join(outdir, f"err{rank}.txt"), "w") as f:
                f.write(str(ex))
        comm.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total,liar", [(2, 30_001, -1), (3, 20_000, 1), (3, 20_000, 2),
                                              (2, 5000, 1)])
def test_library_decode_sharded_links_and_redecodes(tmp_path, world, total, liar):
    mp.spawn(_rank_decode, args=(world, _free_port(), total, 91, liar, -1, str(tmp_path)),
             nprocs=world, join=True)
    ids, vals = synth.f64_columns(total, 91)
    W = len(nxo.encode_f64(ids, vals))
    got = []
    for r in range(world):
        assert not (tmp_path / f"err{r}.txt").exists()
        d = np.load(tmp_path / f"dec{r}.npy")
        off, ncalls, rng = int(d[0]), int(d[1]), d[2:]
        b, e = shard.shard_range(W, world, r)
        assert (int(rng[0]), int(rng[1])) == (b, e)
        assert ncalls == (2 if r == liar else 1)  # the liar decoded again, from the true chain
        rows = np.load(tmp_path / f"rows{r}.npy")
        assert off == len(got) and len(rows) == int(rng[4])
        got.extend(rows.tolist())
    assert np.array_equal(np.array(got, np.uint64), vals)  # every record once, in order


@pytest.mark.parametrize("world,fail_rank,liar", [(2, 0, -1), (3, 2, -1), (3, 1, -1)])
def test_library_decode_sharded_fails_on_every_rank(tmp_path, world, fail_rank, liar):
    mp.spawn(_rank_decode, args=(world, _free_port(), 9000, 92, liar, fail_rank, str(tmp_path)),
             nprocs=world, join=True)
    for r in range(world):
        msg = (tmp_path / f"err{r}.txt").read_text()
        assert not (tmp_path / f"dec{r}.npy").exists()
        if r != fail_rank:
            assert f"rank {fail_rank} failed" in msg
