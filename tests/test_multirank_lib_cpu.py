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
from frames import rich_wire
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


def _rank_share(rank, world, port, seed, decline_rank, fail_rank, corrupt_at, outdir,
                cap_rank=-1):
    import netidx_amd
    from netidx_amd.codec import NxgColumns
    _init(rank, world, port)
    try:
        wire = rich_wire(3000, seed, corrupt_at)
        W = len(wire)

        def decode_range(frame_ptr, flen, b, e, cols):
            # the byte-range decoders decline on rank `decline_rank` (-1: every rank)
            ok = 0 if decline_rank in (-1, rank) else 1
            return (b, e, b, e, 0, ok, 0)

        def decode_share(frame_ptr, flen, k, shares, cols):
            """nxg_decode_share's contract from the oracle: the frame whole, then row share k."""
            assert flen == W and frame_ptr == wire.ctypes.data and shares == world
            if rank == fail_rank:
                raise RuntimeError("this rank's share decode failed")
            if rank == cap_rank:  # this rank's share does not fit its columns (NXG_CAPACITY)
                return 0, 0, 7, 0
            o = nxo.decode(wire).trim()
            if o["err_kind"]:
                return 0, 0, o["err_kind"], o["err_offset"]
            r0, part = nxo.share(o, k, shares)
            np.savez(os.path.join(outdir, f"share{rank}.npz"), **part)
            return r0, len(part["id"]), 0, 0

        comm = netidx_amd.Comm.with_ops(None, world, rank, gloo_allgather(world), gloo_allgatherv,
                                        lambda c: 0, lambda c, p, n: 0, decode_range,
                                        decode_share)
        try:
            off, rng = comm.decode_sharded(wire.ctypes.data, W, NxgColumns())
            np.save(os.path.join(outdir, f"dec{rank}.npy"),
                    np.array([off] + list(rng.tuple()), dtype=np.uint64))
        except netidx_amd.CodecError as ex:
            with open(os.path.join(outdir, f"err{rank}.txt"), "w") as f:
                f.write(str(ex))
        comm.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,decline_rank", [(2, -1), (3, 1), (3, 0)])
def test_library_decode_sharded_falls_back_to_row_shares(tmp_path, world, decline_rank):
    """A range the byte-range decoders decline (ok = 0) on any rank: every rank takes its row
    share of the whole frame's decode (rng.ok = 2), and the shares put back together are the
    whole frame's decode."""
    mp.spawn(_rank_share, args=(world, _free_port(), 41, decline_rank, -1, None, str(tmp_path)),
             nprocs=world, join=True)
    whole = nxo.decode(rich_wire(3000, 41)).trim()
    assert whole["err_kind"] == 0 and len(whole["ctag"]) > 0 and len(whole["ctl_row"]) > 0
    rows = 0
    for r in range(world):
        assert not (tmp_path / f"err{r}.txt").exists()
        d = np.load(tmp_path / f"dec{r}.npy").astype(np.int64)
        off, ok, n_rows = int(d[0]), int(d[6]), int(d[5])
        assert ok == 2 and off == rows
        got = np.load(tmp_path / f"share{r}.npz")
        r0, want = nxo.share(whole, r, world)
        assert r0 == off and n_rows == len(want["id"])
        for k in want:
            if k != "n_heartbeat":
                assert np.array_equal(got[k], want[k]), k
        rows += n_rows
    assert rows == len(whole["id"])


def test_library_decode_sharded_share_reports_the_frame_error(tmp_path):
    """The frame fails as a whole: every rank reports the oracle's (kind, offset), no rows."""
    world = 3
    mp.spawn(_rank_share, args=(world, _free_port(), 42, -1, -1, 1500, str(tmp_path)),
             nprocs=world, join=True)
    whole = nxo.decode(rich_wire(3000, 42, 1500)).trim()
    assert whole["err_kind"] == 1  # UnknownTag
    for r in range(world):
        assert not (tmp_path / f"err{r}.txt").exists()
        d = np.load(tmp_path / f"dec{r}.npy").astype(np.int64)
        assert int(d[6]) == 2 and int(d[5]) == 0
        assert (int(d[7]), int(d[8])) == (whole["err_kind"], whole["err_offset"])


@pytest.mark.parametrize("fail_rank", [0, 2])
def test_library_decode_sharded_share_failure_on_every_rank(tmp_path, fail_rank):
    world = 3
    mp.spawn(_rank_share, args=(world, _free_port(), 43, 1, fail_rank, None, str(tmp_path)),
             nprocs=world, join=True)
    for r in range(world):
        msg = (tmp_path / f"err{r}.txt").read_text()
        assert not (tmp_path / f"dec{r}.npy").exists()
        if r != fail_rank:
            assert f"rank {fail_rank} failed" in msg


def test_library_decode_sharded_share_capacity_on_one_rank(tmp_path):
    """Only rank 1's row share overflows its columns (nxg_decode_share: true with NXG_CAPACITY):
    a local failure, so every rank returns false at the same step, instead of rank 1
    reporting ok = 2 with no rows while the others succeed."""
    world = 3
    mp.spawn(_rank_share, args=(world, _free_port(), 44, 1, -1, None, str(tmp_path), 1),
             nprocs=world, join=True)
    for r in range(world):
        msg = (tmp_path / f"err{r}.txt").read_text()
        assert not (tmp_path / f"dec{r}.npy").exists()
        if r != 1:
            assert "rank 1 failed" in msg
        else:
            assert "does not fit" in msg
