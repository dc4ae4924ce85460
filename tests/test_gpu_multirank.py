"""The library's multi-rank protocols (nxg_multi.cpp) with 2 and 3 processes sharing device 0,
each running the real kernels on its shard of a 10^7-record batch (BASELINE configs[4] at one
tenth of its size).

RCCL refuses two ranks on one device, so the transport is gloo behind nxg_comm_init_ops (device
buffers staged through host memory by the test's callbacks); everything else is the product:
each rank encodes its shard on the GPU straight into its place in the full frame
(nxg_encode_allgather), the full frame is then decoded in byte ranges, one per rank, by the
length-run kernels (nxg_decode_sharded), the summaries linked and the rows numbered. Checked: the
whole frame on every rank byte for byte against the oracle's encoder, and every rank's rows
against the batch's columns at its global row offset.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, total, outdir):
    import torch
    import torch.distributed as dist
    import netidx_amd
    import nxo
    from netidx_amd import shard, synth
    from netidx_amd.codec import Columns
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        codec = netidx_amd.Codec(0)
        b, e = shard.shard_range(total, world, rank)
        ids, vals = synth.f64_columns(e - b, synth.SEED_8GPU, id_offset=b)
        cols = netidx_amd.columns_from_arrays(ids, vals)
        cap = 15 * total + 64
        dout = torch.zeros(cap, dtype=torch.uint8, device="cuda")

        def allgather(mine):
            t = torch.frombuffer(bytearray(mine), dtype=torch.uint8)
            out = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(out, t)
            return b"".join(x.numpy().tobytes() for x in out)

        def allgatherv(buf_ptr, off, n, r):
            assert buf_ptr == dout.data_ptr()
            torch.cuda.synchronize()
            host = dout[: off[-1]].cpu()
            shard.allgather_at_offsets(host, off, r, n)
            dout[: off[-1]].copy_(host)
            torch.cuda.synchronize()

        comm = netidx_amd.Comm.with_ops(codec, world, rank, allgather, allgatherv)
        W, offs = comm.encode_allgather(cols, None, dout.data_ptr(), cap)
        all_ids, all_vals = synth.f64_columns(total, synth.SEED_8GPU)
        want = nxo.encode_f64(all_ids, all_vals)
        frame_ok = W == len(want) and np.array_equal(dout[:W].cpu().numpy(), want)
        del cols
        out = Columns((W // world) // 12 + 1024, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        row_off, rng = comm.decode_sharded(dout, W, out)
        n = int(rng.n_rows)
        got_id = out.id[:n].cpu().numpy().view(np.uint64)
        got_val = out.fixed[:n].cpu().numpy().view(np.uint64)
        rows_ok = np.array_equal(got_id, all_ids[row_off:row_off + n]) and \
            np.array_equal(got_val, all_vals[row_off:row_off + n])
        np.save(os.path.join(outdir, f"r{rank}.npy"),
                np.array([W, int(frame_ok), row_off, n, int(rows_ok), rng.begin, rng.end,
                          rng.entry, rng.exit] + list(offs), dtype=np.int64))
        comm.close()
        codec.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_library_protocols_on_real_kernels(tmp_path, world):
    import torch.multiprocessing as mp
    from netidx_amd import shard
    total = 10_000_000
    mp.spawn(_rank, args=(world, _free_port(), total, str(tmp_path)), nprocs=world, join=True)
    res = [np.load(tmp_path / f"r{r}.npy") for r in range(world)]
    W = int(res[0][0])
    rows = 0
    for r, x in enumerate(res):
        assert int(x[0]) == W and int(x[1]) == 1, f"rank {r}: the gathered frame differs"
        assert int(x[4]) == 1, f"rank {r}: its rows differ from the batch"
        assert int(x[2]) == rows  # row offsets number the ranges in order
        rows += int(x[3])
        assert (int(x[5]), int(x[6])) == shard.shard_range(W, world, r)
        assert list(x[9:]) == list(res[0][9:])  # every rank saw the same shard offsets
    assert rows == total
    assert int(res[0][7]) == 0 and int(res[-1][8]) == W
    for a, b in zip(res, res[1:]):
        assert int(a[8]) == int(b[7])  # each range leaves where the next enters


def _rank_mixed(rank, world, port, n_per, outdir):
    """Config 3 over the library protocols: each rank's shard of a mixed batch encoded straight
    into its place in the full frame (nxg_encode_allgather, the general encoder with the rank's
    text heap), then the frame decoded in byte ranges (nxg_decode_sharded: the fast mixed decoder
    in range mode, each range's entry guessed and linked, a range off the chain decoded again)."""
    import torch
    import torch.distributed as dist
    import netidx_amd
    import nxo
    from netidx_amd import shard, synth
    from netidx_amd.codec import Columns
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        codec = netidx_amd.Codec(0)
        m = synth.mixed_columns(n_per, 700 + rank)
        mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
        heap = torch.from_numpy(m.heap.copy()).cuda()
        cap = 64 * n_per * world + 4096
        dout = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        comm = shard.gloo_comm(codec, world, rank, [dout])
        W, offs = comm.encode_allgather(mc, heap, dout.data_ptr(), cap)
        frame = dout[:W].cpu().numpy()
        o = nxo.decode(frame, cap_rows=n_per * world + 1, cap_children=16 * n_per * world + 1,
                       cap_ctl=1).trim()
        out = Columns.for_frame(W // world + 4096, netidx_amd.LAYOUT_MIXED, "cuda")
        row_off, rng = comm.decode_sharded(dout, W, out)
        g = out.numpy()
        nr = int(rng.n_rows)
        sl = slice(row_off, row_off + nr)
        ok = all(np.array_equal(g[k], o[k][sl]) for k in ("id", "tag", "aux"))
        arr = g["tag"] == 19
        txt = ~arr
        ok &= np.array_equal(g["fixed"][txt], o["fixed"][sl][txt])
        if arr.any():
            c0 = int(o["fixed"][sl][arr][0]) - int(g["fixed"][arr][0])  # children before the range
            ok &= np.array_equal(g["fixed"][arr] + np.uint64(c0), o["fixed"][sl][arr])
            nc = len(g["ctag"])
            for k in ("ctag", "cfixed", "caux"):
                ok &= np.array_equal(g[k], o[k][c0:c0 + nc])
        np.save(os.path.join(outdir, f"m{rank}.npy"),
                np.array([W, row_off, nr, int(ok), rng.entry, rng.exit], dtype=np.int64))
        comm.close()
        codec.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_library_protocols_mixed_frame(tmp_path, world):
    import torch.multiprocessing as mp
    n_per = 300_000
    mp.spawn(_rank_mixed, args=(world, _free_port(), n_per, str(tmp_path)), nprocs=world,
             join=True)
    res = [np.load(tmp_path / f"m{r}.npy") for r in range(world)]
    rows = 0
    for r, x in enumerate(res):
        assert int(x[3]) == 1, f"rank {r}: its rows differ from the oracle's decode"
        assert int(x[1]) == rows
        rows += int(x[2])
    assert rows == n_per * world
    assert int(res[0][4]) == 0 and int(res[-1][5]) == int(res[0][0])
    for a, b in zip(res, res[1:]):
        assert int(a[5]) == int(b[4])


def _rank_rich(rank, world, port, outdir):
    """A frame the byte-range decoders decline (Maps, nested arrays, Error(Value), Unsubscribed,
    ids past 35 bits): nxg_decode_sharded falls back to row shares on every rank at once."""
    import torch
    import torch.distributed as dist
    import netidx_amd
    import nxo
    from frames import rich_wire
    from netidx_amd import shard
    from netidx_amd.codec import Columns
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        codec = netidx_amd.Codec(0)
        wire = rich_wire(30_000, 61)
        W = len(wire)
        dw = torch.from_numpy(wire).cuda()
        out = Columns.for_frame(W // world + 65536, netidx_amd.LAYOUT_MIXED, "cuda")
        comm = shard.gloo_comm(codec, world, rank, [dw])
        row_off, rng = comm.decode_sharded(dw, W, out)
        o = nxo.decode(wire).trim()
        r0, want = nxo.share(o, rank, world)
        g = out.numpy()
        ok = rng.ok == 2 and row_off == r0 and rng.n_rows == len(want["id"]) and all(
            np.array_equal(g[f], want[f]) for f in ("id", "tag", "fixed", "aux", "ctag",
                                                    "cfixed", "caux", "ctl_row", "ctl_off",
                                                    "ctl_len", "ctl_variant"))
        np.save(os.path.join(outdir, f"s{rank}.npy"),
                np.array([int(ok), row_off, rng.n_rows, len(o["id"])], dtype=np.int64))
        comm.close()
        codec.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_library_sharded_decode_falls_back_to_row_shares(tmp_path, world):
    import torch.multiprocessing as mp
    mp.spawn(_rank_rich, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [np.load(tmp_path / f"s{r}.npy") for r in range(world)]
    rows = 0
    for r, x in enumerate(res):
        assert int(x[0]) == 1, f"rank {r}: its row share differs from the oracle's"
        assert int(x[1]) == rows
        rows += int(x[2])
    assert rows == int(res[0][3])


def _rank_config5(rank, world, port, total, want_path, outdir):
    """BASELINE configs[4] at its own size and width: 10^8 f64 records (seed 0x5EED0005) over 8
    ranks sharing device 0. Each rank's 1.25*10^7-record shard is encoded on the GPU straight
    into its place in the 1.498 GB frame (nxg_encode_allgather), the frame checked byte for byte
    against the oracle's encoder, then decoded in 8 byte ranges (nxg_decode_sharded) and every
    rank's rows checked against the batch at its global offset."""
    import torch
    import torch.distributed as dist
    import netidx_amd
    from netidx_amd import shard, synth
    from netidx_amd.codec import Columns
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        codec = netidx_amd.Codec(0)

        def say(msg):  # progress (a quiet minute reads as a hang on the GPU box)
            if rank == 0:
                print(f"config5: {msg}", flush=True)

        b, e = shard.shard_range(total, world, rank)
        ids, vals = synth.f64_columns(e - b, synth.SEED_8GPU, id_offset=b)
        cols = netidx_amd.columns_from_arrays(ids, vals)
        del ids, vals
        want = np.load(want_path, mmap_mode="r")
        say("shards built")
        cap = len(want) + 64
        dout = torch.zeros(cap, dtype=torch.uint8, device="cuda")
        comm = shard.gloo_comm(codec, world, rank, [dout])
        W, offs = comm.encode_allgather(cols, None, dout.data_ptr(), cap)
        say(f"encoded and gathered: {W} bytes")
        del cols
        host = dout[:W].cpu().numpy()
        frame_ok = W == len(want) and np.array_equal(host, want)
        del host
        say(f"frame checked: {frame_ok}")
        out = Columns((W // world) // 12 + 1024, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        row_off, rng = comm.decode_sharded(dout, W, out)
        say(f"decoded: rows {row_off}..{row_off + int(rng.n_rows)}")
        n = int(rng.n_rows)
        ids, vals = synth.f64_columns(n, synth.SEED_8GPU, id_offset=row_off)
        rows_ok = rng.ok == 1 and \
            np.array_equal(out.id[:n].cpu().numpy().view(np.uint64), ids) and \
            np.array_equal(out.fixed[:n].cpu().numpy().view(np.uint64), vals)
        np.save(os.path.join(outdir, f"c{rank}.npy"),
                np.array([W, int(frame_ok), row_off, n, int(rows_ok), rng.begin, rng.end,
                          rng.entry, rng.exit] + list(offs), dtype=np.int64))
        comm.close()
        codec.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_config5_full_size_eight_ranks(tmp_path):
    """configs[4] as BASELINE.json names it: 10^8 records, 8 ranks (processes sharing the one
    GPU of this pool; gloo behind NxgCommOps, since RCCL refuses two ranks on one device)."""
    import torch.multiprocessing as mp
    import nxo
    from netidx_amd import shard, synth
    total, world = 100_000_000, 8
    ids, vals = synth.f64_columns(total, synth.SEED_8GPU)
    want = nxo.encode_f64(ids, vals)
    del ids, vals
    assert len(want) == 1_497_886_336
    want_path = str(tmp_path / "want.npy")
    np.save(want_path, want)
    del want
    mp.spawn(_rank_config5, args=(world, _free_port(), total, want_path, str(tmp_path)),
             nprocs=world, join=True)
    res = [np.load(tmp_path / f"c{r}.npy") for r in range(world)]
    W = int(res[0][0])
    rows = 0
    for r, x in enumerate(res):
        assert int(x[0]) == W == 1_497_886_336 and int(x[1]) == 1, \
            f"rank {r}: the gathered frame differs from the oracle's"
        assert int(x[4]) == 1, f"rank {r}: its rows differ from the batch"
        assert int(x[2]) == rows
        rows += int(x[3])
        assert (int(x[5]), int(x[6])) == shard.shard_range(W, world, r)
        assert list(x[9:]) == list(res[0][9:])
    assert rows == total
    assert int(res[0][7]) == 0 and int(res[-1][8]) == W
    for a, b in zip(res, res[1:]):
        assert int(a[8]) == int(b[7])
