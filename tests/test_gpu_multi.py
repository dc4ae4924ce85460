"""Multi-GPU calls on one GPU: the byte-range decode of one frame (nxg_decode_range +
nxg_range_link, the per-rank half of nxg_decode_sharded) and a one-rank RCCL communicator.

The ranges of a frame are decoded one after another here, as N ranks would decode them at once;
the cuts fall inside records (f64 records are 12-16 bytes), and the linked rows must be the
oracle's decode of the whole frame, bit for bit. RCCL refuses two ranks on one device, so the
N > 1 collectives are exercised by tests/test_multirank_cpu.py (gloo) and by bench.py on a node;
here nxg_comm_init / nxg_encode_allgather / nxg_decode_sharded run with one rank.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import torch
    import netidx_amd
    assert torch.cuda.is_available()
    c = netidx_amd.Codec(0)
    yield c
    c.close()


def _ranges_decode(codec, wire, world):
    import netidx_amd
    import torch
    from netidx_amd import shard
    from netidx_amd.codec import Columns
    W = len(wire)
    dw = torch.from_numpy(np.ascontiguousarray(wire)).cuda()
    rngs, parts = [], []
    for r in range(world):
        b, e = shard.shard_range(W, world, r)
        cols = Columns(max((e - b) // 12 + 2, 1), 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        rng = codec.decode_range(dw, W, b, e, cols)
        rngs.append(rng)
        parts.append(cols.numpy())
    offs, bad = netidx_amd.range_link(rngs, W)
    return rngs, parts, offs, bad


@pytest.mark.parametrize("world", [2, 3, 8, 37])
@pytest.mark.parametrize("kind", ["seq", "x28", "w35"])
def test_byte_ranges_decode_and_link(codec, world, kind):
    import nxo
    from netidx_amd import synth
    n = 400_003
    off = {"seq": 0, "x28": 2**28 - n // 2, "w35": 2**30}[kind]
    ids, vals = synth.f64_columns(n, 101, id_offset=off)
    wire = nxo.encode_f64(ids, vals)
    rngs, parts, offs, bad = _ranges_decode(codec, wire, world)
    assert bad is None and all(r.ok for r in rngs)
    got_id = np.concatenate([p["id"] for p in parts])
    got_val = np.concatenate([p["fixed"] for p in parts])
    o = nxo.decode(wire, cap_rows=n + 1, cap_children=1, cap_ctl=1).trim()
    assert np.array_equal(got_id, o["id"]) and np.array_equal(got_val, o["fixed"])
    assert [int(x) for x in offs] == list(np.cumsum([0] + [r.n_rows for r in rngs[:-1]]))
    # consecutive ranges meet; the first enters at 0, the last leaves at the frame end
    assert rngs[0].entry == 0 and rngs[-1].exit == len(wire)
    for a, b in zip(rngs, rngs[1:]):
        assert a.exit == b.entry and b.begin <= b.entry < b.begin + 16


def test_byte_ranges_tiny_frames(codec):
    """More ranges than records: empty ranges and ranges with no record start link through."""
    import nxo
    from netidx_amd import synth
    for n in (1, 2, 5):
        ids, vals = synth.f64_columns(n, 7)
        wire = nxo.encode_f64(ids, vals)
        rngs, parts, offs, bad = _ranges_decode(codec, wire, 11)
        assert bad is None
        assert np.array_equal(np.concatenate([p["fixed"] for p in parts]), vals)


def test_byte_ranges_irregular_frame_reports_not_ok(codec):
    """Record lengths varying record to record: the length-run decoder declines (ok = 0) and
    the caller decodes the whole frame."""
    import nxo
    from netidx_amd import synth
    n = 200_000
    ids, vals = synth.f64_columns(n, 9)
    ids = np.random.default_rng(3).permutation(ids)
    wire = nxo.encode_f64(ids, vals)
    rngs, parts, offs, bad = _ranges_decode(codec, wire, 2)
    assert not all(r.ok for r in rngs) and offs is None


def test_rccl_one_rank_comm(codec):
    import netidx_amd
    import nxo
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    comm = netidx_amd.Comm(codec, 1, 0, netidx_amd.Comm.unique_id())
    try:
        n = 300_000
        ids, vals = synth.f64_columns(n, 13)
        cols = netidx_amd.columns_from_arrays(ids, vals)
        out = torch.empty(16 * n, dtype=torch.uint8, device="cuda")
        W, offs = comm.encode_allgather(cols, None, out.data_ptr(), out.numel())
        ref = nxo.encode_f64(ids, vals)
        assert W == len(ref) and offs == [0]
        assert np.array_equal(out[:W].cpu().numpy(), ref)
        dec = Columns(n + 1, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        row_off, rng = comm.decode_sharded(out, W, dec)
        assert row_off == 0 and rng.n_rows == n and rng.exit == W
        g = dec.numpy()
        assert np.array_equal(g["id"], ids) and np.array_equal(g["fixed"], vals)
    finally:
        comm.close()
