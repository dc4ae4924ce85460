"""Multi-GPU calls on one GPU: the byte-range decode of one frame (nxg_decode_range +
nxg_range_link, the per-rank half of nxg_decode_sharded) -- ids counting up (the length-run
decoder) and ids in any order (the single-pass decoder in range mode) -- and a one-rank RCCL
communicator.

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


@pytest.mark.parametrize("world", [2, 3, 8, 37])
@pytest.mark.parametrize("kind", ["perm", "perm35", "planted"])
def test_byte_ranges_random_order_ids(codec, world, kind):
    """Ids in any order (a batch updating an arbitrary subset of a publisher's values,
    publisher/mod.rs:776-845): record lengths vary record to record, the length-run probe
    declines, and each range is decoded by the single-pass decoder in range mode (its entry from
    the merge point of the 64 bytes before the range). Every row against the oracle; the ranges
    meet. `planted`: f64 values whose bytes read as record headers (false starts) everywhere."""
    import nxo
    from netidx_amd import synth
    n = 300_007
    ids, vals = synth.f64_columns(n, 111)
    rng = np.random.default_rng(world)
    if kind == "perm35":
        ids = rng.integers(0, 2**35, n, dtype=np.uint64)
    else:
        ids = rng.permutation(ids)
    if kind == "planted":  # each value's bytes: 0x0c 0x04 ... (a 12-byte record header)
        vals = (vals & np.uint64(0x0000ffffffffffff)) | np.uint64(0x0c04 << 48)
    wire = nxo.encode_f64(ids, vals)
    rngs, parts, offs, bad = _ranges_decode(codec, wire, world)
    assert bad is None and all(r.ok for r in rngs), [(r.ok, r.entry, r.exit) for r in rngs]
    got_id = np.concatenate([p["id"] for p in parts])
    got_val = np.concatenate([p["fixed"] for p in parts])
    o = nxo.decode(wire, cap_rows=n + 1, cap_children=1, cap_ctl=1).trim()
    assert np.array_equal(got_id, o["id"]) and np.array_equal(got_val, o["fixed"])
    assert rngs[0].entry == 0 and rngs[-1].exit == len(wire)
    for a, b in zip(rngs, rngs[1:]):
        assert a.exit == b.entry and b.begin <= b.entry < b.begin + 16


def _mixed_wire(n, seed, ctl=False):
    import nxo
    from netidx_amd import synth
    m = synth.mixed_columns(n, seed)
    d = nxo.Decoded(len(m.id), len(m.ctag) + 1, 1)
    for name in ("id", "tag", "fixed", "aux"):
        getattr(d, name)[:len(m.id)] = getattr(m, name)
    d.ctag[:len(m.ctag)] = m.ctag
    d.cfixed[:len(m.ctag)] = m.cfixed
    d.caux[:len(m.ctag)] = m.caux
    d.s.n_rows, d.s.n_children, d.s.n_ctl = len(m.id), len(m.ctag), 0
    w = nxo.encode(d, m.heap)
    if ctl:  # a Heartbeat (02 05) after every 97th message
        o = nxo.decode(np.frombuffer(w, np.uint8), cap_rows=n + 1, cap_children=len(m.ctag) + 1,
                       cap_ctl=1)
        b = np.frombuffer(w, np.uint8)
        parts, p = [], 0
        for k in range(n):
            L = int(b[p]) if b[p] < 0x80 else (int(b[p]) & 0x7f) | (int(b[p + 1]) << 7)
            parts.append(bytes(b[p:p + L]))
            if k % 97 == 96:
                parts.append(b"\x02\x05")
            p += L
        w = b"".join(parts)
    return np.frombuffer(w, np.uint8)


@pytest.mark.parametrize("world", [2, 3, 8, 37])
@pytest.mark.parametrize("ctl", [False, True])
def test_byte_ranges_mixed_frame(codec, world, ctl):
    """A config-3 mixed frame (i64 / f64 / string / datetime / array values, ids in any order;
    with `ctl` a Heartbeat every 97 messages) cut into byte ranges: the f64 decoders decline, the
    fast mixed decoder takes each range in range mode (tile 0's entry guessed from its
    candidates), the ranges meet, and every column of the concatenated ranges equals the
    oracle's decode of the whole frame (child indices are per range: offset by the children of
    the ranges before)."""
    import netidx_amd
    import nxo
    import torch
    from netidx_amd import shard
    from netidx_amd.codec import Columns
    n = 60_000
    wire = _mixed_wire(n, 57 + world, ctl)
    W = len(wire)
    dw = torch.from_numpy(wire.copy()).cuda()
    rngs, parts = [], []
    for r in range(world):
        b, e = shard.shard_range(W, world, r)
        cols = Columns.for_frame(max(e - b, 16) + 64, netidx_amd.LAYOUT_MIXED, "cuda")
        rng = codec.decode_range(dw, W, b, e, cols)
        if not rng.ok:  # a false guessed entry: decoded again from the predecessor's exit
            assert r > 0
            at = rngs[-1].exit
            rng = codec.decode_range(dw, W, min(at, e), e, cols)
            rng.begin = b
        rngs.append(rng)
        parts.append(cols.numpy())
    offs, bad = netidx_amd.range_link(rngs, W)
    assert bad is None and all(r.ok for r in rngs), [(r.ok, r.entry, r.exit) for r in rngs]
    o = nxo.decode(wire, cap_rows=n + 1, cap_children=8 * n + 1, cap_ctl=n + 1).trim()
    cat = {k: np.concatenate([p[k] for p in parts]) for k in ("id", "tag", "aux", "ctag",
                                                             "cfixed", "caux")}
    for k in ("id", "tag", "aux", "ctag", "cfixed", "caux"):
        assert np.array_equal(cat[k], o[k]), k
    coff, fixed = 0, []
    for p in parts:
        f = p["fixed"].copy()
        f[p["tag"] == 19] += np.uint64(coff)
        fixed.append(f)
        coff += len(p["ctag"])
    assert np.array_equal(np.concatenate(fixed), o["fixed"])
    if ctl:
        assert sum(len(p["ctl_row"]) for p in parts) == len(o["ctl_row"])
        assert np.array_equal(np.concatenate([p["ctl_off"] for p in parts]), o["ctl_off"])
    assert rngs[0].entry == 0 and rngs[-1].exit == W
    for a, b in zip(rngs, rngs[1:]):
        assert a.exit == b.entry


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


# ---- row shares (nxg_decode_share): nxg_decode_sharded's fallback ------------------------------

def _share_cols(codec, wire, shares, cols_of):
    """Every row share of one device frame, each into its own columns."""
    import torch
    dw = torch.from_numpy(np.ascontiguousarray(wire)).cuda()
    out = []
    for k in range(shares):
        cols = cols_of(k)
        off, st = codec.decode_share(dw, len(wire), k, shares, cols)
        out.append((off, st, cols.numpy() if st.err_kind == 0 else None))
    return out


def _check_shares(got, o, shares):
    import nxo
    rows = 0
    for k, (off, st, g) in enumerate(got):
        r0, want = nxo.share(o, k, shares)
        assert st.err_kind == 0 and off == r0 == rows
        assert st.n_rows == len(want["id"]) and st.n_heartbeat == want["n_heartbeat"]
        for f in ("id", "tag", "fixed", "aux", "ctag", "cfixed", "caux", "ctl_row", "ctl_off",
                  "ctl_len", "ctl_variant"):
            assert np.array_equal(g[f], want[f]), (k, f)
        assert g["n_heartbeat"] == want["n_heartbeat"]
        rows += st.n_rows
    assert rows == len(o["id"])


@pytest.mark.parametrize("shares", [1, 2, 3, 8, 37])
def test_decode_share_rich_frame(codec, shares):
    """Maps, nested arrays, Error(Value), Heartbeats, Unsubscribed, wide ids: the frame decoded
    whole (the general decoder) and cut into row shares, children and control spans re-based,
    against the oracle's decode cut by the restated contract (nxo.share)."""
    import netidx_amd
    import nxo
    from frames import rich_wire
    from netidx_amd.codec import Columns
    wire = rich_wire(20_000, 51)
    o = nxo.decode(wire).trim()
    assert o["err_kind"] == 0
    got = _share_cols(codec, wire, shares,
                      lambda k: Columns.for_frame(len(wire), netidx_amd.LAYOUT_MIXED, "cuda"))
    _check_shares(got, o, shares)


@pytest.mark.parametrize("shares", [3, 8])
def test_decode_share_f64_and_config3_frames(codec, shares):
    """The fast decoders' frames through the same call: an f64 frame (rows only, F64 layout)
    and a config-3 frame with Heartbeats and long strings."""
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    ids, vals = synth.f64_columns(300_001, 77)
    wire = nxo.encode_f64(ids, vals)
    got = _share_cols(codec, wire, shares,
                      lambda k: Columns(300_001 // shares + 2, 0, 0, netidx_amd.LAYOUT_F64, "cuda"))
    rows = 0
    for k, (off, st, g) in enumerate(got):
        assert st.err_kind == 0 and st.path == 1 and off == rows
        assert np.array_equal(g["id"], ids[off:off + st.n_rows])
        assert np.array_equal(g["fixed"], vals[off:off + st.n_rows])
        rows += st.n_rows
    assert rows == len(ids)
    wire = _mixed_wire(100_000, 5, ctl=True)
    o = nxo.decode(wire).trim()
    got = _share_cols(codec, wire, shares,
                      lambda k: Columns.for_frame(len(wire) // shares + 65536,
                                                  netidx_amd.LAYOUT_MIXED, "cuda"))
    _check_shares(got, o, shares)


def test_decode_share_errors_and_capacity(codec):
    """A frame error leaves no rows in any share (the oracle's kind and offset); a share larger
    than its columns reports NXG_CAPACITY; mixed content into f64 columns NXG_NOT_F64."""
    import netidx_amd
    import nxo
    import torch
    from frames import rich_wire
    from netidx_amd.codec import Columns
    wire = rich_wire(5000, 52, corrupt_at=3100)
    o = nxo.decode(wire).trim()
    assert o["err_kind"] == 1
    for k in range(3):
        cols = Columns.for_frame(len(wire), netidx_amd.LAYOUT_MIXED, "cuda")
        dw = torch.from_numpy(wire).cuda()
        off, st = codec.decode_share(dw, len(wire), k, 3, cols)
        assert (st.err_kind, st.err_offset, st.n_rows, off) == (o["err_kind"], o["err_offset"], 0, 0)
    wire = rich_wire(5000, 53)
    dw = torch.from_numpy(wire).cuda()
    small = Columns(100, 10_000, 10_000, netidx_amd.LAYOUT_MIXED, "cuda")
    off, st = codec.decode_share(dw, len(wire), 1, 4, small)
    assert st.err_kind == 7 and st.n_rows > 100  # NXG_CAPACITY, with the share's size
    f64 = Columns(5000, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    off, st = codec.decode_share(dw, len(wire), 0, 2, f64)
    assert st.err_kind == 8  # NXG_NOT_F64


def test_decode_range_mixed_capacity_is_reported(codec):
    """A mixed range declined because its columns are too small says so (err_kind NXG_CAPACITY),
    so nxg_decode_sharded reports the capacity, not an unsupported range."""
    import netidx_amd
    import torch
    from netidx_amd.codec import Columns
    wire = _mixed_wire(50_000, 6)
    dw = torch.from_numpy(np.ascontiguousarray(wire)).cuda()
    W = len(wire)
    small = Columns(1000, 100_000, 1000, netidx_amd.LAYOUT_MIXED, "cuda")
    rng = codec.decode_range(dw, W, 0, W // 2, small)
    assert rng.ok == 0 and rng.err_kind == 7
    big = Columns.for_frame(W, netidx_amd.LAYOUT_MIXED, "cuda")
    rng = codec.decode_range(dw, W, 0, W // 2, big)
    assert rng.ok == 1 and rng.err_kind == 0
