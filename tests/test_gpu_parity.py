"""GPU parity: the HIP codec vs the CPU oracle and the golden fixtures, through the C ABI.

Bar: bit-exact columns, identical (PackError kind, first failing message offset), and
byte-identical re-encoding. At the BASELINE sizes the check is the size-independent round trip
encode -> decode -> encode plus a sampled oracle comparison.
"""
import json
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "manifest.json")))


@pytest.fixture(scope="module")
def codec():
    import torch
    import netidx_amd
    assert torch.cuda.is_available()
    c = netidx_amd.Codec(0)
    yield c
    c.close()


def gpu_decode(codec, wire, layout=None, flags=0, host=False):
    import torch
    import netidx_amd
    from netidx_amd.codec import Columns
    n = len(wire)
    layout = layout or netidx_amd.LAYOUT_MIXED
    cols = Columns.for_frame(n, layout, "cpu" if host else "cuda")
    if host:
        frame = np.frombuffer(bytes(wire), np.uint8)
    else:
        frame = torch.from_numpy(np.frombuffer(bytes(wire), np.uint8).copy()).cuda()
    st = codec.decode_into(frame, n, cols, flags, check=False)
    return cols, st


def as_rows(d, n=None):
    return [list(map(int, r)) for r in zip(d["id"], d["tag"], d["fixed"], d["aux"])]


def assert_same_as_oracle(cols, st, wire, big_caps=False):
    """big_caps: the oracle gets room for every child an invalid frame may announce (16 per
    remaining byte, the ValArray guard), so that its first error is a decode error, as the
    reference's (which has no capacity) -- not a capacity error met on the way."""
    import nxo
    o = (nxo.decode(wire, cap_children=16 * len(wire) + 16) if big_caps else nxo.decode(wire)).trim()
    assert (st.err_kind, st.err_offset if st.err_kind else 0) == (o["err_kind"], o["err_offset"])
    if st.err_kind:
        return
    g = cols.numpy()
    assert st.n_rows == len(o["id"])
    assert np.array_equal(g["id"], o["id"])
    assert np.array_equal(g["fixed"], o["fixed"])
    assert np.array_equal(g["tag"], o["tag"])
    if "aux" in g:
        assert np.array_equal(g["aux"], o["aux"])
        for k in ("ctag", "cfixed", "caux", "ctl_row", "ctl_off", "ctl_len", "ctl_variant"):
            assert np.array_equal(g[k], o[k]), k
        assert st.n_heartbeat == o["n_heartbeat"]


# ---- golden fixtures ----------------------------------------------------------------------------
@pytest.mark.parametrize("b", MANIFEST["batches"], ids=lambda b: b["name"])
def test_golden_batches(codec, b):
    wire = open(os.path.join(GOLD, b["file"]), "rb").read()
    cols, st = gpu_decode(codec, wire)
    assert st.err_kind == 0
    g = cols.numpy()
    e = b["expect"]
    assert as_rows(g) == e["rows"]
    if "aux" in g:
        assert [list(map(int, r)) for r in zip(g["ctag"], g["cfixed"], g["caux"])] == e["children"]
        assert [list(map(int, r)) for r in zip(g["ctl_row"], g["ctl_off"], g["ctl_len"],
                                               g["ctl_variant"])] == e["ctl"]
    assert st.n_heartbeat == e["n_heartbeat"]
    # the homogeneous batches must take the f64 kernel
    if b["name"].startswith("f64_") and max(r[0] for r in e["rows"]) < 2**28:
        assert st.path == 1
    # byte-identical re-encode from the decoded columns (heap = the frame itself)
    import torch
    heap = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).cuda()
    out = codec.encode_batch(cols, heap)
    assert out.cpu().numpy().tobytes() == wire


@pytest.mark.parametrize("c", MANIFEST["errors"], ids=lambda c: c["name"])
def test_golden_errors(codec, c):
    wire = bytes.fromhex(c["hex"])
    cols, st = gpu_decode(codec, wire)
    assert (st.err_kind, st.err_offset) == (c["kind"], c["offset"])


@pytest.mark.parametrize("c", MANIFEST["edge_ok"], ids=lambda c: c["name"])
def test_golden_edge_ok(codec, c):
    wire = bytes.fromhex(c["hex"])
    cols, st = gpu_decode(codec, wire)
    assert st.err_kind == 0
    assert as_rows(cols.numpy()) == c["rows"]


# ---- f64 fast path ---------------------------------------------------------------------------
def f64_wire(n, seed, id_offset=0):
    from netidx_amd import synth
    import nxo
    ids, vals = synth.f64_columns(n, seed, id_offset)
    return ids, vals, nxo.encode_f64(ids, vals).tobytes()


@pytest.mark.parametrize("n", [0, 1, 2, 7, 1000, 1365, 1366, 1367, 4096, 100_003])
def test_f64_sizes(codec, n):
    import netidx_amd
    ids, vals, wire = f64_wire(n, 11 + n)
    for layout in (netidx_amd.LAYOUT_F64, netidx_amd.LAYOUT_MIXED):
        cols, st = gpu_decode(codec, wire, layout)
        assert st.err_kind == 0 and st.n_rows == n
        g = cols.numpy()
        assert np.array_equal(g["id"], ids) and np.array_equal(g["fixed"], vals)
        if n:
            assert st.path == 1


def test_f64_id_widths_and_tile_edges(codec):
    """ids of 1..4 varint bytes shift record boundaries across every 16 KiB tile edge."""
    import nxo
    rng = np.random.default_rng(5)
    n = 60_000
    ids = rng.choice(np.array([0, 127, 128, 16383, 16384, 2**21 - 1, 2**21, 2**28 - 1],
                              np.uint64), n)
    vals = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    wire = nxo.encode_f64(ids, vals).tobytes()
    cols, st = gpu_decode(codec, wire)
    assert st.path == 1
    assert_same_as_oracle(cols, st, wire)


def test_f64_adversarial_payloads_fall_back_exactly(codec):
    """f64 payload bytes that look like record headers (0x0c 0x04 .. 0x09) must not fool the
    merge-point search; anything unprovable falls back to the general kernel."""
    import nxo
    n = 50_000
    ids = np.arange(n, dtype=np.uint64)
    # payload = 0c 04 00 09 0c 04 00 09 in every value: fake records everywhere
    vals = np.full(n, 0x0C0400090C040009, np.uint64)
    vals[::7] = 0x0D04800109000000
    wire = nxo.encode_f64(ids, vals).tobytes()
    cols, st = gpu_decode(codec, wire)
    assert_same_as_oracle(cols, st, wire)


def test_f64_with_heartbeat_falls_back(codec):
    import netidx_amd
    ids, vals, wire = f64_wire(5000, 3)
    wire = wire[:12 * 100] + b"\x02\x05" + wire[12 * 100:]
    cols, st = gpu_decode(codec, wire)
    assert st.path == 2
    assert_same_as_oracle(cols, st, wire)
    # F64-only columns cannot hold a control message
    cols, st = gpu_decode(codec, wire, netidx_amd.LAYOUT_F64)
    assert st.err_kind == netidx_amd.NOT_F64


def test_f64_error_position(codec):
    ids, vals, wire = f64_wire(20_000, 9)
    w = bytearray(wire)
    w[150_001] = 0xFF  # corrupt somewhere in the middle
    cols, st = gpu_decode(codec, bytes(w))
    assert_same_as_oracle(cols, st, bytes(w))


def test_f64_truncated_frame(codec):
    ids, vals, wire = f64_wire(20_000, 10)
    for cut in (1, 5, 11, 13):
        w = wire[:-cut]
        cols, st = gpu_decode(codec, w)
        assert_same_as_oracle(cols, st, w)


# ---- general path ---------------------------------------------------------------------------
def mixed_wire(n, seed):
    from netidx_amd import synth
    import nxo
    m = synth.mixed_columns(n, seed)
    d = nxo.Decoded(n, len(m.ctag) + 1, 1)
    s = d.s
    for name in ("id", "tag", "fixed", "aux"):
        getattr(d, name)[:n] = getattr(m, name)
    d.ctag[:len(m.ctag)] = m.ctag
    d.cfixed[:len(m.ctag)] = m.cfixed
    d.caux[:len(m.ctag)] = m.caux
    s.n_rows, s.n_children, s.n_ctl = n, len(m.ctag), 0
    return m, nxo.encode(d, m.heap)


@pytest.mark.parametrize("n", [1, 10, 5000, 200_000])
def test_mixed_vs_oracle(codec, n):
    m, wire = mixed_wire(n, 100 + n)
    cols, st = gpu_decode(codec, wire)
    assert st.path in (2, 4) and st.err_kind == 0  # 4 unless a recent frame fell back
    assert_same_as_oracle(cols, st, wire)


def test_mixed_host_memory_paths(codec):
    m, wire = mixed_wire(20_000, 77)
    cols, st = gpu_decode(codec, wire, host=True)
    assert_same_as_oracle(cols, st, wire)


def test_mixed_encode_from_columns_matches_oracle(codec):
    import netidx_amd
    import torch
    m, wire = mixed_wire(50_000, 55)
    cols = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    out = codec.encode_batch(cols, heap)
    assert out.cpu().numpy().tobytes() == wire


def test_random_messages_python_twin(codec):
    """Every Value tag, control messages, nesting (the golden twin's generator) at scale."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mg", os.path.join(GOLD, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    rng = random.Random(99)
    msgs = []
    for i in range(4000):
        k = rng.random()
        if k < 0.05:
            msgs.append(("hb",))
        elif k < 0.08:
            msgs.append(("raw", 2, mg.enc_varint(rng.getrandbits(20))))
        else:
            msgs.append(("u", rng.getrandbits(rng.choice([7, 14, 30, 63])), mg.rand_value(rng)))
    wire, _ = mg.batch(msgs)
    cols, st = gpu_decode(codec, wire)
    assert_same_as_oracle(cols, st, wire)
    import torch
    heap = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).cuda()
    assert codec.encode_batch(cols, heap).cpu().numpy().tobytes() == wire


def test_fuzz_random_bytes_match_oracle(codec):
    """Decoding random bytes never crashes and agrees with the oracle on accept/reject
    (netidx-netproto/src/test.rs:449-456 + first-error parity)."""
    rng = np.random.default_rng(1234)
    for i in range(300):
        n = int(rng.integers(0, 200))
        w = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        if i % 3 == 0:  # mostly-small bytes keep messages decodable for longer
            w = (rng.integers(0, 256, n, dtype=np.uint8) % 20).astype(np.uint8).tobytes()
        cols, st = gpu_decode(codec, w)
        assert_same_as_oracle(cols, st, w)


def test_long_values_span_tiles(codec):
    """Strings/bytes longer than a tile: speculation inside them must be repaired exactly."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mg", os.path.join(GOLD, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    rng = random.Random(5)
    msgs = []
    for i in range(60):
        L = rng.choice([10, 300, 9000, 40000])
        # the bytes payload is itself a valid-looking stream of f64 updates
        fake = b"".join(mg.update(j, (9, rng.getrandbits(64))) for j in range(L // 12 + 1))[:L]
        msgs.append(("u", i, (13, fake)))
        msgs.append(("u", i, (9, rng.getrandbits(64))))
    wire, _ = mg.batch(msgs)
    cols, st = gpu_decode(codec, wire)
    assert_same_as_oracle(cols, st, wire)


def _mg():
    import importlib.util
    spec = importlib.util.spec_from_file_location("mg", os.path.join(GOLD, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    return mg


def test_encode_staged_every_tag(codec):
    """Updates only (no control messages): the general encoder's staged, class-bucketed path
    with every Value tag, Maps, Errors and nesting (the stack walk), byte-identical."""
    import torch
    mg = _mg()
    rng = random.Random(321)
    msgs = [("u", rng.getrandbits(rng.choice([7, 14, 30, 63])), mg.rand_value(rng))
            for _ in range(6000)]
    wire, _ = mg.batch(msgs)
    cols, st = gpu_decode(codec, wire)
    assert_same_as_oracle(cols, st, wire)
    heap = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).cuda()
    assert codec.encode_batch(cols, heap).cpu().numpy().tobytes() == wire


def test_encode_arrays_of_fixed_size_elements(codec):
    """Arrays of 1..9 elements of every fixed-size tag (the encoder sizes arrays of up to 8 such
    elements from one load of their tags, at any alignment of their first child), with a
    varint or text element now and then (the element-by-element path), byte-identical."""
    import torch
    mg = _mg()
    rng = random.Random(4321)
    fixed_tags = [0, 2, 4, 6, 8, 9, 10, 11, 14, 15, 16, 20, 23, 24, 25, 26]
    msgs = []
    for i in range(8000):
        k = rng.randrange(1, 10)
        els = []
        for _ in range(k):
            v = mg.rand_value(rng, 3)
            while v[0] not in fixed_tags:
                v = mg.rand_value(rng)
            els.append(v)
        if rng.random() < 0.1:
            els[rng.randrange(k)] = rng.choice([(1, rng.getrandbits(14)), (12, b"abc"),
                                                (5, rng.getrandbits(40))])
        msgs.append(("u", rng.getrandbits(rng.choice([7, 21, 30])), (19, els)))
        if rng.random() < 0.3:  # scalars between them shift the arrays' first child slots
            msgs.append(("u", i, (9, rng.getrandbits(64))))
    wire, _ = mg.batch(msgs)
    cols, st = gpu_decode(codec, wire)
    assert_same_as_oracle(cols, st, wire)
    heap = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).cuda()
    assert codec.encode_batch(cols, heap).cpu().numpy().tobytes() == wire


def test_encode_tiles_past_the_staging(codec):
    """Values longer than the encoder's LDS staging (28 bytes per row): those tiles write their
    rows straight to the frame; short tiles around them stay staged."""
    import torch
    mg = _mg()
    rng = random.Random(8)
    msgs = []
    for i in range(5000):
        if i % 1500 == 7:
            msgs.append(("u", i, (13, bytes(rng.getrandbits(8) for _ in range(40000)))))
        elif i % 3 == 0:
            msgs.append(("u", i, (12, b"x" * rng.randrange(0, 33))))
        else:
            msgs.append(("u", i, (9, rng.getrandbits(64))))
    wire, _ = mg.batch(msgs)
    cols, st = gpu_decode(codec, wire)
    assert_same_as_oracle(cols, st, wire)
    heap = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).cuda()
    assert codec.encode_batch(cols, heap).cpu().numpy().tobytes() == wire


@pytest.mark.parametrize("bad_tag", [17, 28, 200])
def test_encode_unknown_tag_fails(codec, bad_tag):
    """A column tag the wire format has no encoding for (Value::encode never writes 17; >= 28
    are not Value tags) fails the encode instead of writing a frame."""
    import netidx_amd
    n = 3000
    ids = np.arange(n, dtype=np.uint64)
    fixed = np.arange(n, dtype=np.uint64) * 3
    tag = np.full(n, 6, np.uint8)
    tag[n // 2] = bad_tag
    aux = np.zeros(n, np.uint32)
    cols = netidx_amd.columns_from_arrays(ids, fixed, tag, aux)
    with pytest.raises(Exception):
        codec.encode_batch(cols)


# ---- encode f64 + round trip at BASELINE sizes ---------------------------------------------
def test_f64_encode_matches_oracle(codec):
    import netidx_amd
    import nxo
    from netidx_amd import synth
    for n in (0, 1, 1023, 1024, 1025, 300_001):
        ids, vals = synth.f64_columns(n, 42)
        if n > 1000:
            ids[::3] = np.uint64(2**40) + ids[::3]  # wide ids too
        cols = netidx_amd.columns_from_arrays(ids, vals)
        out = codec.encode_batch(cols).cpu().numpy().tobytes()
        assert out == nxo.encode_f64(ids, vals).tobytes()


def test_f64_roundtrip_baseline_size(codec):
    """Config 2/4: 10^7 records, encode -> decode -> encode byte-identical, sampled oracle."""
    import netidx_amd
    import nxo
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n = 10_000_000
    ids, vals = synth.f64_columns(n)
    cols = netidx_amd.columns_from_arrays(ids, vals)
    wire = codec.encode_batch(cols)
    assert wire.numel() == 147_886_336
    out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    st = codec.decode_into(wire, wire.numel(), out)
    assert st.path == 1 and st.n_rows == n
    assert torch.equal(out.id[:n], cols.id[:n]) and torch.equal(out.fixed[:n], cols.fixed[:n])
    again = codec.encode_batch(out)
    assert torch.equal(again, wire)
    # sampled oracle: the first and last 1 MB decode identically
    w = wire[:1_000_008].cpu().numpy()
    o = nxo.decode(w).trim()
    k = len(o["id"])
    assert np.array_equal(o["id"], ids[:k]) and np.array_equal(o["fixed"], vals[:k])
    assert nxo.encode_f64(ids[-70_000:], vals[-70_000:]).tobytes() == \
        wire[-(len(nxo.encode_f64(ids[-70_000:], vals[-70_000:]))):].cpu().numpy().tobytes()


def test_async_api_and_streams(codec):
    import netidx_amd
    import torch
    from netidx_amd.codec import Columns
    ids, vals, wire = f64_wire(100_000, 21)
    dw = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).cuda()
    out = Columns(100_000, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    s = torch.cuda.Stream()
    codec.set_stream(s.cuda_stream)
    for _ in range(3):
        codec.decode_async(dw.data_ptr(), dw.numel(), out)
        st = codec.sync()
        assert st.n_rows == 100_000 and st.path == 1
    codec.set_stream(0)
    assert np.array_equal(out.numpy()["fixed"], vals)
