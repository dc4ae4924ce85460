"""GPU parity of the fast mixed decoder (nxg_decode_mixed.hip, status path 4).

Frames of short Update messages with flat values take the fast decoder; everything else must be
rejected by it and rerun on the general decoder (path 2). Either way the columns, the first
error and the re-encoding must equal the oracle's (nx_oracle.c nxo_decode, which restates
netidx-netproto/src/publisher.rs:73-96 + netidx-value/src/lib.rs:470-506), and the fast decoder's
columns must equal the general decoder's on the same frame.
"""
import os
import random
import zlib

import numpy as np
import pytest

from test_gpu_parity import _mg, assert_same_as_oracle, gpu_decode, mixed_wire

pytestmark = pytest.mark.gpu

@pytest.fixture
def codec():
    # a fresh context per test: a rejected frame makes a context skip the fast decoder for the
    # next calls (kMixFailCalls)
    import torch
    import netidx_amd
    assert torch.cuda.is_available()
    c = netidx_amd.Codec(0)
    yield c
    c.close()


def _general_codec():
    import netidx_amd
    os.environ["NXG_MIXED_PATH"] = "general"
    try:
        return netidx_amd.Codec(0)
    finally:
        del os.environ["NXG_MIXED_PATH"]


def flat_value(rng, mg, err22=False):
    """A Value the fast decoder takes: a leaf, an Array of leaves or (err22) an Error(String) in
    its Error(Value) spelling (tag 22 + 12, which re-encodes as tag 18), in a message shorter
    than 128 bytes."""
    while True:
        if err22 and rng.random() < 0.02:
            return (22, (12, b"err"))
        v = mg.rand_value(rng)
        t = v[0]
        if t in (21, 22):
            continue
        if t == 19:
            v = (19, [e for e in v[1] if e[0] not in (19, 21, 22)])
        if len(mg.update(2**35 - 1, v)) < 128:
            return v


def flat_wire(n, seed, id_bits=(7, 14, 21, 30, 35), err22=False):
    mg = _mg()
    rng = random.Random(seed)
    msgs = [("u", rng.getrandbits(rng.choice(id_bits)), flat_value(rng, mg, err22))
            for _ in range(n)]
    wire, _ = mg.batch(msgs)
    return wire


def hint():
    import netidx_amd
    return netidx_amd.HINT_MIXED


def reencode(codec, cols, wire):
    import torch
    heap = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).cuda()
    return codec.encode_batch(cols, heap).cpu().numpy().tobytes()


@pytest.mark.parametrize("n", [1, 2, 3, 40, 63, 64, 65, 500, 4096, 30_000])
def test_fast_every_leaf_tag(codec, n):
    wire = flat_wire(n, 1000 + n)
    cols, st = gpu_decode(codec, wire, flags=hint())
    assert st.err_kind == 0 and st.path == 4, (st.path, st.err_kind)
    assert_same_as_oracle(cols, st, wire)
    assert reencode(codec, cols, wire) == wire


@pytest.mark.parametrize("n", [1, 10, 5000, 200_000])
def test_fast_config3_shape(codec, n):
    m, wire = mixed_wire(n, 300 + n)
    cols, st = gpu_decode(codec, wire, flags=hint())
    assert st.err_kind == 0 and st.path == 4
    assert_same_as_oracle(cols, st, wire)


def test_fast_without_hint_after_f64_rejects(codec):
    """No hint: the f64 decoder rejects the frame, the fast mixed decoder takes it."""
    m, wire = mixed_wire(20_000, 7)
    cols, st = gpu_decode(codec, wire)
    assert st.err_kind == 0 and st.path == 4
    assert_same_as_oracle(cols, st, wire)


def test_fast_equals_general_every_column(codec):
    gen = _general_codec()
    try:
        for n, seed in ((100_000, 1), (3000, 2)):
            wire = flat_wire(n, seed, err22=True)
            a, sa = gpu_decode(codec, wire, flags=hint())
            b, sb = gpu_decode(gen, wire, flags=hint())
            assert (sa.path, sb.path) == (4, 2)
            ga, gb = a.numpy(), b.numpy()
            assert set(ga) == set(gb)
            for k in ga:
                assert np.array_equal(ga[k], gb[k]), k
            assert (sa.n_rows, sa.n_children, sa.n_ctl) == (sb.n_rows, sb.n_children, sb.n_ctl)
    finally:
        gen.close()


def test_fast_tile_edges(codec):
    """Messages of every length 4..127 around the 4 KiB tile boundaries: entries in the first
    two chunks of a tile, messages that cover a whole chunk, a frame ending on a tile edge."""
    mg = _mg()
    rng = random.Random(17)
    for total in (4096, 8192, 8192 + 37, 3 * 4096 - 5):
        msgs, size = [], 0
        while True:
            ln = rng.choice([0, 1, 5, 30, 60, 90, 110])  # string bytes -> message 8..120 B
            v = (12, b"q" * ln)
            enc = mg.update(3, v)
            if size + len(enc) > total:
                break
            msgs.append(("u", 3, v))
            size += len(enc)
        # pad to the exact size with a last message when it fits one
        rest = total - size
        if 5 <= rest <= 127:
            msgs.append(("u", 3, (12, b"z" * (rest - 5))))
        wire, _ = mg.batch(msgs)
        cols, st = gpu_decode(codec, wire, flags=hint())
        assert st.err_kind == 0 and st.path == 4, (total, len(wire))
        assert_same_as_oracle(cols, st, wire)


def test_fast_longest_messages(codec):
    """127-byte messages (the longest one-byte length), back to back across tiles."""
    mg = _mg()
    one = mg.update(5, (12, b"x" * 122))
    assert len(one) == 127 and one[0] == 127
    wire, _ = mg.batch([("u", 5, (12, b"x" * 122))] * 200)
    cols, st = gpu_decode(codec, wire, flags=hint())
    assert st.err_kind == 0 and st.path == 4
    assert_same_as_oracle(cols, st, wire)


def _rejected(codec, wire, strict=True, big_caps=False):
    cols, st = gpu_decode(codec, wire, flags=hint())
    if strict:
        assert st.path == 2 or st.err_kind != 0
    assert_same_as_oracle(cols, st, wire, big_caps)


def _with(mg, n, seed, extra_at, extra):
    rng = random.Random(seed)
    msgs = [("u", rng.getrandbits(14), flat_value(rng, mg)) for _ in range(n)]
    msgs.insert(extra_at, extra)
    return mg.batch(msgs)[0]


@pytest.mark.parametrize("case", ["unsubscribed", "long_array", "map", "nested",
                                  "error_value", "wide_id", "abstract_long", "huge_string"])
def test_rejected_frames_fall_back_exactly(codec, case):
    mg = _mg()
    extra = {
        "unsubscribed": ("raw", 2, mg.enc_varint(99)),
        "long_array": ("u", 1, (19, [(9, 1)] * 20)),  # 128 bytes or more: not text
        "huge_string": ("u", 1, (12, b"L" * 17000)),  # a three-byte length prefix
        "map": ("u", 1, (21, [((9, 1), (12, b"k"))])),
        "nested": ("u", 1, (19, [(19, [(9, 5)])])),
        "error_value": ("u", 1, (22, (9, 7))),
        "wide_id": ("u", (1 << 60) + 3, (9, 1)),
        "abstract_long": ("u", 1, (27, bytes(range(200)))),
    }[case]
    for at in (0, 2500, 5000):
        _rejected(codec, _with(mg, 5000, 11, at, extra))


def test_errors_and_truncation_fall_back_exactly(codec):
    wire = flat_wire(6000, 21)
    rng = np.random.default_rng(5)
    for cut in (1, 2, 7, 100, 4096, 5000):
        _rejected(codec, wire[:-cut], strict=False)
    for _ in range(12):
        w = bytearray(wire)
        w[int(rng.integers(0, len(w)))] ^= int(rng.integers(1, 256))
        _rejected(codec, bytes(w), strict=False)
    # bad UTF-8 in a string, an unknown value tag, a short DateTime
    mg = _mg()
    _rejected(codec, _with(mg, 3000, 3, 1500, ("raw", 4, mg.enc_varint(7) + b"\x0c\x02\xc3\x28")))
    _rejected(codec, _with(mg, 3000, 4, 1500, ("raw", 4, mg.enc_varint(7) + b"\x1c")))
    _rejected(codec, _with(mg, 3000, 5, 1500, ("raw", 4, mg.enc_varint(7) + b"\x0a\x00\x00")))


def test_capacity_is_reported(codec):
    import netidx_amd
    from netidx_amd.codec import Columns
    import torch
    m, wire = mixed_wire(5000, 9)
    frame = torch.from_numpy(np.frombuffer(wire, np.uint8).copy()).cuda()
    cols = Columns(4000, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
    st = codec.decode_into(frame, len(wire), cols, hint(), check=False)
    assert st.err_kind == netidx_amd.CAPACITY


def test_fuzz_small_frames(codec):
    """Random bytes that look like short Updates: accept/reject and first error as the oracle."""
    rng = np.random.default_rng(77)
    for i in range(200):
        n = int(rng.integers(1, 400))
        w = bytearray(rng.integers(0, 30, n, dtype=np.uint8).tobytes())
        p = 0
        while p + 2 < n:  # sprinkle plausible headers
            L = int(rng.integers(4, 40))
            w[p] = L
            w[p + 1] = 4
            p += L
        _rejected(codec, bytes(w), strict=False, big_caps=True)


def test_fast_long_arrays(codec):
    """Arrays of up to 120 one- and two-byte elements: more elements per round than the
    lane-parallel list holds (the per-lane path), next to short ones (the list)."""
    mg = _mg()
    rng = random.Random(8)
    msgs = []
    for i in range(3000):
        k = rng.random()
        if k < 0.3:
            v = (19, [(16, None)] * rng.randrange(60, 121))
        elif k < 0.5:
            v = (19, [(24, rng.randint(-128, 127)) for _ in range(rng.randrange(1, 55))])
        elif k < 0.7:
            v = (19, [(9, rng.getrandbits(64)) for _ in range(rng.randrange(0, 12))])
        else:
            v = flat_value(rng, mg)
        msgs.append(("u", i, v))
    wire, _ = mg.batch(msgs)
    cols, st = gpu_decode(codec, wire, flags=hint())
    assert st.err_kind == 0 and st.path == 4
    assert_same_as_oracle(cols, st, wire)
    assert reencode(codec, cols, wire) == wire


@pytest.mark.parametrize("mix", [0.0, 0.02, 0.3])
def test_fast_deferred_array_batches(codec, mix):
    """Arrays of one fixed-size element tag each (the emit gathers their elements over rounds, up
    to 256 elements of 64 arrays a batch), DateTime / Duration arrays among them, and a share
    `mix` of arrays whose later elements differ in size (a fixed size of another length, a varint
    or text: the batch's walk per array), between scalars and Arrays without elements."""
    mg = _mg()
    rng = random.Random(int(mix * 1000) + 17)
    fixed_tags = [0, 2, 4, 6, 8, 9, 10, 11, 14, 15, 16, 20, 23, 24, 25, 26]
    msgs = []
    for i in range(20_000):
        u = rng.random()
        if u < 0.15:
            msgs.append(("u", i, (9, rng.getrandbits(64))))
            continue
        if u < 0.18:
            msgs.append(("u", i, (19, [])))
            continue
        t = rng.choice(fixed_tags)
        while True:  # (rand_value draws every tag at depth 0)
            v = mg.rand_value(rng)
            if v[0] == t:
                break
        els = [v] * rng.randrange(1, 12)
        if len(els) > 1 and rng.random() < mix:
            els[rng.randrange(1, len(els))] = rng.choice(
                [(1, rng.getrandbits(14)), (12, "é€".encode()), (24, -5), (9, 7), (10, (5, 6)),
                 (11, (3, 4))])
        if len(mg.update(i, (19, els))) < 128:
            msgs.append(("u", i, (19, els)))
    wire, _ = mg.batch(msgs)
    cols, st = gpu_decode(codec, wire, flags=hint())
    assert st.err_kind == 0 and st.path == 4, (st.path, st.err_kind)
    assert_same_as_oracle(cols, st, wire)
    assert reencode(codec, cols, wire) == wire


UTF8_VALID = [
    b"", b"a", b"\x7f", "\u0080".encode(), "߿".encode(), "ࠀ".encode(),
    "퟿".encode(), "".encode(), "￿".encode(), "\U00010000".encode(),
    "\U0010ffff".encode(), "é€😀Ωж".encode(), ("x" * 61 + "€").encode(),  # sequence at byte 61
    ("€" * 40).encode(), ("y" * 63 + "😀" + "z" * 50).encode(),  # across the wave's 64 lanes
    ("q" * 15 + "é").encode(), ("q" * 16 + "é").encode(), ("q" * 14 + "€").encode(),
]
UTF8_INVALID = [
    b"\x80", b"a\xbf", b"\xc0\x80", b"\xc1\xbf", b"\xe0\x80\x80", b"\xe0\x9f\xbf",
    b"\xed\xa0\x80", b"\xed\xbf\xbf", b"\xf0\x80\x80\x80", b"\xf0\x8f\xbf\xbf",
    b"\xf4\x90\x80\x80", b"\xf5\x80\x80\x80", b"\xff", b"\xe2\x82", b"ab\xe2", b"\xc3",
    b"\xc3(", b"\xe2\x28\xa1", b"\xf0\x9f\x98", b"\xc3\xa9\xa9", b"\xe2\x82\xac\x80",
    b"x" * 62 + b"\xe2\x82", b"x" * 70 + b"\xf0\x9f\x98\x80\x80",
]


def _string_frame(mg, s, as_element, tag=12, n=300, seed=0):
    rng = random.Random(seed)
    msgs = [("u", rng.getrandbits(20), flat_value(rng, mg)) for _ in range(n)]
    v = (19, [(9, 7), (tag, s), (6, -1)]) if as_element else (tag, s)
    msgs.insert(n // 2, ("u", 99, v))
    # messages of 128 bytes or more are the general decoder's unless they hold text
    return mg.batch(msgs)[0], len(mg.update(99, v)) < 128 or not as_element


@pytest.mark.parametrize("as_element", [False, True])
def test_fast_utf8_valid_sequences(as_element):
    """Text with every UTF-8 sequence length and the boundary code points, as a row and as an
    array element: decoded on the fast path, identical to the oracle. (A fresh context per frame:
    a frame the fast decoder declines makes a context skip it for the next calls.)"""
    mg = _mg()
    for k, s in enumerate(UTF8_VALID):
        for tag in (12, 18):
            wire, fast = _string_frame(mg, s, as_element, tag, seed=k)
            cols, st = _decode_fresh(wire)
            assert st.err_kind == 0 and st.path == (4 if fast else 2), (s, tag, st.path)
            assert_same_as_oracle(cols, st, wire)


def _decode_fresh(wire):
    import netidx_amd
    c = netidx_amd.Codec(0)
    try:
        return gpu_decode(c, wire, flags=hint())
    finally:
        c.close()


@pytest.mark.parametrize("as_element", [False, True])
def test_fast_utf8_invalid_sequences(as_element):
    """Overlong forms, surrogates, code points past U+10FFFF, stray and missing continuation
    bytes, sequences cut by the end of the text: the first error as the oracle's; Bytes (13)
    with the same bytes are not text and stay on the fast path."""
    mg = _mg()
    for k, s in enumerate(UTF8_INVALID):
        wire, _ = _string_frame(mg, s, as_element, seed=100 + k)
        cols, st = _decode_fresh(wire)
        assert st.err_kind != 0, s
        assert_same_as_oracle(cols, st, wire)
        wire, fast = _string_frame(mg, s, as_element, tag=13, seed=200 + k)
        cols, st = _decode_fresh(wire)
        assert st.err_kind == 0 and st.path == (4 if fast else 2), s
        assert_same_as_oracle(cols, st, wire)


# ---- Heartbeats and two-byte length prefixes ---------------------------------------------------
@pytest.mark.parametrize("case", ["first", "middle", "last", "runs", "every_other", "only"])
def test_fast_heartbeats(codec, case):
    """From::Heartbeat (02 05) anywhere in the frame stays on the fast path: a control span
    (ctl_row = the next row, ctl_off, ctl_len 2, variant 5) as the oracle's."""
    mg = _mg()
    rng = random.Random(zlib.crc32(case.encode()))  # (hash() of a str varies per process)
    msgs = [("u", rng.getrandbits(20), flat_value(rng, mg)) for _ in range(6000)]
    if case == "first":
        msgs.insert(0, ("hb",))
    elif case == "middle":
        msgs.insert(3000, ("hb",))
    elif case == "last":
        msgs.append(("hb",))
    elif case == "runs":  # runs of up to 300 (more than a tile's worth at some tile edges)
        for at in (10, 2000, 4000, 5999):
            msgs[at:at] = [("hb",)] * rng.choice([1, 2, 63, 64, 65, 300])
    elif case == "every_other":
        msgs = [m for x in msgs[:3000] for m in (x, ("hb",))]
    else:
        msgs = [("hb",)] * 900  # 1800 bytes: one tile
    wire, _ = mg.batch(msgs)
    cols, st = gpu_decode(codec, wire, flags=hint())
    assert st.err_kind == 0 and st.path == 4, (st.path, st.err_kind)
    assert_same_as_oracle(cols, st, wire)
    assert reencode(codec, cols, wire) == wire


def test_heartbeats_past_the_tile_list_fall_back(codec):
    """A tile of more Heartbeats than the emit pass's list holds: the general decoder."""
    mg = _mg()
    wire, _ = mg.batch([("u", 1, (9, 5))] + [("hb",)] * 5000 + [("u", 2, (9, 6))])
    cols, st = gpu_decode(codec, wire, flags=hint())
    assert st.err_kind == 0
    assert_same_as_oracle(cols, st, wire)


@pytest.mark.parametrize("tag", [12, 13, 18, 22])
def test_fast_two_byte_prefix_text(codec, tag):
    """Text values of 120 .. 16000 bytes (two-byte length prefixes), among short messages and
    across tile edges: the fast path where a message fits the tile's image or leaves it (the
    text then checked from global memory); longer than a tile may fall back. Columns as the
    oracle's either way."""
    mg = _mg()
    rng = random.Random(tag)
    for lens in ([120, 121, 122, 123, 124, 125, 126, 127, 128, 129, 130, 200, 255, 256, 257],
                 [1000, 3000, 4000, 4090], [4100, 9000, 16000]):
        msgs = []
        for i in range(3000):
            if rng.random() < 0.02:
                ln = rng.choice(lens)
                body = bytes(rng.randrange(0x61, 0x7b) for _ in range(ln))
                if i % 3 == 0 and tag != 13:
                    body = body[:ln // 2 - 1] + "é".encode() + body[ln // 2 + 1:]
                v = (22, (12, body)) if tag == 22 else (tag, body)
                msgs.append(("u", rng.getrandbits(30), v))
            else:
                msgs.append(("u", rng.getrandbits(14), flat_value(rng, mg)))
        wire, _ = mg.batch(msgs)
        cols, st = gpu_decode(codec, wire, flags=hint())
        assert st.err_kind == 0, st.err_kind
        if max(lens) < 4096:
            assert st.path == 4, (lens, st.path)
        assert_same_as_oracle(cols, st, wire)
        if tag != 22:  # (Error(String) re-encodes in its one-tag spelling, 18)
            assert reencode(codec, cols, wire) == wire


@pytest.mark.parametrize("share", [0.3, 1.0])
def test_fast_text_heavy_frames(codec, share):
    """Frames whose bytes are nearly all long text (a third, or every message, 1000 .. 16000
    bytes): almost every 4 KiB tile starts inside a message, so no tile of the count pass can
    anchor a wave's first tile; each wave takes the chain's exit from the wave before it. Still
    the fast path, every column as the oracle's."""
    mg = _mg()
    rng = random.Random(int(share * 10))
    msgs = []
    for i in range(6000 if share < 1 else 3000):
        if rng.random() < share:
            body = bytes(rng.randrange(0x61, 0x7b) for _ in range(rng.randrange(1000, 16000)))
            msgs.append(("u", rng.getrandbits(30), (12, body)))
        else:
            msgs.append(("u", rng.getrandbits(14), flat_value(rng, mg)))
    wire, _ = mg.batch(msgs)
    assert len(wire) > 200 * 64 * 1024 // 16  # many waves of 64 tiles
    cols, st = gpu_decode(codec, wire, flags=hint())
    assert st.err_kind == 0 and st.path == 4, (st.path, st.err_kind)
    assert_same_as_oracle(cols, st, wire)


@pytest.mark.parametrize("where", [5, 150, 1000, 3000, 5999])
def test_long_text_bad_utf8_first_error(where):
    """Invalid UTF-8 inside a long string, in the tile's image or past it: the oracle's first
    error (the general decoder reports it)."""
    mg = _mg()
    rng = random.Random(where)
    body = bytearray(b"t" * 6000)
    body[where] = 0xC3  # a lead without its continuation
    msgs = [("u", rng.getrandbits(14), flat_value(rng, mg)) for _ in range(400)]
    msgs.insert(200, ("u", 77, (12, bytes(body[:max(where + 10, 130)]))))
    wire, _ = mg.batch(msgs)
    cols, st = _decode_fresh(wire)
    assert st.err_kind != 0
    assert_same_as_oracle(cols, st, wire)


@pytest.mark.parametrize("n", [1000, 200_000])
def test_fast_config3_with_heartbeats_and_long_strings(codec, n):
    """Config 3 as a live subscriber sees it (synth.mixed_columns_ctl: 1 % Heartbeats, 1 % of
    the rows 200-byte strings): on the fast path, every column as the oracle's, and the encode
    of the same columns gives the frame back."""
    import netidx_amd
    import torch
    from netidx_amd import synth
    m, cr, co, cl, cv = synth.mixed_columns_ctl(n, 400 + n)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux,
                                        cr, co, cl, cv)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    wire = codec.encode_batch(mc, heap).cpu().numpy().tobytes()
    cols, st = gpu_decode(codec, wire, flags=hint())
    assert st.err_kind == 0 and st.path == 4, (st.path, st.err_kind)
    assert st.n_heartbeat == len(cr) and st.n_ctl == len(cr)
    assert_same_as_oracle(cols, st, wire)
    assert reencode(codec, cols, wire) == wire
