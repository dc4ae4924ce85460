"""The sequential-id f64 decoder (nxg_decode_f64_seq.hip) against the CPU oracle.

A publisher updating all of its values in publication order sends ids that count up by one
(netidx-core/src/utils.rs:130-134), so where each record starts is a closed form of its index; the
decoder checks every record (length, variant, id width, value tag, id == i0 + k) and hands anything
else to the length-run decoder. These tests pin:
  - bit-exact columns for frames of 1..4000 records and long ones, ids starting anywhere and
    crossing every varint width change (2^7, 2^14, 2^21, 2^28), and that the sequential-id kernel
    decoded them (DevStatus.diag[1]);
  - the hand-over: an id out of order anywhere (first, middle, last record), a non-canonical
    varint, a Heartbeat, trailing garbage, a truncated frame, ids past 2^35 -- each decoded (or
    rejected) exactly as the oracle does, by the next decoder in line;
  - after a hand-over the connection skips the kernel for a while, then tries it again.
Reference rules: netidx-core/src/pack.rs:504-555, netidx-value/src/lib.rs:470-506,
netidx/src/channel.rs:504-521.
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


def _decode(codec, wire, n_cap):
    import torch
    import netidx_amd
    from netidx_amd.codec import Columns
    cols = Columns(max(n_cap, 1), 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    dw = torch.from_numpy(np.ascontiguousarray(wire)).cuda()
    st = codec.decode_into(dw, dw.numel(), cols, 0, check=False)
    return cols, st, codec.last_diag()


def _check_vs_oracle(cols, st, wire):
    import nxo
    o = nxo.decode(np.ascontiguousarray(wire), cap_rows=len(wire) // 2 + 2, cap_children=len(wire) + 1,
                   cap_ctl=len(wire) // 2 + 2).trim()
    assert st.err_kind == o["err_kind"], (st.err_kind, o["err_kind"])
    if o["err_kind"]:
        assert st.err_offset == o["err_offset"]
        return o
    n = len(o["id"])
    assert st.n_rows == n
    g = cols.numpy()
    assert np.array_equal(g["id"][:n], o["id"])
    assert np.array_equal(g["fixed"][:n], o["fixed"])
    return o


def _seq_wire(n, i0, seed):
    import nxo
    from netidx_amd import synth
    ids, vals = synth.f64_columns(n, seed, id_offset=i0)
    return ids, vals, nxo.encode_f64(ids, vals)


@pytest.mark.parametrize("i0", [0, 1, 100, 127, 128, 16000, 16383, 16384, 2**21 - 300, 2**21,
                                2**28 - 2000, 2**28, 2**35 - 5000])
def test_seq_sizes_and_id_starts(codec, i0):
    rng = np.random.default_rng(i0 & 0xffff)
    sizes = [1, 2, 63, 64, 65, 255, 256, 257, 1023, 1024, 1025, 4000] + \
        [int(x) for x in rng.integers(1, 6000, 4)]
    for n in sizes:
        ids, vals, wire = _seq_wire(n, i0, n)
        cols, st, diag = _decode(codec, wire, n)
        _check_vs_oracle(cols, st, wire)
        assert st.path == 1 and diag[1] == 1, (i0, n, diag)


def test_seq_long_frame_every_width(codec):
    """10^6 records from id 2^21 - 300000 (3- and 4-byte ids) and a frame from 0 crossing 2^7
    and 2^14: every row against the oracle, on the sequential-id kernel."""
    for n, i0 in ((1_000_000, 2**21 - 300_000), (400_000, 0)):
        ids, vals, wire = _seq_wire(n, i0, 7)
        cols, st, diag = _decode(codec, wire, n)
        _check_vs_oracle(cols, st, wire)
        assert diag[1] == 1


def test_seq_config2_10m(codec):
    """BASELINE configs[1]: 10^7 sequential ids, every row, on the sequential-id kernel."""
    ids, vals, wire = _seq_wire(10_000_000, 0, 0x5EED0002)
    assert len(wire) == 147_886_336
    cols, st, diag = _decode(codec, wire, len(ids))
    _check_vs_oracle(cols, st, wire)
    assert diag[1] == 1


def test_seq_past_the_infinity_cache(codec):
    """2.5 * 10^7 records (370 MB): the XCD-contiguous workgroup order."""
    ids, vals, wire = _seq_wire(25_000_000, 5, 11)
    assert len(wire) > 256 << 20
    cols, st, diag = _decode(codec, wire, len(ids))
    _check_vs_oracle(cols, st, wire)
    assert diag[1] == 1


def _fresh():
    import netidx_amd
    return netidx_amd.Codec(0)


@pytest.mark.parametrize("where", ["first", "second", "middle", "wave_edge", "last"])
def test_seq_hands_over_when_an_id_is_out_of_order(where):
    """One id swapped with its neighbour, or one id skipped: the frame is still a valid f64 frame,
    decoded by the next decoder exactly like the oracle (and not by the sequential-id kernel)."""
    import nxo
    from netidx_amd import synth
    n = 5000
    ids, vals = synth.f64_columns(n, 3, id_offset=1000)
    k = {"first": 0, "second": 1, "middle": n // 2, "wave_edge": 255, "last": n - 2}[where]
    ids = ids.copy()
    ids[k], ids[k + 1] = ids[k + 1], ids[k]
    wire = nxo.encode_f64(ids, vals)
    c = _fresh()
    try:
        cols, st, diag = _decode(c, wire, n)
        _check_vs_oracle(cols, st, wire)
        assert st.path == 1 and diag[1] != 1
        # a gap (an id skipped) at the end
        ids2, vals2 = synth.f64_columns(n, 4, id_offset=1000)
        ids2 = ids2.copy()
        ids2[-1] += 1
        wire2 = nxo.encode_f64(ids2, vals2)
        cols, st, diag = _decode(c, wire2, n)
        _check_vs_oracle(cols, st, wire2)
        assert diag[1] != 1
    finally:
        c.close()


def test_seq_skips_after_a_hand_over_then_tries_again():
    """A connection whose frames are not sequential pays the failed attempt once: the next 64
    calls go straight to the length-run decoder; after them the kernel is tried again."""
    import nxo
    from netidx_amd import synth
    n = 3000
    ids, vals = synth.f64_columns(n, 5)
    wire_seq = nxo.encode_f64(ids, vals)
    perm = np.random.default_rng(6).permutation(ids)
    wire_perm = nxo.encode_f64(perm, vals)
    c = _fresh()
    try:
        cols, st, diag = _decode(c, wire_perm, n)
        _check_vs_oracle(cols, st, wire_perm)
        seen = []
        for _ in range(70):
            cols, st, diag = _decode(c, wire_seq, n)
            _check_vs_oracle(cols, st, wire_seq)
            seen.append(diag[1] == 1)
        assert not any(seen[:60]) and seen[-1]
    finally:
        c.close()


def _rec(L, id_bytes, val8):
    return bytes([L, 4]) + id_bytes + bytes([9]) + val8


def test_seq_edge_frames_match_the_oracle():
    """Frames that look sequential to a point: each must decode (or fail) exactly as the oracle,
    whichever decoder ends up with it."""
    import nxo
    from netidx_amd import synth
    n = 700
    ids, vals, wire = _seq_wire(n, 0, 9)
    w = bytes(wire)
    v8 = bytes(8)
    cases = {
        # a Heartbeat in the middle (a valid frame: the mixed path takes it)
        "heartbeat": w[: 12 * 100] + b"\x02\x05" + w[12 * 100:],
        # trailing garbage and a truncated last record
        "trailing": w + b"\x01",
        "truncated": w[:-3],
        # record 5's id as a non-canonical two-byte varint (0x85 0x00): valid, decodes to 5
        "noncanonical": w[: 12 * 5] + _rec(13, b"\x85\x00", v8) + w[12 * 6:],
        # an Update whose value is not an f64 (tag 4 = U64) at the end
        "u64_last": w[:-13] + bytes([13, 4, 0x80 | ((n - 1) & 0x7f), (n - 1) >> 7, 4]) + v8,
        # ids past 2^35: 6-byte varints
        "wide": nxo.encode_f64(np.arange(2**35 - 3, 2**35 + 3, dtype=np.uint64), np.zeros(6, np.uint64)),
        # a single record, and a frame of one byte
        "one": w[:12],
        "byte": w[:1],
    }
    c = _fresh()
    try:
        for name, b in cases.items():
            arr = np.frombuffer(b, np.uint8)
            import torch
            import netidx_amd
            from netidx_amd.codec import Columns
            cols = Columns(len(b) + 1, len(b) + 1, len(b) + 1, netidx_amd.LAYOUT_MIXED, "cuda")
            dw = torch.from_numpy(arr.copy()).cuda()
            st = c.decode_into(dw, dw.numel(), cols, 0, check=False)
            o = nxo.decode(arr, cap_rows=len(b) + 1, cap_children=len(b) + 1, cap_ctl=len(b) + 1).trim()
            assert st.err_kind == o["err_kind"], name
            if o["err_kind"]:
                assert st.err_offset == o["err_offset"], name
                continue
            g = cols.numpy()
            for k in ("id", "fixed"):
                assert np.array_equal(g[k][: len(o[k])], o[k]), (name, k)
    finally:
        c.close()
    # (a fresh connection: the frames above made this one skip the sequential-id kernel)
    c = _fresh()
    try:
        cols, st, diag = _decode(c, np.frombuffer(w[:12], np.uint8), 1)
        _check_vs_oracle(cols, st, np.frombuffer(w[:12], np.uint8))
        assert diag[1] == 1
    finally:
        c.close()


def test_seq_capacity_short():
    """Columns one row short: the capacity error, as on the other decoders."""
    import netidx_amd
    ids, vals, wire = _seq_wire(1000, 0, 12)
    c = _fresh()
    try:
        cols, st, diag = _decode(c, wire, 999)
        assert st.err_kind == netidx_amd.CAPACITY and diag[1] == 1
    finally:
        c.close()


def test_seq_async_and_frames_async(codec):
    """The async entry points take the sequential-id kernel too: a backlog of 6 frames into 3
    column sets, each checked against the encoder's columns."""
    import torch
    import netidx_amd
    from netidx_amd.codec import Columns
    n = 200_000
    frames, refs = [], []
    for j in range(3):
        ids, vals, wire = _seq_wire(n, 1000 * j, 20 + j)
        frames.append(torch.from_numpy(np.ascontiguousarray(wire)).cuda())
        refs.append((ids, vals))
    outs = [Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda") for _ in range(3)]
    sel = [0, 1, 2, 2, 1, 0]
    codec.decode_frames_async([frames[j].data_ptr() for j in sel], [frames[j].numel() for j in sel],
                              [outs[j] for j in sel])
    st = codec.sync()
    assert st.err_kind == 0 and codec.last_diag()[1] == 1
    for j in range(3):
        g = outs[j].numpy()
        assert np.array_equal(g["id"], refs[j][0]) and np.array_equal(g["fixed"], refs[j][1])
    for j in range(3):
        outs[j].id.zero_()
        codec.decode_async(frames[j].data_ptr(), frames[j].numel(), outs[j])
    codec.sync()
    for j in range(3):
        assert np.array_equal(outs[j].numpy()["id"], refs[j][0])


def test_async_backlog_keeps_wire_order_after_a_late_fallback():
    """a frame the sequential-id kernel declines is decoded again at sync,
    after the frames behind it. A later frame into the same columns must still be the one left
    in them, and an async encode that read those columns must see the frame decoded before it.
    A fresh context, so the sequential-id kernel is tried first on every frame."""
    import torch
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n = 150_000
    codec = netidx_amd.Codec(0)
    try:
        ids_a, vals_a = synth.f64_columns(n, 31)
        perm = np.random.default_rng(5).permutation(n)
        ids_a = ids_a[perm]
        wire_a = nxo.encode_f64(ids_a, vals_a)  # ids in random order: declined, rerun at sync
        ids_b, vals_b, wire_b = _seq_wire(n, 500, 32)
        fa = torch.from_numpy(np.ascontiguousarray(wire_a)).cuda()
        fb = torch.from_numpy(np.ascontiguousarray(wire_b)).cuda()
        cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        codec.decode_frames_async([fa.data_ptr(), fb.data_ptr()], [fa.numel(), fb.numel()],
                                  [cols, cols])
        st = codec.sync()
        assert st.err_kind == 0
        g = cols.numpy()
        assert np.array_equal(g["id"], ids_b) and np.array_equal(g["fixed"], vals_b)
        # the same through single async calls, then an async encode of the declined frame's
        # columns: the encode must read the rerun's rows, not the declined attempt's (a fresh
        # context: this one now skips the sequential-id kernel for a while)
        codec.close()
        codec = netidx_amd.Codec(0)
        other = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        out = torch.zeros(len(wire_a) + 64, dtype=torch.uint8, device="cuda")
        codec.decode_async(fa.data_ptr(), fa.numel(), other)
        n_len = codec.encode_async(other, None, out.data_ptr(), out.numel())
        codec.decode_async(fb.data_ptr(), fb.numel(), cols)
        codec.sync()
        assert n_len.value == len(wire_a)
        assert np.array_equal(out[:len(wire_a)].cpu().numpy(), wire_a)
        g = other.numpy()
        assert np.array_equal(g["id"], ids_a) and np.array_equal(g["fixed"], vals_a)
        # a mixed frame (declined by the f64 decoders) before a sequential one, same columns
        codec.close()
        codec = netidx_amd.Codec(0)
        m = synth.mixed_columns(20_000, 9)
        mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed,
                                            m.caux)
        mw = codec.encode_batch(mc, torch.from_numpy(m.heap.copy()).cuda())
        mixed = Columns.for_frame(max(mw.numel(), len(wire_b)), netidx_amd.LAYOUT_MIXED, "cuda")
        codec.decode_frames_async([mw.data_ptr(), fb.data_ptr()], [mw.numel(), fb.numel()],
                                  [mixed, mixed])
        codec.sync()
        g = mixed.numpy()
        assert np.array_equal(g["id"], ids_b) and np.array_equal(g["fixed"], vals_b)
    finally:
        codec.close()
