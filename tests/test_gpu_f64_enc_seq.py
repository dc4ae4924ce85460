"""The sequential-id f64 encoder (nxg_encode_f64_seq.hip) against the CPU oracle's encoder.

A publisher that updates all of its values in publication order hands handle_updates ids that
count up by one (netidx-core/src/utils.rs:130-134), so record k of the frame starts at a closed
form of k and the encoder needs no length scan and no look-back. These tests pin:
  - byte-identical frames (oracle/nx_oracle.c's encoder, which restates pack.rs:476-486, 522-535
    and Value::encode, lib.rs:404-407) for batches of 1..70001 records whose ids start anywhere
    and cross every varint width change (2^7, 2^14, 2^21, 2^28) up to 2^35, written at every
    16-byte phase of the output pointer, with no byte written outside the frame;
  - that the sequential-id kernel wrote them (not the tiled fallback);
  - the hand-over: ids out of order anywhere, ids past 2^35, random ids -- encoded by the tiled
    encoder, byte-identical; after it the kernel is skipped for 64 encodes, then tried again;
  - capacity errors, sizing (nxg_encoded_len), and a backlog of async encodes with a late
    fallback whose output a later decode of the backlog reads.
Reference: netidx/src/publisher/server.rs:604-629, netidx/src/channel.rs:177-202.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SENT = 0xEE


@pytest.fixture(scope="module")
def codec():
    import torch
    import netidx_amd
    assert torch.cuda.is_available()
    c = netidx_amd.Codec(0)
    yield c
    c.close()


def _vals(n, rng):
    v = rng.integers(0, 2**64, n, dtype=np.uint64)
    specials = np.array([0, 0x8000000000000000, 0x7FF0000000000000, 0xFFF8000000000000,
                         0x0000000000000001, 0xFFFFFFFFFFFFFFFF], np.uint64)
    k = min(n, len(specials))
    v[:k] = specials[:k]
    return v


def _encode(codec, ids, vals, off=0, cap=None):
    """Encode through nxg_encode_updates into a sentinel-filled device buffer at byte `off`;
    returns (frame bytes, whether anything outside the frame changed)."""
    import torch
    import netidx_amd
    cols = netidx_amd.columns_from_arrays(ids, vals)
    n = codec.encoded_len(cols)
    buf = torch.full((n + off + 64,), SENT, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # (the fill runs on torch's stream, the encode on the codec's)
    m = codec.encode_into(cols, None, buf.data_ptr() + off, n if cap is None else cap)
    assert m == n
    h = buf.cpu().numpy()
    outside = bool((h[:off] != SENT).any() or (h[off + n:] != SENT).any())
    return h[off:off + n], outside


def _check(codec, ids, vals, off=0, kernel="seq"):
    import nxo
    ref = nxo.encode_f64(ids, vals)
    got, outside = _encode(codec, ids, vals, off)
    assert len(got) == len(ref) and np.array_equal(got, ref), \
        f"encode differs from the oracle (n={len(ids)}, i0={int(ids[0])}, off={off})"
    assert not outside, "bytes written outside the frame"
    if kernel:
        assert codec.last_encode_kernel() == kernel


@pytest.mark.parametrize("i0", [0, 1, 100, 77, 2**14 - 300, 2**21 - 700, 2**28 - 1000,
                                2**35 - 3000])
def test_seq_encode_small_batches_every_phase(codec, i0):
    rng = np.random.default_rng(i0 % 1000 + 7)
    for n in (1, 2, 3, 63, 64, 65, 255, 256, 257, 511, 512, 513, 1000, 2049, 4000):
        n = min(n, 2**35 - i0)
        ids = np.arange(i0, i0 + n, dtype=np.uint64)
        vals = _vals(n, rng)
        for off in ((0, 1, 7, 15) if n in (1, 257, 4000) else (0, 9)):
            _check(codec, ids, vals, off)


@pytest.mark.parametrize("i0,n,off", [(0, 70_001, 3), (2**21 - 1_000_000, 3_000_000, 5),
                                      (2**28 - 12_345, 1_000_003, 0)])
def test_seq_encode_long_batches(codec, i0, n, off):
    rng = np.random.default_rng(n)
    ids = np.arange(i0, i0 + n, dtype=np.uint64)
    _check(codec, ids, _vals(n, rng), off)


def test_seq_encode_hands_over_and_skips():
    """Ids that are not a run of consecutive ids (a swap at the first / a wave edge / the middle /
    the last record, ids past 2^35, random ids): the tiled encoder writes the frame, byte-
    identical; the next 64 f64 encodes skip the sequential kernel, the 65th tries it again."""
    import netidx_amd
    c = netidx_amd.Codec(0)
    try:
        rng = np.random.default_rng(3)
        n = 5000
        base = np.arange(1000, 1000 + n, dtype=np.uint64)
        vals = _vals(n, rng)
        cases = []
        for a in (0, 255, 256, 2500, n - 2):
            ids = base.copy()
            ids[a], ids[a + 1] = ids[a + 1], ids[a]
            cases.append(ids)
        cases.append(np.arange(2**35 - 100, 2**35 + 100, dtype=np.uint64))
        cases.append(rng.integers(0, 2**40, n, dtype=np.uint64))
        for ids in cases:
            c.close()
            c = netidx_amd.Codec(0)  # a fresh connection: the kernel is tried first
            _check(c, ids, vals[:len(ids)], off=3, kernel="tile")
        # skip-and-retry: _encode is two encodes (sizing + writing)
        c.close()
        c = netidx_amd.Codec(0)
        bad = base.copy()
        bad[10] = 7
        _check(c, bad, vals, kernel="tile")  # declined in the sizing pass: 64 encodes skip it
        for k in range(31):
            _check(c, base, vals, kernel="tile")  # 62 more encodes
        _check(c, base, vals, kernel=None)  # the 64th skipped one sizes; the next one writes
        assert c.last_encode_kernel() == "seq"
    finally:
        c.close()


def test_seq_encode_capacity_and_sizing(codec):
    import netidx_amd
    import torch
    import nxo
    n = 3000
    ids = np.arange(5, 5 + n, dtype=np.uint64)
    vals = _vals(n, np.random.default_rng(4))
    ref = nxo.encode_f64(ids, vals)
    cols = netidx_amd.columns_from_arrays(ids, vals)
    assert codec.encoded_len(cols) == len(ref)
    buf = torch.full((len(ref) + 64,), SENT, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    with pytest.raises(netidx_amd.CodecError, match="too small"):
        codec.encode_into(cols, None, buf.data_ptr(), len(ref) - 1)
    assert (buf.cpu().numpy() == SENT).all(), "a declined encode wrote bytes"
    assert codec.encode_into(cols, None, buf.data_ptr(), len(ref) + 64) == len(ref)
    assert np.array_equal(buf[: len(ref)].cpu().numpy(), ref)


def test_seq_encode_async_backlog_with_late_fallback():
    """A backlog of async encodes (sequential, then ids out of order, then sequential) and a
    decode of the second one's output queued behind them: nxg_ctx_sync reruns the declined encode
    on the tiled encoder and, because that rewrote the frame after the decode read it, decodes
    it again; every frame and the decoded columns equal the oracle's."""
    import netidx_amd
    import torch
    import nxo
    from netidx_amd.codec import Columns
    c = netidx_amd.Codec(0)
    try:
        rng = np.random.default_rng(5)
        n = 20_000
        batches = []
        for k in range(3):
            ids = np.arange(100 * k, 100 * k + n, dtype=np.uint64)
            if k == 1:
                ids = rng.permutation(ids)
            batches.append((ids, _vals(n, rng)))
        refs = [nxo.encode_f64(i, v) for i, v in batches]
        cols = [netidx_amd.columns_from_arrays(i, v) for i, v in batches]
        outs = [torch.zeros(len(r) + 64, dtype=torch.uint8, device="cuda") for r in refs]
        torch.cuda.synchronize()
        lens = [c.encode_async(cl, None, o.data_ptr(), o.numel()) for cl, o in zip(cols, outs)]
        dec = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        c.decode_async(outs[1].data_ptr(), len(refs[1]), dec)
        st = c.sync()
        for ln, o, r in zip(lens, outs, refs):
            assert ln.value == len(r) and np.array_equal(o[: len(r)].cpu().numpy(), r)
        o = nxo.decode(refs[1]).trim()
        assert st.n_rows == n
        assert np.array_equal(dec.numpy()["id"], o["id"])
        assert np.array_equal(dec.numpy()["fixed"], o["fixed"])
    finally:
        c.close()
