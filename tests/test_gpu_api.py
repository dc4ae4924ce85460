"""C-ABI behaviour on the GPU: the MAX_BATCH frame split of the encode seam, async calls and the
status ring.

- nxg_encode_frames cuts the payload exactly as WriteChannel::queue_send + try_flush
  (netidx/src/channel.rs:177-202, 237-257): checked against nxg_frame_split over the oracle's
  message lengths, at 10^8 records (1.498 GB > MAX_BATCH: the reference's two frames).
- async encode into a buffer that is too small fails at nxg_ctx_sync (no frame with holes).
- a call that launches no kernel (an empty frame) still clears the status slot the call 512
  later uses, so a capacity failure two ring laps back cannot leak into a good decode.
- one nxg_ctx_sync finishes every pending call: a decode that needs the general fallback and an
  encode after it both complete.
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


@pytest.fixture(scope="module", params=["seq", "run"])
def dcodec(request):
    """Decode tests run on both f64 front ends: the sequential-id kernel first (the default), and
    the length-run decoder (NXG_F64_PATH=run), whose stream of frames fuses frame j + 1's probe
    into frame j's emit."""
    import os
    import netidx_amd
    os.environ["NXG_F64_PATH"] = "" if request.param == "seq" else "run"
    try:
        c = netidx_amd.Codec(0)
    finally:
        del os.environ["NXG_F64_PATH"]
    yield c
    c.close()


def _vl(ids):
    ids = np.asarray(ids, np.uint64)
    n = np.ones(len(ids), np.int64)
    for k in range(1, 10):
        n += ids >= np.uint64(1 << (7 * k))
    return n


def test_encode_frames_max_batch_split_1e8(codec):
    import netidx_amd
    import nxo
    import torch
    from netidx_amd import synth
    n = 100_000_000
    ids, vals = synth.f64_columns(n, synth.SEED_8GPU)
    cols = netidx_amd.columns_from_arrays(ids, vals)
    out = torch.empty(1_497_886_336 + 64, dtype=torch.uint8, device="cuda")
    total, chunks = codec.encode_frames(cols, None, out.data_ptr(), out.numel())
    assert total == 1_497_886_336
    # the reference's cut: queue_send over the oracle's message lengths (11 + varint_len(id))
    ref_chunks = netidx_amd.frame_split(11 + _vl(ids))
    assert chunks == list(ref_chunks) and len(chunks) == 2 and sum(chunks) == total
    assert chunks[0] <= 0x3FFFFFFF
    del cols
    got = out[:total].cpu().numpy()
    ref = nxo.encode_f64(ids, vals)
    assert np.array_equal(got, ref)
    # the second frame starts with a message (ids near 7.2e7 take 4 varint bytes: L = 15)
    c0 = chunks[0]
    assert ref[c0] == 15 and ref[c0 + 1] == 4


def test_encode_frames_small_and_empty(codec):
    import netidx_amd
    import torch
    from netidx_amd import synth
    ids, vals = synth.f64_columns(1000, 5)
    cols = netidx_amd.columns_from_arrays(ids, vals)
    out = torch.empty(16000, dtype=torch.uint8, device="cuda")
    total, chunks = codec.encode_frames(cols, None, out.data_ptr(), out.numel())
    assert chunks == [total] and total == int((11 + _vl(ids)).sum())
    empty = netidx_amd.columns_from_arrays(np.zeros(0, np.uint64), np.zeros(0, np.uint64))
    total, chunks = codec.encode_frames(empty, None, out.data_ptr(), out.numel())
    assert total == 0 and chunks == []


def test_async_encode_too_small_fails_at_sync(codec):
    import netidx_amd
    import torch
    from netidx_amd import synth
    ids, vals = synth.f64_columns(50_000, 6)
    cols = netidx_amd.columns_from_arrays(ids, vals)
    need = int((11 + _vl(ids)).sum())
    out = torch.empty(need - 100, dtype=torch.uint8, device="cuda")
    codec.encode_async(cols, None, out.data_ptr(), out.numel())
    with pytest.raises(netidx_amd.CodecError):
        codec.sync()
    # the ctx stays usable
    big = torch.empty(need + 16, dtype=torch.uint8, device="cuda")
    ln = codec.encode_async(cols, None, big.data_ptr(), big.numel())
    codec.sync()
    assert ln.value == need


def test_status_ring_empty_call_clears_its_slot(codec):
    """Call i fails with a capacity error; call i + 512 launches nothing (empty frame); call
    i + 1024 reuses call i's slot and must not inherit its bits."""
    import netidx_amd
    import nxo
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    ids, vals = synth.f64_columns(2000, 7)
    wire = torch.from_numpy(nxo.encode_f64(ids, vals)).cuda()
    small = Columns(100, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    good = Columns(2000, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    st = codec.decode_into(wire, wire.numel(), small, check=False)
    assert st.err_kind == netidx_amd.CAPACITY
    for k in range(1, 1025):
        if k == 512:
            st = codec.decode_into(wire, 0, good, check=False)
            assert st.err_kind == 0 and st.n_rows == 0
        else:
            st = codec.decode_into(wire, wire.numel(), good, check=False)
            assert st.err_kind == 0 and st.n_rows == 2000, (k, st.err_kind)


def test_sync_finishes_every_pending_call(codec):
    import netidx_amd
    import nxo
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    ids, vals = synth.f64_columns(30_000, 8)
    w = nxo.encode_f64(ids, vals).tobytes()
    hb = w[:12 * 100] + b"\x02\x05" + w[12 * 100:]  # a Heartbeat between records 99 and 100
    d_plain = torch.from_numpy(np.frombuffer(w, np.uint8).copy()).cuda()
    d_hb = torch.from_numpy(np.frombuffer(hb, np.uint8).copy()).cuda()
    outs = [Columns.for_frame(len(x), netidx_amd.LAYOUT_MIXED, "cuda") for x in (w, hb, w)]
    cols = netidx_amd.columns_from_arrays(ids, vals)
    eout = torch.empty(len(w) + 16, dtype=torch.uint8, device="cuda")
    codec.decode_async(d_plain.data_ptr(), len(w), outs[0])
    codec.decode_async(d_hb.data_ptr(), len(hb), outs[1])
    ln = codec.encode_async(cols, None, eout.data_ptr(), eout.numel())
    codec.decode_async(d_plain.data_ptr(), len(w), outs[2])
    codec.sync()
    for o, x in zip(outs, (w, hb, w)):
        ref = nxo.decode(x).trim()
        g = o.numpy()
        assert np.array_equal(g["id"], ref["id"]) and np.array_equal(g["fixed"], ref["fixed"])
    assert outs[1].s.n_heartbeat == 1
    assert ln.value == len(w) and eout[: len(w)].cpu().numpy().tobytes() == w


@pytest.mark.parametrize("seed", [11, 12])
def test_decode_frames_stream(dcodec, seed):
    """nxg_decode_frames_async: a backlog of frames of varied shape, each into its own columns --
    f64 frames of odd and even record counts (the 16-byte pair stores at both row parities),
    ids across the varint widths, an empty frame, a frame with a Heartbeat (the fast path rejects
    it, the fallback decodes it), a frame with ids in random order (the irregular-frame path) --
    every column against the oracle's decode of the same bytes."""
    import netidx_amd
    import nxo
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    rng = np.random.default_rng(seed)
    frames = []
    for k, n in enumerate([1, 2, 3, 129, 257, 70_001, 0, 250_000, 40_000, 100_000, 5]):
        ids, vals = synth.f64_columns(n, seed * 100 + k, id_offset=int(rng.integers(0, 3)) * 16_000)
        if k == 8:  # random order: record lengths vary record to record
            ids = rng.permutation(np.arange(n, dtype=np.uint64) + np.uint64(2**21 - 20_000))
        w = nxo.encode_f64(ids, vals).tobytes()
        if k == 9:  # a Heartbeat between records 499 and 500
            w = (nxo.encode_f64(ids[:500], vals[:500]).tobytes() + b"\x02\x05" +
                 nxo.encode_f64(ids[500:], vals[500:]).tobytes())
        frames.append(w)
    dev = [torch.from_numpy(np.frombuffer(w, np.uint8).copy()).cuda() if w else
           torch.empty(16, dtype=torch.uint8, device="cuda") for w in frames]
    outs = [Columns.for_frame(max(len(w), 16), netidx_amd.LAYOUT_MIXED, "cuda") for w in frames]
    dcodec.decode_frames_async([d.data_ptr() for d in dev], [len(w) for w in frames], outs)
    dcodec.sync()
    for w, o in zip(frames, outs):
        ref = nxo.decode(w).trim()
        g = o.numpy()
        assert o.s.n_rows == len(ref["id"])
        assert np.array_equal(g["id"], ref["id"]) and np.array_equal(g["fixed"], ref["fixed"])
    assert outs[9].s.n_heartbeat == 1


def test_decode_frames_stream_shared_columns_1e7(dcodec):
    """The bench's shape: one 10^7-record f64 frame decoded 6 times as a stream into one set of
    columns (the probe of frame j + 1 runs beside the emit of frame j), bit-exact."""
    import netidx_amd
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n = 10_000_000
    ids, vals = synth.f64_columns(n, synth.SEED_F64)
    cols = netidx_amd.columns_from_arrays(ids, vals)
    wire = dcodec.encode_batch(cols)
    out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    for rep in range(2):
        out.id.zero_()
        out.fixed.zero_()
        dcodec.decode_frames_async([wire.data_ptr()] * 6, [wire.numel()] * 6, [out] * 6)
        st = dcodec.sync()
        assert st.path == 1 and st.n_rows == n
        assert torch.equal(out.id[:n], cols.id[:n]) and torch.equal(out.fixed[:n], cols.fixed[:n])


def test_async_fallback_frame_overwritten_fails_loudly():
    """A decode that falls back in nxg_ctx_sync re-reads its frame after the later calls of the
    backlog ran. A later async encode that wrote into that frame buffer (stream-ordered reuse)
    makes the sync fail with a clear error instead of decoding the overwritten bytes;
    the context stays usable, and the same backlog without the reuse decodes bit-exact."""
    import netidx_amd
    import nxo
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    c = netidx_amd.Codec(0)
    try:
        rng = np.random.default_rng(77)
        n = 50_000
        ids, vals = synth.f64_columns(n, 78)
        ids = rng.permutation(ids)  # the sequential-id kernel declines: a fallback at sync
        w = nxo.encode_f64(ids, vals)
        frame = torch.from_numpy(w.copy()).cuda()
        out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        i2, v2 = synth.f64_columns(n, 79)
        cols2 = netidx_amd.columns_from_arrays(i2, v2)
        c.decode_async(frame.data_ptr(), frame.numel(), out)
        c.encode_async(cols2, None, frame.data_ptr(), frame.numel())  # writes into the frame
        with pytest.raises(netidx_amd.CodecError, match="wrote into that frame"):
            c.sync()
        # without the reuse: the same backlog shape decodes bit-exact
        frame = torch.from_numpy(w.copy()).cuda()
        eout = torch.empty(frame.numel() + 64, dtype=torch.uint8, device="cuda")
        c.decode_async(frame.data_ptr(), frame.numel(), out)
        c.encode_async(cols2, None, eout.data_ptr(), eout.numel())
        st = c.sync()
        ref = nxo.decode(w).trim()
        assert st.n_rows == n
        assert np.array_equal(out.numpy()["id"], ref["id"])
        assert np.array_equal(out.numpy()["fixed"], ref["fixed"])
    finally:
        c.close()
