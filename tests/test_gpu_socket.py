"""End to end through a loopback TCP socket (the path starts and ends in a socket buffer):
publisher = device encode (nxg_encode_updates) + flush_buf framing; subscriber = read_task
reassembly (nxg_frame_reader_*) + device decode of each host frame (nxg_decode_updates stages it
H2D). Checks the decoded columns and a byte-identical re-encode."""
import socket
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_loopback_mixed_batches():
    import torch
    import netidx_amd
    from netidx_amd import synth
    pub, sub = netidx_amd.Codec(0), netidx_amd.Codec(0)
    batches = []
    for k in range(3):
        m = synth.mixed_columns(50_000 + 1000 * k)
        mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
        heap = torch.from_numpy(m.heap.copy()).cuda()
        batches.append((mc, heap, pub.encode_batch(mc, heap).cpu().numpy().tobytes()))
    srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]

    def publisher():
        c = socket.create_connection(("127.0.0.1", port))
        for _, _, wire in batches:
            c.sendall(netidx_amd.frame_header(len(wire)) + wire)
        c.close()

    t = threading.Thread(target=publisher)
    t.start()
    conn, _ = srv.accept()
    r = netidx_amd.FrameReader()
    got = []
    buf = bytearray(1 << 16)
    while True:
        n = conn.recv_into(buf)
        if not n:
            break
        r.feed(buf, n)
        got.extend(r.frames())
    t.join()
    conn.close()
    srv.close()
    assert [len(f) for f in got] == [len(w) for _, _, w in batches]
    for f, (mc, heap, wire) in zip(got, batches):
        assert f == wire
        cols, st = sub.decode_batch(torch.from_numpy(np.frombuffer(f, np.uint8).copy()).cuda())
        n = mc.s.n_rows
        assert st.err_kind == 0 and st.n_rows == n
        assert torch.equal(cols.id[:n], mc.id[:n]) and torch.equal(cols.tag[:n], mc.tag[:n])
        frame = torch.from_numpy(np.frombuffer(f, np.uint8).copy()).cuda()
        assert sub.encode_batch(cols, frame).cpu().numpy().tobytes() == wire


def _config1_pub(lst, pub, batches, heaps, res):
    """The publisher side of a session: accept + handshake, To::Subscribe -> From::Subscribed,
    then each batch of device columns encoded on the GPU and written as frames."""
    import netidx_amd
    try:
        s = lst.accept()
        m = netidx_amd.msg_parse(s.recv_frame(), to=True)
        res["sub"] = (m.variant, m.path_len)
        s.send(netidx_amd.msg_subscribed("/local/bench/0", 0, 16))
        for cols, heap in zip(batches, heaps):
            s.publish(pub, cols, heap)
        res["stats"] = s.stats()
        s.close()
    except Exception as e:  # surfaced by the test
        res["err"] = repr(e)


@pytest.mark.parametrize("kind", ["f64", "mixed"])
def test_session_end_to_end(kind):
    """BASELINE configs[0]'s data path through the library only: nxg_session_* handshake and
    subscription, nxg_session_publish (GPU encode -> pinned -> socket) and
    nxg_session_recv_decode (socket -> pinned -> GPU decode). The decoded device columns equal the
    generator's columns; each frame's bytes equal the oracle encoder's."""
    import torch
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    pub, sub = netidx_amd.Codec(0), netidx_amd.Codec(0)
    batches, heaps, ref = [], [], []
    for k in range(3):
        n = 200_000 + 7 * k
        if kind == "f64":
            ids, vals = synth.f64_columns(n, 300 + k)
            batches.append(netidx_amd.columns_from_arrays(ids, vals))
            heaps.append(None)
            ref.append((ids, vals, None))
        else:
            m = synth.mixed_columns(n, 400 + k)
            batches.append(netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag,
                                                          m.cfixed, m.caux))
            heaps.append(torch.from_numpy(m.heap.copy()).cuda())
            ref.append((m.id, m.fixed, m))
    lst = netidx_amd.Session.listen()
    res = {}
    t = threading.Thread(target=_config1_pub, args=(lst, pub, batches, heaps, res))
    t.start()
    s = netidx_amd.Session.connect("127.0.0.1", lst.port)
    s.send(netidx_amd.msg_subscribe("/local/bench/0"))
    first = netidx_amd.msg_parse(s.recv_frame())
    assert first.variant == 3 and first.value_tag == 16
    for k, (ids, vals, m) in enumerate(ref):
        n = len(ids)
        layout = netidx_amd.LAYOUT_F64 if m is None else netidx_amd.LAYOUT_MIXED
        out = Columns(n + 1, (len(m.ctag) + 1) if m is not None else 0, 1, layout, "cuda")
        st, flen = s.recv_decode(sub, out, 0 if m is None else netidx_amd.HINT_MIXED)
        assert st.err_kind == 0 and st.n_rows == n
        g = out.numpy()
        assert np.array_equal(g["id"][:n], ids)
        if m is None:
            assert np.array_equal(g["fixed"][:n], vals)
            assert flen == len(nxo.encode_f64(ids, vals))
        else:
            assert np.array_equal(g["tag"][:n], m.tag)
            assert np.array_equal(g["ctag"][:len(m.ctag)], m.ctag)
            plain = (m.tag != 12) & (m.tag != 19)
            assert np.array_equal(g["fixed"][:n][plain], m.fixed[plain])
    t.join()
    s.close()
    lst.close()
    assert "err" not in res, res.get("err")
    assert res["sub"] == (0, len("/local/bench/0")) and res["stats"]["frames_out"] == 4
