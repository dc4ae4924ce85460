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
