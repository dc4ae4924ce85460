"""Host framing on the CPU: read_task's frame assembly (nxg_frame_reader_*, channel.rs:379-443)
fed a byte stream cut at arbitrary points, and BASELINE configs[0] -- a publisher and a
subscriber of one f64 path over a loopback TCP socket (CPU-only plumbing: the frames are made
and parsed by the library's host code; the oracle stands in for the codec since this config
has no GPU)."""
import random
import socket
import struct
import threading

import numpy as np
import pytest

import netidx_amd
import nxo


def frames_of(payloads, encrypted=None):
    out = b""
    for k, p in enumerate(payloads):
        out += netidx_amd.frame_header(len(p), bool(encrypted and encrypted[k])) + p
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_reader_reassembles_any_cut(seed):
    rng = random.Random(seed)
    payloads = [bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 5, 300, 5000])))
                for _ in range(40)]
    stream = frames_of(payloads)
    r = netidx_amd.FrameReader()
    got, i = [], 0
    while i < len(stream):
        k = rng.choice([1, 2, 3, 7, 100, 4096])
        r.feed(stream[i:i + k])
        i += k
        got.extend(r.frames())
    assert got == payloads
    assert r.buffered() == 0


def test_reader_waits_for_the_whole_frame():
    r = netidx_amd.FrameReader()
    r.feed(struct.pack(">I", 10) + b"12345")
    assert list(r.frames()) == [] and r.buffered() == 9
    r.feed(b"67890" + struct.pack(">I", 0))
    assert list(r.frames()) == [b"1234567890", b""]


def test_reader_rejects_encrypted_frames():
    # bit 31 set: a krb5-wrapped frame; without a security context read_task fails with
    # "encryption is not supported" (channel.rs:420-422)
    r = netidx_amd.FrameReader()
    r.feed(frames_of([b"ok", b"secret"], encrypted=[False, True]))
    it = r.frames()
    assert next(it) == b"ok"
    with pytest.raises(netidx_amd.CodecError, match="encryption is not supported"):
        next(it)


def test_config1_loopback_one_f64_path():
    """simple_publisher / simple_subscriber (BASELINE configs[0]) reduced to the data path: the
    publisher sends From::Update(Id(0), F64(x)) for a series of values, one batch per update, as
    flush_buf frames them; the subscriber reassembles frames with read_task's logic and decodes."""
    vals = [1.0, -0.0, 2.5, float("inf"), 1e-300, 3.25]
    srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]

    def publisher():
        c = socket.create_connection(("127.0.0.1", port))
        for v in vals:
            bits = np.array([struct.unpack("<Q", struct.pack("<d", v))[0]], np.uint64)
            wire = nxo.encode_f64(np.array([0], np.uint64), bits).tobytes()
            c.sendall(netidx_amd.frame_header(len(wire)) + wire)
        c.close()

    t = threading.Thread(target=publisher)
    t.start()
    conn, _ = srv.accept()
    r = netidx_amd.FrameReader()
    got = []
    while True:
        data = conn.recv(7)  # small reads: frames arrive in pieces
        if not data:
            break
        r.feed(data)
        for f in r.frames():
            d = nxo.decode(f)
            assert d.s.err_kind == 0 and d.s.n_rows == 1 and d.id[0] == 0
            got.append(struct.unpack("<d", struct.pack("<Q", int(d.fixed[0])))[0])
    t.join()
    conn.close()
    srv.close()
    assert [struct.pack("<d", x) for x in got] == [struct.pack("<d", x) for x in vals]
