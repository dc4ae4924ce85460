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


VERSION_RAW = bytes.fromhex("00000008" "0000000000000003")  # write_raw(&3u64), channel.rs:63-80
HELLO_ANON_RAW = bytes.fromhex("00000002" "0200")          # Hello::Anonymous: lw(1)=2, variant 0


def recv_exact(c, n):
    b = b""
    while len(b) < n:
        k = c.recv(n - len(b))
        assert k, "connection closed"
        b += k
    return b


def test_handshake_bytes_subscriber_side():
    """A hand-written publisher (the bytes of ClientCtx::hello, publisher/server.rs:367-381)
    against the library's subscriber (hello_publisher, subscriber/connection.rs:120-140)."""
    srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    got = {}

    def publisher():
        c, _ = srv.accept()
        c.sendall(VERSION_RAW)
        got["version"] = recv_exact(c, 12)
        got["hello"] = recv_exact(c, 6)
        c.sendall(HELLO_ANON_RAW)
        # the channel: the subscriber's first frame is To::Subscribe
        n = struct.unpack(">I", recv_exact(c, 4))[0]
        got["subscribe"] = recv_exact(c, n)
        c.close()

    t = threading.Thread(target=publisher)
    t.start()
    s = netidx_amd.Session.connect("127.0.0.1", port)
    s.send(netidx_amd.msg_subscribe("/foo/bar", timestamp=7, permissions=3))
    t.join()
    s.close()
    srv.close()
    assert got["version"] == VERSION_RAW and got["hello"] == HELLO_ANON_RAW
    # To::Subscribe {path, resolver V4 0.0.0.0:0, timestamp u64, permissions u32, token Bytes}
    body = (b"\x00" + b"\x08/foo/bar" + b"\x00" + bytes(6) + struct.pack(">QI", 7, 3) + b"\x00")
    assert got["subscribe"] == bytes([len(body) + 1]) + body
    m = netidx_amd.msg_parse(got["subscribe"], to=True)
    assert (m.variant, m.timestamp, m.permissions, m.path_len) == (0, 7, 3, 8)


def test_handshake_bytes_publisher_side():
    """A hand-written subscriber against the library's publisher: the version and Hello bytes,
    and a Hello other than Anonymous refused."""
    lst = netidx_amd.Session.listen()
    res = {}

    def accept():
        try:
            res["s"] = lst.accept()
        except netidx_amd.CodecError as e:
            res["err"] = str(e)

    for hello, ok in ((HELLO_ANON_RAW, True), (bytes.fromhex("00000002" "0202"), False)):
        res.clear()
        t = threading.Thread(target=accept)
        t.start()
        c = socket.create_connection(("127.0.0.1", lst.port))
        assert recv_exact(c, 12) == VERSION_RAW
        c.sendall(VERSION_RAW + hello)
        if ok:
            assert recv_exact(c, 6) == HELLO_ANON_RAW
        t.join()
        c.close()
        if ok:
            res["s"].close()
        else:
            assert "not supported" in res["err"]
    lst.close()


def test_bogus_frame_length_allocates_nothing_up_front():
    """A peer that sends a frame header claiming 1 GiB and then a few bytes before closing: the
    receive fails with the connection closed, quickly, and the receive buffer grew only with the
    bytes that came (read_task grows its buffer as bytes arrive, channel.rs:426-437)."""
    import time
    srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]

    def publisher():
        c, _ = srv.accept()
        c.sendall(VERSION_RAW)
        recv_exact(c, 18)
        c.sendall(HELLO_ANON_RAW)
        c.sendall(struct.pack(">I", 1 << 30) + b"x" * 10)
        c.close()

    t = threading.Thread(target=publisher)
    t.start()
    s = netidx_amd.Session.connect("127.0.0.1", port)
    t0 = time.perf_counter()
    with pytest.raises(netidx_amd.CodecError, match="closed"):
        s.recv_frame()
    assert time.perf_counter() - t0 < 5
    t.join()
    s.close()
    srv.close()


def test_control_messages():
    """From::Subscribed / Heartbeat built and parsed by the library; every byte derived from the
    derive rules (lib.rs:289-381) and Value::encode (value lib.rs:361-468)."""
    m = netidx_amd.msg_subscribed("/a", 5, 9, struct.unpack("<Q", struct.pack("<d", 1.5))[0])
    # body: variant 1 + path 3 + id 1 + value 9 = 14 bytes; lw(14) = 15
    assert m == bytes([15, 3, 2]) + b"/a" + b"\x05\x09" + struct.pack(">d", 1.5)
    p = netidx_amd.msg_parse(m)
    assert (p.variant, p.id, p.value_tag, p.path_off, p.path_len) == (3, 5, 9, 3, 2)
    assert struct.pack(">Q", p.value_fixed) == struct.pack(">d", 1.5)
    assert netidx_amd.msg_heartbeat() == b"\x02\x05"
    assert netidx_amd.msg_parse(b"\x02\x05").variant == 5
    s = netidx_amd.msg_subscribed("/s", 1, 12, 0, 3, b"abc")
    p = netidx_amd.msg_parse(s)
    assert p.value_tag == 12 and s[p.value_fixed:p.value_fixed + p.value_aux] == b"abc"
    # agrees with the oracle's decode of the same message as a control span
    d = nxo.decode(m).trim()
    assert len(d["ctl_variant"]) == 1 and d["ctl_variant"][0] == 3 and d["ctl_len"][0] == len(m)


def test_config1_loopback_one_f64_path():
    """simple_publisher / simple_subscriber (BASELINE configs[0], examples/examples/
    simple_publisher.rs:21-47, simple_subscriber.rs:21-55) over loopback TCP, every byte on the
    wire made by the library: a machine-local resolver (nxg_resolver_*), the publisher publishes
    its path there (ClientHello::WriteOnly, ToWrite::Publish), the subscriber resolves it
    (ClientHello::ReadOnly, ToRead::Resolve -> FromRead::Publisher + Resolved) and connects to the
    address it got; then the session handshake, To::Subscribe, From::Subscribed with the current
    value, one From::Update per value (nxg_msg_update) and Heartbeats, each in its own frame. No
    GPU in this config. The oracle only checks the received updates."""
    vals = [1.0, -0.0, 2.5, float("inf"), 1e-300, 3.25]
    bits = [struct.unpack("<Q", struct.pack("<d", v))[0] for v in vals]
    path = "/local/bench/0"
    res = netidx_amd.Resolver()
    lst = netidx_amd.Session.listen()
    wc = netidx_amd.ResolverClient.write("127.0.0.1", res.port, ("127.0.0.1", lst.port))
    wc.publish(path)
    assert res.n_published() == 1 and wc.ttl == 120
    done = {}

    def publisher():
        s = lst.accept()
        sub = netidx_amd.msg_parse(s.recv_frame(), to=True)
        done["path"] = sub.variant, sub.path_len
        s.send(netidx_amd.msg_subscribed(path, 0, 9, bits[0]))
        for k, b in enumerate(bits[1:]):
            if k % 2:
                s.send(netidx_amd.msg_heartbeat())
            s.send(netidx_amd.msg_update(0, 9, b))
        done["stats"] = s.stats()
        s.close()

    t = threading.Thread(target=publisher)
    t.start()
    rc = netidx_amd.ResolverClient.read("127.0.0.1", res.port)
    r = rc.resolve(path)
    assert r.n_publishers == 1 and r.addr == ("127.0.0.1", lst.port)
    assert r.permissions == 0x3F and r.resolver_port == res.port
    sub = netidx_amd.Session.connect(*r.addr)
    sub.send(netidx_amd.msg_subscribe(path, timestamp=r.timestamp, permissions=r.permissions,
                                      resolver=(r.resolver_ipv4, r.resolver_port)))
    first = netidx_amd.msg_parse(sub.recv_frame())
    assert first.variant == 3 and first.id == 0 and first.value_tag == 9
    got, hb = [first.value_fixed], 0
    while len(got) < len(vals):
        f = sub.recv_frame()
        m = netidx_amd.msg_parse(f)
        if m.variant == 5:
            hb += 1
            continue
        assert m.variant == 4 and m.id == 0 and m.value_tag == 9 and m.msg_len == len(f)
        d = nxo.decode(f).trim()  # checker
        assert d["err_kind"] == 0 and int(d["fixed"][0]) == m.value_fixed
        got.append(m.value_fixed)
    t.join()
    st = sub.stats()
    sub.close()
    lst.close()
    rc.close()
    wc.close()
    res.stop()
    assert got == bits and hb == 2 and done["path"] == (0, len(path))
    assert st["frames_in"] == len(vals) + hb and done["stats"]["frames_out"] == len(vals) + hb


def test_msg_update_bytes():
    """From::Update built by the library: SURVEY.md Appendix B's known answers."""
    one = struct.unpack("<Q", struct.pack("<d", 1.0))[0]
    assert netidx_amd.msg_update(0, 9, one).hex() == "0c0400093ff0000000000000"
    nz = struct.unpack("<Q", struct.pack("<d", -0.0))[0]
    assert netidx_amd.msg_update(128, 9, nz).hex() == "0d0480010980" + "00" * 7
    assert netidx_amd.msg_update(0, 16).hex() == "04040010"
    assert netidx_amd.msg_update(5, 12, 0, 120, b"a" * 120).hex() == "7d04050c78" + "61" * 120
    for v in (0, 1, 2**21, 2**35 + 3):
        m = netidx_amd.msg_update(v, 6, 2**64 - 5)
        d = nxo.decode(m).trim()
        assert d["err_kind"] == 0 and int(d["id"][0]) == v and int(d["fixed"][0]) == 2**64 - 5
