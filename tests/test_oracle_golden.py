"""The CPU oracle pinned against the golden fixtures and the reference's own tests (CPU only).

Reference tests restated here:
* varint round trip: netidx-core/src/test.rs:16-63 (all d in [0, 2^32) with a 7-byte buffer
  is sampled in strides here; the full sweep runs under -m slow);
* encoded_len == bytes written and decode(encode(x)) == x: netidx-netproto/src/test.rs:15-21;
* decoding random bytes never crashes: netidx-netproto/src/test.rs:449-456.
"""
import json
import os
import random
import struct

import numpy as np
import pytest

import nxo

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "manifest.json")))
KAT = json.load(open(os.path.join(GOLD, "kat.json")))


def test_varint_sweep_short_buffer():
    L = nxo.lib()
    # strided sample of the u32 sweep (test.rs:43-49) + the low range exhaustively
    assert L.nxo_varint_sweep(0, 1 << 22, 1) == 0
    for lo in range(0, 1 << 32, 1 << 26):
        assert L.nxo_varint_sweep(lo, lo + 4096, 1) == 0
    assert L.nxo_varint_sweep((1 << 32) - 4096, 1 << 32, 1) == 0


@pytest.mark.slow
def test_varint_sweep_full_u32():
    assert nxo.lib().nxo_varint_sweep(0, 1 << 32, 1) == 0


def test_varint_len_boundaries():
    L = nxo.lib()
    for k in range(1, 10):
        assert L.nxo_varint_len((1 << (7 * k)) - 1) == k
        assert L.nxo_varint_len(1 << (7 * k)) == k + 1
    assert L.nxo_varint_len(0) == 1
    assert L.nxo_varint_len(2**64 - 1) == 10


def test_kats_decode_roundtrip():
    for k in KAT:
        b = bytes.fromhex(k["hex"])
        if b[0] in (0x0a, 0x05, 0x07):  # bare Value vectors: wrap as Update(Id 0, v)
            continue
        d = nxo.decode(b)
        t = d.trim()
        assert t["err_kind"] == 0, k["name"]
        assert nxo.encode(d, b) == b, k["name"]


@pytest.mark.parametrize("b", MANIFEST["batches"], ids=lambda b: b["name"])
def test_golden_batches(b):
    wire = open(os.path.join(GOLD, b["file"]), "rb").read()
    d = nxo.decode(wire)
    t = d.trim()
    e = b["expect"]
    assert t["err_kind"] == 0
    rows = [list(map(int, r)) for r in zip(t["id"], t["tag"], t["fixed"], t["aux"])]
    assert rows == e["rows"]
    ch = [list(map(int, r)) for r in zip(t["ctag"], t["cfixed"], t["caux"])]
    assert ch == e["children"]
    ctl = [list(map(int, r)) for r in zip(t["ctl_row"], t["ctl_off"], t["ctl_len"], t["ctl_variant"])]
    assert ctl == e["ctl"]
    assert t["n_heartbeat"] == e["n_heartbeat"]
    # round trip: canonical input re-encodes byte-identically
    assert nxo.encode(d, wire) == wire


@pytest.mark.parametrize("c", MANIFEST["errors"], ids=lambda c: c["name"])
def test_golden_errors(c):
    t = nxo.decode(bytes.fromhex(c["hex"])).trim()
    assert (t["err_kind"], t["err_offset"]) == (c["kind"], c["offset"])


@pytest.mark.parametrize("c", MANIFEST["edge_ok"], ids=lambda c: c["name"])
def test_golden_edge_ok(c):
    t = nxo.decode(bytes.fromhex(c["hex"])).trim()
    assert t["err_kind"] == 0
    rows = [list(map(int, r)) for r in zip(t["id"], t["tag"], t["fixed"], t["aux"])]
    assert rows == c["rows"]


@pytest.mark.parametrize("b", MANIFEST["archive"], ids=lambda b: b["name"])
def test_golden_archive(b):
    """Archive batches (Vec<BatchItem>, netidx-archive/src/logfile/mod.rs:188-205): every row and
    child against the twin's expected decode, the bytes consumed, and the re-encode."""
    wire = open(os.path.join(GOLD, b["file"]), "rb").read()
    d, consumed = nxo.decode_archive(wire)
    t = d.trim()
    e = b["expect"]
    assert t["err_kind"] == 0 and consumed == b["consumed"]
    rows = [list(map(int, r)) for r in zip(t["id"], t["tag"], t["fixed"], t["aux"])]
    assert rows == e["rows"]
    ch = [list(map(int, r)) for r in zip(t["ctag"], t["cfixed"], t["caux"])]
    assert ch == e["children"]
    assert nxo.encode_archive(d, wire) == wire[:consumed]


@pytest.mark.parametrize("c", MANIFEST["archive_errors"], ids=lambda c: c["name"])
def test_golden_archive_errors(c):
    d, r = nxo.decode_archive(bytes.fromhex(c["hex"]))
    t = d.trim()
    assert (t["err_kind"], t["err_offset"]) == (c["kind"], c["offset"]) and r == -c["kind"]


@pytest.mark.parametrize("c", MANIFEST["archive_edge_ok"], ids=lambda c: c["name"])
def test_golden_archive_edge_ok(c):
    d, consumed = nxo.decode_archive(bytes.fromhex(c["hex"]))
    t = d.trim()
    assert t["err_kind"] == 0 and consumed == c["consumed"]
    rows = [list(map(int, r)) for r in zip(t["id"], t["tag"], t["fixed"], t["aux"])]
    assert rows == c["rows"]


def test_encode_f64_matches_decode():
    rng = np.random.default_rng(7)
    ids = rng.integers(0, 2**63, 5000, dtype=np.uint64)
    ids[:100] = np.arange(100)
    vals = rng.integers(0, 2**63, 5000, dtype=np.uint64)
    w = nxo.encode_f64(ids, vals)
    t = nxo.decode(w).trim()
    assert t["err_kind"] == 0
    assert np.array_equal(t["id"], ids) and np.array_equal(t["fixed"], vals)
    assert (t["tag"] == 9).all()


def test_datetime_validity_rules():
    L = nxo.lib()
    assert L.nxo_datetime_valid(0, 0)
    assert L.nxo_datetime_valid(-1, 999999999)
    assert not L.nxo_datetime_valid(0, 1000000000)
    assert L.nxo_datetime_valid(59, 1999999999)
    assert not L.nxo_datetime_valid(59, 2000000000)
    assert not L.nxo_datetime_valid(2**62, 0)


def test_utf8_rules():
    L = nxo.lib()
    ok = ["", "abc", "é", "€", "😀", "߿", "￿", "\U0010ffff"]
    for s in ok:
        b = s.encode()
        assert L.nxo_utf8_valid(b, len(b)), s
    bad = [b"\x80", b"\xc0\x80", b"\xc1\xbf", b"\xe0\x80\x80", b"\xed\xa0\x80", b"\xf4\x90\x80\x80",
           b"\xf5\x80\x80\x80", b"\xc3", b"\xe2\x82", b"\xff"]
    for b in bad:
        assert not L.nxo_utf8_valid(b, len(b)), b


def test_fuzz_never_crashes():
    rng = random.Random(1234)
    for _ in range(3000):
        n = rng.randrange(0, 64)
        b = bytes(rng.getrandbits(8) for _ in range(n))
        t = nxo.decode(b).trim()
        assert t["err_kind"] in (0, 1, 2, 3, 4, 6)
