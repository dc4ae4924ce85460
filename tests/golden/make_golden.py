#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

This is an independent pure-Python restatement of the reference wire rules. It shares no code
with the C oracle (oracle/nx_oracle.c) or with the HIP codec. It pins the oracle with:

* Known-answer vectors hand-derived from the reference rules. Each one
  cites the rule it follows.
* Small message batches that cover every From variant and every Value wire tag. For each batch
  the fixture holds the wire bytes and the expected columnar decode.
* Malformed inputs with their expected (PackError kind, first failing message offset).

The reference is Rust only and cannot run in this image. These vectors
are derived from its source text, not produced by executing it.

Usage: python tests/golden/make_golden.py   (rewrites tests/golden/*.json and *.bin)
"""
import json
import os
import random
import struct

HERE = os.path.dirname(os.path.abspath(__file__))

# --- primitives: netidx-core/src/pack.rs:472-555 -------------------------------------------


def varint_len(v):  # pack.rs:472-474
    hb = (v | 1).bit_length() - 1
    return (hb * 9 + 73) >> 6


def enc_varint(v):  # pack.rs:476-486
    out = bytearray()
    for _ in range(10):
        if v < 0x80:
            out.append(v)
            break
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    return bytes(out)


def lw(n):  # pack.rs:522-525
    return n + varint_len(n + varint_len(n))


def zz32(n):
    return ((n << 1) ^ (n >> 31)) & 0xFFFFFFFF


def zz64(n):
    return ((n << 1) ^ (n >> 63)) & 0xFFFFFFFFFFFFFFFF


# --- Value model: ("tag", payload) ---------------------------------------------------------
# U32 0, V32 1, I32 2, Z32 3, U64 4, V64 5, I64 6, Z64 7, F32 8, F64 9, DateTime 10,
# Duration 11, String 12, Bytes 13, true 14, false 15, Null 16, Error(String) 18, Array 19,
# Decimal 20, Map 21, Error(other) 22, U8 23, I8 24, U16 25, I16 26, Abstract 27
# (netidx-value/src/lib.rs:361-468)


def enc_value(v):
    t, p = v
    if t in (0,):
        return b"\x00" + struct.pack(">I", p)
    if t == 1:
        return b"\x01" + enc_varint(p)
    if t == 2:
        return b"\x02" + struct.pack(">i", p)
    if t == 3:
        return b"\x03" + enc_varint(zz32(p))
    if t == 4:
        return b"\x04" + struct.pack(">Q", p)
    if t == 5:
        return b"\x05" + enc_varint(p)
    if t == 6:
        return b"\x06" + struct.pack(">q", p)
    if t == 7:
        return b"\x07" + enc_varint(zz64(p))
    if t == 8:
        return b"\x08" + struct.pack(">I", p)  # f32 bit pattern
    if t == 9:
        return b"\x09" + struct.pack(">Q", p)  # f64 bit pattern
    if t == 10:
        return b"\x0a" + struct.pack(">qI", p[0], p[1])
    if t == 11:
        return b"\x0b" + struct.pack(">QI", p[0], p[1])
    if t in (12, 13, 18):
        return bytes([t]) + enc_varint(len(p)) + p
    if t in (14, 15, 16):
        return bytes([t])
    if t == 19:
        return b"\x13" + enc_varint(len(p)) + b"".join(enc_value(e) for e in p)
    if t == 20:
        return b"\x14" + p
    if t == 21:
        return b"\x15" + enc_varint(len(p)) + b"".join(enc_value(k) + enc_value(x) for k, x in p)
    if t == 22:
        return b"\x16" + enc_value(p)
    if t == 23:
        return b"\x17" + struct.pack(">B", p)
    if t == 24:
        return b"\x18" + struct.pack(">b", p)
    if t == 25:
        return b"\x19" + struct.pack(">H", p)
    if t == 26:
        return b"\x1a" + struct.pack(">h", p)
    if t == 27:  # abstract_type.rs:272-278: len-wrapped {uuid, payload}
        content = p
        return b"\x1b" + enc_varint(lw(len(content))) + content
    raise ValueError(t)


def enc_msg(variant, body):
    """netidx-derive enum encode: varint(lw(1+fields)) u8 variant fields (lib.rs:289-381)."""
    inner = bytes([variant]) + body
    return enc_varint(lw(len(inner))) + inner


def update(i, v):
    return enc_msg(4, enc_varint(i) + enc_value(v))


HEARTBEAT = enc_msg(5, b"")


# --- expected columnar decode ---------------------------------------------------------------
class Cols:
    def __init__(self):
        self.rows = []  # (id, tag, fixed, aux)
        self.children = []  # (tag, fixed, aux)
        self.ctl = []  # (row, off, len, variant)
        self.n_heartbeat = 0


def flatten(cols, v, off_of_payload):
    """Expected slot (tag, fixed, aux) of a canonical Value whose wire payload (bytes after
    the tag byte) starts at off_of_payload. Children are allocated depth-first."""
    t, p = v
    signed = {2: 32, 3: 32, 6: 64, 7: 64, 24: 8, 26: 16}
    if t in signed:
        return (t, p & 0xFFFFFFFFFFFFFFFF, 0)
    if t in (0, 1, 4, 5, 8, 9, 23, 25):
        return (t, p, 0)
    if t in (10, 11):
        return (t, p[0] & 0xFFFFFFFFFFFFFFFF, p[1])
    if t in (12, 13, 18):
        return (t, off_of_payload + varint_len(len(p)), len(p))
    if t == 14:
        return (14, 1, 0)
    if t == 15:
        return (15, 0, 0)
    if t == 16:
        return (16, 0, 0)
    if t == 20:
        return (20, off_of_payload, 16)
    if t == 27:
        return (27, off_of_payload + varint_len(lw(len(p))), len(p))
    if t in (19, 21, 22):
        elems = p if t == 19 else ([x for kv in p for x in kv] if t == 21 else [p])
        base = len(cols.children)
        cols.children.extend([None] * len(elems))
        o = off_of_payload + (0 if t == 22 else varint_len(len(p)))
        for i, e in enumerate(elems):
            cols.children[base + i] = flatten(cols, e, o + 1)
            o += len(enc_value(e))
        cnt = len(p) if t != 22 else 1
        return (t, base, cnt)
    raise ValueError(t)


def batch(msgs):
    """msgs: list of ('u', id, value) | ('hb',) | ('raw', variant, body). Returns wire, cols."""
    wire = bytearray()
    cols = Cols()
    for m in msgs:
        start = len(wire)
        if m[0] == "u":
            _, i, v = m
            enc = update(i, v)
            hdr = varint_len(lw(1 + len(enc_varint(i)) + len(enc_value(v))))
            payload_off = start + hdr + 1 + len(enc_varint(i)) + 1
            slot = flatten(cols, v, payload_off)
            cols.rows.append((i,) + slot)
            wire += enc
        elif m[0] == "hb":
            cols.ctl.append((len(cols.rows), start, len(HEARTBEAT), 5))
            cols.n_heartbeat += 1
            wire += HEARTBEAT
        else:
            _, variant, body = m
            enc = enc_msg(variant, body)
            cols.ctl.append((len(cols.rows), start, len(enc), variant))
            wire += enc
    return bytes(wire), cols


def cols_json(c):
    return {
        "rows": [list(r) for r in c.rows],
        "children": [list(r) for r in c.children],
        "ctl": [list(r) for r in c.ctl],
        "n_heartbeat": c.n_heartbeat,
    }


# --- fixture content -------------------------------------------------------------------------
def f64bits(x):
    return struct.unpack(">Q", struct.pack(">d", x))[0]


def f32bits(x):
    return struct.unpack(">I", struct.pack(">f", x))[0]


def kats():
    """SURVEY.md Appendix B, each derived from the cited rule."""
    out = []

    def k(name, got, want_hex, rule):
        assert got.hex() == want_hex.replace(" ", ""), (name, got.hex(), want_hex)
        out.append({"name": name, "hex": got.hex(), "rule": rule})

    k("heartbeat", HEARTBEAT, "02 05", "publisher.rs:95 unit variant 5; lw(1)=2")
    k("update_id0_f64_1", update(0, (9, f64bits(1.0))), "0c 04 00 09 3f f0 00 00 00 00 00 00",
      "lw(1+1+9)=12; f64 BE pack.rs:588")
    k("update_id128_f64_neg0", update(128, (9, f64bits(-0.0))),
      "0d 04 80 01 09 80 00 00 00 00 00 00 00", "varint(128)=80 01")
    k("update_id2p21_f64_2.5", update(1 << 21, (9, f64bits(2.5))),
      "0f 04 80 80 80 01 09 40 04 00 00 00 00 00 00", "vl(2^21)=4")
    k("datetime_1.5s", enc_value((10, (1, 500000000))), "0a 00 00 00 00 00 00 00 01 1d cd 65 00",
      "pack.rs:1563-1565 i64 BE + u32 BE")
    k("v64_300", enc_value((5, 300)), "05 ac 02", "lib.rs:386-389")
    k("z64_minus1", enc_value((7, -1)), "07 01", "zz64(-1)=1")
    s = update(5, (12, b"a" * 120))
    assert len(s) == 125
    k("update_string120", s, "7d 04 05 0c 78" + "61" * 120, "lw(124)=125")
    k("update_null_id0", update(0, (16, None)), "04 04 00 10", "smallest Update")
    body127 = enc_msg(0, enc_varint(125) + b"p" * 125)
    assert len(body127) == 129 and body127[:2] == b"\x81\x01"
    out.append({"name": "body127_prefix", "hex": body127.hex(), "rule": "lw(127)=129 -> 81 01"})
    return out


def rand_value(rng, depth=0):
    t = rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 19, 20, 21,
                    22, 23, 24, 25, 26, 27] if depth < 3 else [4, 9, 12, 16, 24])
    if t == 0:
        return (0, rng.getrandbits(32))
    if t == 1:
        return (1, rng.getrandbits(rng.choice([7, 14, 32])))
    if t == 2:
        return (2, rng.randint(-2**31, 2**31 - 1))
    if t == 3:
        return (3, rng.randint(-2**31, 2**31 - 1))
    if t in (4,):
        return (4, rng.getrandbits(64))
    if t == 5:
        return (5, rng.getrandbits(rng.choice([7, 21, 35, 64])))
    if t == 6:
        return (6, rng.randint(-2**63, 2**63 - 1))
    if t == 7:
        return (7, rng.randint(-2**63, 2**63 - 1))
    if t == 8:
        return (8, rng.getrandbits(32))
    if t == 9:
        return (9, rng.getrandbits(64))
    if t == 10:
        return (10, (rng.randint(-8210266876800, 8210266876799), rng.randrange(10**9)))
    if t == 11:
        return (11, (rng.getrandbits(64), rng.randrange(10**9)))
    if t in (12, 18):
        alphabet = "abcxyz019 é€😀Ωж"
        return (t, "".join(rng.choice(alphabet) for _ in range(rng.randrange(12))).encode())
    if t == 13:
        return (13, bytes(rng.getrandbits(8) for _ in range(rng.randrange(20))))
    if t in (14, 15, 16):
        return (t, None)
    if t == 19:
        return (19, [rand_value(rng, depth + 1) for _ in range(rng.randrange(5))])
    if t == 20:
        return (20, bytes(rng.getrandbits(8) for _ in range(16)))
    if t == 21:
        return (21, [(rand_value(rng, depth + 1), rand_value(rng, depth + 1))
                     for _ in range(rng.randrange(3))])
    if t == 22:
        inner = rand_value(rng, depth + 1)
        if inner[0] == 12:  # Error(String) is canonically tag 18
            return (18, inner[1])
        return (22, inner)
    if t == 23:
        return (23, rng.getrandbits(8))
    if t == 24:
        return (24, rng.randint(-128, 127))
    if t == 25:
        return (25, rng.getrandbits(16))
    if t == 26:
        return (26, rng.randint(-32768, 32767))
    if t == 27:
        return (27, bytes(rng.getrandbits(8) for _ in range(16 + rng.randrange(10))))
    raise ValueError


def path_body(s):
    b = s.encode()
    return enc_varint(len(b)) + b


def batches():
    rng = random.Random(0x5EED0001)
    out = []
    # all-f64, sequential ids (config 2 shape)
    msgs = [("u", i, (9, rng.getrandbits(64))) for i in range(300)]
    out.append(("f64_seq", msgs))
    # f64 with ids spanning 1..5 varint bytes
    msgs = [("u", rng.choice([0, 1, 127, 128, 16383, 16384, 2**21 - 1, 2**21, 2**28 - 1, 2**28,
                               2**35, 2**63]), (9, f64bits(rng.uniform(-1e6, 1e6))))
            for _ in range(200)]
    out.append(("f64_idwidths", msgs))
    # f64 specials
    specials = [0.0, -0.0, float("inf"), float("-inf")]
    msgs = [("u", i, (9, f64bits(x))) for i, x in enumerate(specials)]
    msgs += [("u", 10, (9, 0x7FF8000000000001)), ("u", 11, (9, 0x7FF0000000000001)),
             ("u", 12, (9, 0x0000000000000001)), ("u", 13, (9, 0x800FFFFFFFFFFFFF))]
    out.append(("f64_specials", msgs))
    # every value tag
    msgs = [("u", i, rand_value(rng)) for i in range(400)]
    out.append(("mixed_all_tags", msgs))
    # control messages interleaved
    msgs = [("hb",), ("u", 1, (9, f64bits(1.5))), ("raw", 0, path_body("/a/b")),
            ("raw", 1, path_body("/denied")), ("raw", 2, enc_varint(77)),
            ("raw", 3, path_body("/x") + enc_varint(5) + enc_value((12, b"hi"))),
            ("hb",), ("u", 2, (16, None)),
            ("raw", 6, enc_varint(9) + enc_value((9, f64bits(2.0))) + enc_varint(3)),
            ("raw", 6, enc_varint(9) + enc_value((9, f64bits(2.0)))),  # default WriteId
            ("hb",)]
    out.append(("control", msgs))
    # long strings / arrays: multi-byte length prefixes
    msgs = [("u", 3, (12, b"x" * 200)), ("u", 4, (13, bytes(range(256)) * 70)),
            ("u", 5, (19, [(9, f64bits(float(k))) for k in range(40)])),
            ("u", 6, (12, "é".encode() * 5000))]
    out.append(("long", msgs))
    return out


def errors():
    """(name, wire, kind, offset). Kinds: 1 UnknownTag 2 TooBig 3 InvalidFormat 4 BufferShort."""
    good = update(1, (9, f64bits(1.0)))
    out = [
        ("zero_len", good + b"\x00", 4, len(good)),                      # pack.rs:545-547
        ("unknown_variant", good + enc_msg(7, b""), 1, len(good)),       # derive _ => UnknownTag
        ("unknown_value_tag", good + enc_msg(4, b"\x01\x1c"), 1, len(good)),
        ("truncated_f64", good + good[:-3], 4, len(good)),
        ("f64_short_take", bytes([0x0b]) + good[1:], 4, 0),              # take(10) < needed
        ("bad_utf8", enc_msg(4, b"\x01\x0c\x02\xc3\x28"), 3, 0),
        ("string_toobig", enc_msg(4, b"\x01\x0c\x05ab"), 2, 0),
        ("array_guard", enc_msg(4, b"\x01\x13" + enc_varint(10**6)), 2, 0),
        ("varint_10_cont", good + enc_msg(4, b"\x01\x05" + b"\xff" * 10), 3, len(good)),
        ("datetime_bad_ns", enc_msg(4, b"\x01\x0a" + struct.pack(">qI", 0, 1500000000)), 3, 0),
        ("datetime_out_of_range", enc_msg(4, b"\x01\x0a" + struct.pack(">qI", 2**62, 0)), 3, 0),
        ("empty_variant", b"\x01", 4, 0),
        ("len_varint_short", b"\x80", 4, 0),
        ("second_error_ignored", good + enc_msg(9, b"") + b"\x00", 1, len(good)),
    ]
    return out


def edge_ok():
    """Non-canonical but accepted inputs."""
    out = []
    # 1: non-minimal varint length prefix: 8c 00 => L=12, take(11) after 2 bytes (13 B message)
    body = b"\x04\x00\x09" + struct.pack(">Q", f64bits(3.0))
    out.append(("nonminimal_len", b"\x8c\x00" + body, [(0, 9, f64bits(3.0), 0)]))
    # 2: tag 17 -> Null
    out.append(("tag17_null", enc_msg(4, b"\x07\x11"), [(7, 16, 0, 0)]))
    # 3: V32 truncation of a 64-bit varint
    out.append(("v32_trunc", enc_msg(4, b"\x01\x01" + enc_varint(2**40 + 5)), [(1, 1, 5, 0)]))
    # 5: trailing bytes inside a length-wrapped message are skipped
    out.append(("trailing", enc_msg(4, b"\x02\x10junk"), [(2, 16, 0, 0)]))
    # 6: length prefix past the end of the frame but the value fits: consumes the rest
    w = bytes([0x40]) + b"\x04\x03\x10" + b"zz"
    out.append(("take_past_end", w, [(3, 16, 0, 0)]))
    # 7: Duration nanos >= 1e9 normalised
    out.append(("duration_norm", enc_msg(4, b"\x01\x0b" + struct.pack(">QI", 5, 2500000000)),
                [(1, 11, 7, 500000000)]))
    # leap second accepted at :59
    out.append(("datetime_leap", enc_msg(4, b"\x01\x0a" + struct.pack(">qI", 59, 1500000000)),
                [(1, 10, 59, 1500000000)]))
    # Error(Value) whose inner value is a String normalises to tag 18
    w = enc_msg(4, b"\x01\x16\x0c\x02hi")
    out.append(("error22_string", w, [(1, 18, 6, 2)]))
    return out


# --- archive batches ---------------------------------------------------------------------------
# <Vec<BatchItem> as Pack> (pack.rs:934-973): varint count, then per item varint(Id u32) and an
# Event (netidx/src/subscriber/mod.rs:154-177): 0x40 = Unsubscribed, else a bare Value -- not
# length-wrapped (netidx-archive/src/logfile/mod.rs:150-205).
UNSUB = 0x40


def archive(items, trailing=b""):
    """items: [(id, value or None for Unsubscribed)]. Returns wire, cols (rows carry the u32
    Id), consumed."""
    wire = bytearray(enc_varint(len(items)))
    cols = Cols()
    for i, v in items:
        wire += enc_varint(i)
        if v is None:
            cols.rows.append((i & 0xFFFFFFFF, UNSUB, 0, 0))
            wire.append(UNSUB)
        else:
            slot = flatten(cols, v, len(wire) + 1)
            cols.rows.append((i & 0xFFFFFFFF,) + slot)
            wire += enc_value(v)
    return bytes(wire) + trailing, cols, len(wire)


def archive_batches():
    rng = random.Random(0x5EED0002)
    out = [
        # netidx-archive/src/logfile/test.rs:10-43: every item Event::Update(Value::U64(42))
        ("ref_basic", [(0, (4, 42)), (1, (4, 42))], b""),
        ("empty", [], b""),
        ("unsub_only", [(7, None), (2**32 - 1, None)], b""),
        ("mixed", [(rng.getrandbits(32), None if rng.random() < 0.1 else rand_value(rng))
                   for _ in range(500)], b""),
        ("long", [(3, (12, b"x" * 5000)), (4, (13, bytes(range(256)) * 40)), (5, None),
                  (6, (19, [(9, f64bits(float(k))) for k in range(300)])),
                  (7, (12, "\u00e9".encode() * 3000)), (8, (16, None))], b""),
        # bytes after the batch (the rest of an mmap'd file) are not read
        ("trailing", [(1, (9, f64bits(2.5))), (2, (16, None))], b"\xff\x1c\x00junk"),
    ]
    return out


def archive_errors():
    """(name, wire, kind, offset): offset = the failing item's start (0: count / size guard)."""
    one = enc_varint(5) + enc_value((4, 42))
    return [
        ("count_short", b"", 4, 0),                                   # decode_varint on empty
        ("toobig", enc_varint(1000) + one, 2, 0),                     # check_sz: 24000 > 10<<8
        ("event_empty", enc_varint(1) + enc_varint(9), 4, 1),         # chunk()[0] panic -> Short
        ("fewer_items", enc_varint(3) + one + one, 4, 1 + 2 * len(one)),
        ("bad_tag", enc_varint(2) + one + enc_varint(6) + b"\x1c", 1, 1 + len(one)),
        ("bad_utf8", enc_varint(1) + enc_varint(6) + b"\x0c\x02\xc3\x28", 3, 1),
        ("id_varint_10", enc_varint(1) + b"\xff" * 10 + b"\x10", 3, 1),
        ("string_toobig", enc_varint(1) + enc_varint(6) + b"\x0c\x09ab", 2, 1),
    ]


def archive_edge_ok():
    """Accepted non-canonical inputs: an Id varint wider than u32 is truncated (Id(v as u32))."""
    w = enc_varint(1) + enc_varint(2**40 + 7) + enc_value((16, None))
    return [("id_truncated", w, [(7, 16, 0, 0)], len(w))]


def main():
    kat = kats()
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    manifest = {"batches": [], "errors": [], "edge_ok": [], "archive": [],
                "archive_errors": [], "archive_edge_ok": []}
    for name, msgs in batches():
        wire, cols = batch(msgs)
        fn = f"batch_{name}.bin"
        with open(os.path.join(HERE, fn), "wb") as f:
            f.write(wire)
        manifest["batches"].append({"name": name, "file": fn, "len": len(wire),
                                    "expect": cols_json(cols)})
    for name, wire, kind, off in errors():
        manifest["errors"].append({"name": name, "hex": wire.hex(), "kind": kind, "offset": off})
    for name, wire, rows in edge_ok():
        manifest["edge_ok"].append({"name": name, "hex": wire.hex(),
                                    "rows": [list(r) for r in rows]})
    for name, items, trailing in archive_batches():
        wire, cols, consumed = archive(items, trailing)
        fn = f"archive_{name}.bin"
        with open(os.path.join(HERE, fn), "wb") as f:
            f.write(wire)
        manifest["archive"].append({"name": name, "file": fn, "len": len(wire),
                                    "consumed": consumed, "expect": cols_json(cols)})
    for name, wire, kind, off in archive_errors():
        manifest["archive_errors"].append({"name": name, "hex": wire.hex(), "kind": kind,
                                           "offset": off})
    for name, wire, rows, consumed in archive_edge_ok():
        manifest["archive_edge_ok"].append({"name": name, "hex": wire.hex(), "consumed": consumed,
                                            "rows": [list(r) for r in rows]})
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(kat), "KATs,", len(manifest["batches"]), "batches,",
          len(manifest["errors"]), "error cases,", len(manifest["edge_ok"]), "edge cases,",
          len(manifest["archive"]), "archive batches,", len(manifest["archive_errors"]),
          "archive error cases")


if __name__ == "__main__":
    main()
