"""ctypes binding of the CPU oracle (oracle/build/libnx_oracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module. It is
the checker, never the thing measured or shipped.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "libnx_oracle.so")

U64P = C.POINTER(C.c_uint64)
U32P = C.POINTER(C.c_uint32)
U8P = C.POINTER(C.c_uint8)


class NxoCols(C.Structure):
    _fields_ = [
        ("cap_rows", C.c_uint64), ("cap_children", C.c_uint64), ("cap_ctl", C.c_uint64),
        ("n_rows", C.c_uint64), ("n_children", C.c_uint64), ("n_ctl", C.c_uint64),
        ("n_heartbeat", C.c_uint64),
        ("id", U64P), ("tag", U8P), ("fixed", U64P), ("aux", U32P),
        ("ctag", U8P), ("cfixed", U64P), ("caux", U32P),
        ("ctl_row", U64P), ("ctl_off", U64P), ("ctl_len", U32P), ("ctl_variant", U8P),
        ("err_kind", C.c_int32), ("err_offset", C.c_uint64),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built: {LIB_PATH} (run make -C oracle)")
        L = C.CDLL(LIB_PATH)
        L.nxo_varint_len.restype = C.c_uint32
        L.nxo_varint_len.argtypes = [C.c_uint64]
        L.nxo_encode_varint.restype = C.c_uint32
        L.nxo_encode_varint.argtypes = [C.c_uint64, U8P]
        L.nxo_decode_varint.restype = C.c_int
        L.nxo_decode_varint.argtypes = [U8P, C.c_uint64, U64P, U32P]
        L.nxo_varint_sweep.restype = C.c_uint64
        L.nxo_varint_sweep.argtypes = [C.c_uint64, C.c_uint64, C.c_int]
        L.nxo_decode_frame.restype = C.c_int
        L.nxo_decode_frame.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(NxoCols)]
        L.nxo_encoded_len.restype = C.c_int64
        L.nxo_encoded_len.argtypes = [C.POINTER(NxoCols), C.c_void_p]
        L.nxo_encode.restype = C.c_int64
        L.nxo_encode.argtypes = [C.POINTER(NxoCols), C.c_void_p, C.c_void_p, C.c_uint64]
        L.nxo_encode_f64.restype = C.c_int64
        L.nxo_encode_f64.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64]
        L.nxo_datetime_valid.restype = C.c_int
        L.nxo_datetime_valid.argtypes = [C.c_int64, C.c_uint32]
        L.nxo_utf8_valid.restype = C.c_int
        L.nxo_utf8_valid.argtypes = [C.c_void_p, C.c_uint64]
        L.nxo_publish_commit.restype = C.c_int64
        L.nxo_publish_commit.argtypes = [C.c_void_p] * 7 + [C.c_uint64, C.c_uint64, C.c_void_p,
                                                            C.c_uint64, C.c_void_p, C.c_void_p,
                                                            C.c_uint32] + [C.c_void_p] * 7 + \
            [C.c_uint64, C.c_void_p, C.c_void_p]
        L.nxo_publish_commit2.restype = C.c_int64
        L.nxo_publish_commit2.argtypes = [C.c_void_p] * 10 + [C.c_uint64, C.c_uint64, C.c_void_p,
                                                              C.c_uint64, C.c_void_p, C.c_void_p,
                                                              C.c_uint32] + [C.c_void_p] * 10 + \
            [C.c_uint64, C.c_void_p, C.c_void_p]
        L.nxo_decimal_eq.restype = C.c_int
        L.nxo_decimal_eq.argtypes = [C.c_void_p, C.c_void_p]
        L.nxo_publish_unsubscribes.restype = C.c_int64
        L.nxo_publish_unsubscribes.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32,
                                               C.c_void_p, C.c_void_p]
        L.nxo_decode_archive.restype = C.c_int64
        L.nxo_decode_archive.argtypes = [C.c_void_p, C.c_uint64, C.POINTER(NxoCols)]
        L.nxo_encode_archive.restype = C.c_int64
        L.nxo_encode_archive.argtypes = [C.POINTER(NxoCols), C.c_void_p, C.c_void_p, C.c_uint64]
        L.nxo_dispatch.restype = C.c_int64
        L.nxo_dispatch.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p, C.c_uint64,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                   C.c_void_p]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


class Decoded:
    """Numpy view of an oracle decode (same columnar contract as include/nxg_codec.h)."""

    def __init__(self, cap_rows, cap_children, cap_ctl):
        self.id = np.zeros(cap_rows, np.uint64)
        self.tag = np.zeros(cap_rows, np.uint8)
        self.fixed = np.zeros(cap_rows, np.uint64)
        self.aux = np.zeros(cap_rows, np.uint32)
        self.ctag = np.zeros(cap_children, np.uint8)
        self.cfixed = np.zeros(cap_children, np.uint64)
        self.caux = np.zeros(cap_children, np.uint32)
        self.ctl_row = np.zeros(cap_ctl, np.uint64)
        self.ctl_off = np.zeros(cap_ctl, np.uint64)
        self.ctl_len = np.zeros(cap_ctl, np.uint32)
        self.ctl_variant = np.zeros(cap_ctl, np.uint8)
        self.s = NxoCols(cap_rows, cap_children, cap_ctl, 0, 0, 0, 0,
                         _p(self.id, U64P), _p(self.tag, U8P), _p(self.fixed, U64P),
                         _p(self.aux, U32P), _p(self.ctag, U8P), _p(self.cfixed, U64P),
                         _p(self.caux, U32P), _p(self.ctl_row, U64P), _p(self.ctl_off, U64P),
                         _p(self.ctl_len, U32P), _p(self.ctl_variant, U8P), 0, 0)

    def trim(self):
        s = self.s
        n, c, k = s.n_rows, s.n_children, s.n_ctl
        return {
            "id": self.id[:n], "tag": self.tag[:n], "fixed": self.fixed[:n], "aux": self.aux[:n],
            "ctag": self.ctag[:c], "cfixed": self.cfixed[:c], "caux": self.caux[:c],
            "ctl_row": self.ctl_row[:k], "ctl_off": self.ctl_off[:k],
            "ctl_len": self.ctl_len[:k], "ctl_variant": self.ctl_variant[:k],
            "n_heartbeat": s.n_heartbeat, "err_kind": s.err_kind, "err_offset": s.err_offset,
        }


def decode(wire, cap_rows=None, cap_children=None, cap_ctl=None):
    wire = np.frombuffer(bytes(wire), np.uint8) if not isinstance(wire, np.ndarray) else wire
    n = len(wire)
    d = Decoded(cap_rows if cap_rows is not None else n // 4 + 1,
                cap_children if cap_children is not None else n + 1,
                cap_ctl if cap_ctl is not None else n // 2 + 1)
    lib().nxo_decode_frame(wire.ctypes.data, n, C.byref(d.s))
    d.wire = wire
    return d


def encode(d, heap):
    heap = np.frombuffer(bytes(heap), np.uint8) if not isinstance(heap, np.ndarray) else heap
    n = lib().nxo_encoded_len(C.byref(d.s), heap.ctypes.data)
    if n < 0:
        raise ValueError(f"encode error {-n}")
    out = np.zeros(max(n, 1), np.uint8)
    m = lib().nxo_encode(C.byref(d.s), heap.ctypes.data, out.ctypes.data, n)
    assert m == n, (m, n)
    return out[:n].tobytes()


TAG_UNSUBSCRIBED = 0x40


def decode_archive(buf, cap_rows=None, cap_children=None):
    """nxo_decode_archive (an archive batch, Vec<BatchItem>). Returns (Decoded, consumed or
    -kind)."""
    buf = np.frombuffer(bytes(buf), np.uint8) if not isinstance(buf, np.ndarray) else buf
    n = len(buf)
    d = Decoded(cap_rows if cap_rows is not None else n // 2 + 1,
                cap_children if cap_children is not None else n + 1, 1)
    r = lib().nxo_decode_archive(buf.ctypes.data if n else None, n, C.byref(d.s))
    d.wire = buf
    return d, int(r)


def encode_archive(d, heap):
    """nxo_encode_archive of the rows of `d` (Decoded-shaped columns) with text at `heap`."""
    heap = np.frombuffer(bytes(heap), np.uint8) if not isinstance(heap, np.ndarray) else heap
    hp = heap.ctypes.data if len(heap) else None
    n = lib().nxo_encode_archive(C.byref(d.s), hp, None, 0)
    if n < 0:
        raise ValueError(f"encode error {-n}")
    out = np.zeros(max(n, 1), np.uint8)
    m = lib().nxo_encode_archive(C.byref(d.s), hp, out.ctypes.data, n)
    assert m == n, (m, n)
    return out[:n].tobytes()


def encode_f64(ids, vals):
    ids = np.ascontiguousarray(ids, np.uint64)
    vals = np.ascontiguousarray(vals, np.uint64)
    cap = 21 * len(ids) + 16
    out = np.zeros(cap, np.uint8)
    n = lib().nxo_encode_f64(ids.ctypes.data, vals.ctypes.data, len(ids), out.ctypes.data, cap)
    if n < 0:
        raise ValueError(f"encode error {-n}")
    return out[:n]


NO_SLOT = 0xFFFFFFFF


def dispatch(ids, slot_of_id, slot_sub_id, slot_stream_off, stream_chan, slot_has_last, n_chans):
    """nxo_dispatch (process_updates_batch, connection.rs:546-567) on numpy arrays.
    Returns (chan_off, ent_sub, ent_row, last_row, n_unmatched)."""
    ids = np.ascontiguousarray(ids, np.uint64)
    slot_of_id = np.ascontiguousarray(slot_of_id, np.uint32)
    slot_sub_id = np.ascontiguousarray(slot_sub_id, np.uint64)
    slot_stream_off = np.ascontiguousarray(slot_stream_off, np.uint32)
    stream_chan = np.ascontiguousarray(stream_chan, np.uint32)
    slot_has_last = np.ascontiguousarray(slot_has_last, np.uint8)
    fan = int((slot_stream_off[1:].astype(np.int64) - slot_stream_off[:-1]).max()) if len(slot_sub_id) else 0
    cap = max(len(ids) * fan, 1)
    chan_off = np.zeros(n_chans + 1, np.uint64)
    ent_sub = np.zeros(cap, np.uint64)
    ent_row = np.zeros(cap, np.uint64)
    last_row = np.zeros(max(len(slot_sub_id), 1), np.uint64)
    um = np.zeros(1, np.uint64)
    n = lib().nxo_dispatch(ids.ctypes.data, len(ids), len(slot_of_id), slot_of_id.ctypes.data,
                           len(slot_sub_id), slot_sub_id.ctypes.data, slot_stream_off.ctypes.data,
                           stream_chan.ctypes.data, slot_has_last.ctypes.data, n_chans,
                           chan_off.ctypes.data, ent_sub.ctypes.data, ent_row.ctypes.data, cap,
                           last_row.ctypes.data, um.ctypes.data)
    if n < 0:
        raise ValueError(f"dispatch error {-n}")
    return chan_off, ent_sub[:n], ent_row[:n], last_row[: len(slot_sub_id)], int(um[0])


PUB_UPDATE, PUB_UPDATE_CHANGED, PUB_UPDATE_CLIENT = 0, 1, 2
UNSUPPORTED = 10


def publish_commit(id, tag, fixed, aux, heap, kind, to_client, slot_of_id, slot_client_off,
                   client, n_clients, cur_tag, cur_fixed, cur_aux, cur_heap, children=None,
                   cur_children=None):
    """nxo_publish_commit2 (UpdateBatch::commit, publisher/mod.rs:776-845) on numpy arrays.
    children / cur_children: (ctag, cfixed, caux) of the batch's / the current values'
    Array/Map/Error(Value) elements, or None. Returns (client_off, ent_id, ent_row, cur_row,
    n_unmatched), or raises ValueError(code)."""
    a = {}
    ch = children if children is not None else ([], [], [])
    cch = cur_children if cur_children is not None else ([], [], [])
    for k, v, dt in [("id", id, np.uint64), ("tag", tag, np.uint8), ("fixed", fixed, np.uint64),
                     ("aux", aux, np.uint32), ("heap", heap, np.uint8), ("kind", kind, np.uint8),
                     ("to", to_client, np.uint32), ("soi", slot_of_id, np.uint32),
                     ("off", slot_client_off, np.uint32), ("cl", client, np.uint32),
                     ("ctag", cur_tag, np.uint8), ("cfix", cur_fixed, np.uint64),
                     ("caux", cur_aux, np.uint32), ("cheap", cur_heap, np.uint8),
                     ("bct", ch[0], np.uint8), ("bcf", ch[1], np.uint64), ("bca", ch[2], np.uint32),
                     ("cct", cch[0], np.uint8), ("ccf", cch[1], np.uint64),
                     ("cca", cch[2], np.uint32)]:
        a[k] = np.ascontiguousarray(v if len(v) else np.zeros(1), dt)
    n = len(id)
    n_slots = len(slot_client_off) - 1
    fan = int((a["off"][1:].astype(np.int64) - a["off"][:-1]).max()) if n_slots > 0 else 0
    cap = max(n * max(fan, 1), 1)
    client_off = np.zeros(n_clients + 1, np.uint64)
    ent_id = np.zeros(cap, np.uint64)
    ent_row = np.zeros(cap, np.uint64)
    cur_row = np.zeros(max(n_slots, 1), np.uint64)
    um = np.zeros(1, np.uint64)
    d = lambda k: a[k].ctypes.data
    dc = lambda k, have: a[k].ctypes.data if have else None
    hb, hc = children is not None, cur_children is not None
    r = lib().nxo_publish_commit2(d("id"), d("tag"), d("fixed"), d("aux"), dc("bct", hb),
                                  dc("bcf", hb), dc("bca", hb), d("heap"), d("kind"), d("to"), n,
                                  len(slot_of_id), d("soi"), n_slots, d("off"), d("cl"),
                                  n_clients, d("ctag"), d("cfix"), d("caux"), dc("cct", hc),
                                  dc("ccf", hc), dc("cca", hc), d("cheap"),
                                  client_off.ctypes.data, ent_id.ctypes.data, ent_row.ctypes.data,
                                  cap, cur_row.ctypes.data, um.ctypes.data)
    if r < 0:
        raise ValueError(-r)
    return client_off, ent_id[:r], ent_row[:r], cur_row[:n_slots], int(um[0])


def decimal_eq(a, b):
    """nxo_decimal_eq on two 16-byte rust_decimal encodings."""
    a = np.frombuffer(bytes(a), np.uint8).copy()
    b = np.frombuffer(bytes(b), np.uint8).copy()
    assert len(a) == len(b) == 16
    return bool(lib().nxo_decimal_eq(a.ctypes.data, b.ctypes.data))


def publish_unsubscribes(ids, clients, n_clients):
    """nxo_publish_unsubscribes: returns (client_off, ent_id)."""
    ids = np.ascontiguousarray(ids, np.uint64)
    cl = np.ascontiguousarray(clients, np.uint32)
    off = np.zeros(n_clients + 1, np.uint64)
    ent = np.zeros(max(len(ids), 1), np.uint64)
    r = lib().nxo_publish_unsubscribes(ids.ctypes.data if len(ids) else None,
                                       cl.ctypes.data if len(cl) else None, len(ids), n_clients,
                                       off.ctypes.data, ent.ctypes.data)
    if r < 0:
        raise ValueError(-r)
    return off, ent[:r]


CONTAINER_TAGS = (19, 21, 22)  # Array, Map, Error(Value): `fixed` is the first child slot


def share(o, k, shares):
    """Row share k of `shares` of a trimmed decode `o` (the contract of nxg_decode_share,
    include/nxg_codec.h), restated on numpy: rows [N*k/shares, N*(k+1)/shares), the child slots
    of their subtrees (children are allocated depth-first in row order), the control spans with
    ctl_row in the share (the last share: also those after the last row); child indices and
    ctl_row re-based. Returns (first row, dict of columns + n_heartbeat)."""
    N = len(o["id"])
    r0, r1 = N * k // shares, N * (k + 1) // shares
    tag, fixed = o["tag"], o["fixed"]
    cont = np.isin(tag, CONTAINER_TAGS)
    nch = len(o["ctag"])

    def first_child(r):
        idx = np.flatnonzero(cont[r:])
        return int(fixed[r + idx[0]]) if len(idx) else nch

    c0, c1 = first_child(r0), first_child(r1)
    ctl_row = o["ctl_row"]
    k0 = int(np.searchsorted(ctl_row, r0, "left"))
    k1 = len(ctl_row) if k == shares - 1 else int(np.searchsorted(ctl_row, r1, "left"))
    ct = o["ctag"][c0:c1]
    out = {
        "id": o["id"][r0:r1], "tag": tag[r0:r1],
        "fixed": np.where(cont[r0:r1], fixed[r0:r1] - np.uint64(c0), fixed[r0:r1]),
        "aux": o["aux"][r0:r1], "ctag": ct,
        "cfixed": np.where(np.isin(ct, CONTAINER_TAGS), o["cfixed"][c0:c1] - np.uint64(c0),
                           o["cfixed"][c0:c1]),
        "caux": o["caux"][c0:c1], "ctl_row": ctl_row[k0:k1] - np.uint64(r0),
        "ctl_off": o["ctl_off"][k0:k1], "ctl_len": o["ctl_len"][k0:k1],
        "ctl_variant": o["ctl_variant"][k0:k1],
    }
    out["n_heartbeat"] = int((out["ctl_variant"] == 5).sum())
    return r0, out


def partition_by_tag(tag, fixed, aux, bins=256):
    """Checker for nxg_partition_by_tag (the type-partitioned view): the rows grouped
    by tag with a stable sort (record order within a tag), as numpy restates it -- integer
    bookkeeping only, no codec rule involved. Returns {count, off, row_of, fixed, aux, rank}."""
    tag = np.asarray(tag, np.uint8)
    n = len(tag)
    row_of = np.argsort(tag, kind="stable").astype(np.uint32)
    count = np.bincount(tag, minlength=bins).astype(np.uint64)
    off = np.zeros(bins + 1, np.uint64)
    off[1:] = np.cumsum(count)
    rank = np.empty(n, np.uint32)
    rank[row_of] = (np.arange(n, dtype=np.uint64) - off[tag[row_of]]).astype(np.uint32)
    return {"count": count, "off": off, "row_of": row_of, "fixed": np.asarray(fixed)[row_of],
            "aux": np.asarray(aux)[row_of], "rank": rank}
