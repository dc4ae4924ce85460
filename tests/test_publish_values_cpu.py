"""UpdateChanged equality on every Value variant, CPU side: the oracle's commit
(nxo_publish_commit2) against a Python restatement of UpdateBatch::commit
(netidx/src/publisher/mod.rs:776-845) whose Value::eq (netidx-value/src/op.rs:133-172) works on
value trees, not columns:

  Decimal     numeric equality, as rust_decimal's PartialEq (via Ord): Fraction(m, 10^scale) with
              the sign; every zero equal whatever its sign and scale
  Array       same length, elements equal in order
  Map         entries equal in order (maps here are built as the reference's encoder writes them:
              keys sorted and unique, so two equal maps have the same entries in the same order)
  Error(v)    inner values equal; Error(String) is the same value whether its columns say tag 18
              or tag 22 over a String child
  Abstract    the same bytes (uuid + payload)

The trees are laid out in the columnar contract (include/nxg_codec.h: a container's elements are
consecutive child slots at fixed .. fixed + count, a Map's as key, value pairs) by `Layout`, so the
same case feeds the oracle and, in tests/test_gpu_publish.py, the GPU. Also the commit's
unsubscribes (publisher/mod.rs:820-832) against a dict-of-lists restatement. Parity unpinned:
the reference has no vectors for these comparisons."""
import math
import random
import struct
from fractions import Fraction

import numpy as np
import pytest

import nxo

DEPTH_LIMIT = 32  # NXG_MAX_DEPTH


class TooDeep(Exception):
    pass


# ---- value trees -------------------------------------------------------------------------------
# ("sc", tag, fixed, aux)   scalar (fixed-width tags)
# ("txt", tag, bytes)       String 12 / Bytes 13 / Error(String) 18 / Abstract 27
# ("dec", bytes16)          Decimal 20
# ("arr", [v...])           Array 19
# ("map", [(k, v)...])      Map 21
# ("err", v)                Error(Value) 22


def dec_value(b):
    flags, lo, mid, hi = struct.unpack("<IIII", bytes(b))
    m = lo | (mid << 32) | (hi << 64)
    scale = (flags >> 16) & 0xFF
    q = Fraction(m, 10 ** scale)
    return -q if flags >> 31 else q


def norm(v):
    if v[0] == "err" and v[1][0] == "txt" and v[1][1] == 12:
        return ("txt", 18, v[1][2])
    if v[0] == "sc" and v[1] == 17:
        return ("sc", 16, 0, 0)
    return v


def scalar_eq(a, b):
    (_, ta, fa, aa), (_, tb, fb, ab) = a, b
    if ta != tb:
        return False
    if ta == 8:
        l, r = (struct.unpack("<f", struct.pack("<I", x & 0xFFFFFFFF))[0] for x in (fa, fb))
        return (math.isnan(l) and math.isnan(r)) or l == r
    if ta == 9:
        l, r = (struct.unpack("<d", struct.pack("<Q", x))[0] for x in (fa, fb))
        return (math.isnan(l) and math.isnan(r)) or l == r
    if ta in (10, 11):
        return fa == fb and aa == ab
    if ta in (14, 15, 16):
        return True
    return fa == fb


def value_eq(a, b, depth=0):
    """Value::eq on trees. Raises TooDeep where the columnar comparison gives up (a slot at
    depth > 32), in the same depth-first order."""
    if depth > DEPTH_LIMIT:
        raise TooDeep()
    a, b = norm(a), norm(b)
    if a[0] != b[0]:
        return False
    k = a[0]
    if k == "sc":
        return scalar_eq(a, b)
    if k == "txt":
        return a[1] == b[1] and a[2] == b[2]
    if k == "dec":
        return dec_value(a[1]) == dec_value(b[1])
    if k == "arr":
        if len(a[1]) != len(b[1]):
            return False
        return all(value_eq(x, y, depth + 1) for x, y in zip(a[1], b[1]))
    if k == "map":
        if len(a[1]) != len(b[1]):
            return False
        for (ka, va), (kb, vb) in zip(a[1], b[1]):
            if not value_eq(ka, kb, depth + 1) or not value_eq(va, vb, depth + 1):
                return False
        return True
    return value_eq(a[1], b[1], depth + 1)  # err


class Layout:
    """Top-level values -> (tag, fixed, aux) columns, child columns and a heap."""

    def __init__(self):
        self.ctag, self.cfixed, self.caux = [], [], []
        self.heap = bytearray()

    def _text(self, b):
        off = len(self.heap)
        self.heap += b
        return off

    def _slot(self, v):
        k = v[0]
        if k == "sc":
            return v[1], v[2], v[3]
        if k == "txt":
            return v[1], self._text(v[2]), len(v[2])
        if k == "dec":
            return 20, self._text(v[1]), 16
        if k in ("arr", "map", "err"):
            elems = v[1] if k == "arr" else [x for kv in v[1] for x in kv] if k == "map" else [v[1]]
            base = len(self.ctag)
            self.ctag.extend([0] * len(elems))
            self.cfixed.extend([0] * len(elems))
            self.caux.extend([0] * len(elems))
            for i, e in enumerate(elems):
                t, f, a = self._slot(e)
                self.ctag[base + i], self.cfixed[base + i], self.caux[base + i] = t, f, a
            tag = {"arr": 19, "map": 21, "err": 22}[k]
            cnt = len(v[1]) if k != "err" else 1
            return tag, base, cnt
        raise ValueError(k)

    def top(self, vals):
        t, f, a = zip(*[self._slot(v) for v in vals]) if vals else ((), (), ())
        return (np.array(t, np.uint8), np.array(f, np.uint64), np.array(a, np.uint32))

    def children(self):
        return (np.array(self.ctag, np.uint8), np.array(self.cfixed, np.uint64),
                np.array(self.caux, np.uint32))

    def heap_array(self):
        return np.frombuffer(bytes(self.heap) + b"\0", np.uint8).copy()


# ---- random values that collide often ------------------------------------------------------------
def dec_bytes(m, scale, neg):
    return struct.pack("<IIII", (scale << 16) | (0x80000000 if neg else 0), m & 0xFFFFFFFF,
                       (m >> 32) & 0xFFFFFFFF, (m >> 64) & 0xFFFFFFFF)


DECIMALS = [
    dec_bytes(0, 0, False), dec_bytes(0, 5, True),          # zeros: all equal
    dec_bytes(15, 1, False), dec_bytes(150, 2, False),      # 1.5 twice
    dec_bytes(15, 1, True), dec_bytes(1500000, 6, True),    # -1.5 twice
    dec_bytes(3, 0, False), dec_bytes(3 * 10 ** 28, 28, False),  # 3 at scales 0 and 28
    dec_bytes(2 ** 96 - 1, 0, False), dec_bytes(2 ** 96 - 1, 28, False),
    dec_bytes(7, 40, False),                                # a scale byte past 28 (non-canonical)
]
ABSTRACT = [bytes(range(16)) + b"p", bytes(range(16)) + b"q", bytes(range(16)) + b"p",
            bytes(16)]
STRINGS = [b"", b"a", b"ab", b"xyz"]


def rand_scalar(rng):
    u = rng.randrange(6)
    if u == 0:
        f = rng.choice([0.0, -0.0, 1.5, float("nan")])
        return ("sc", 9, struct.unpack("<Q", struct.pack("<d", f))[0], 0)
    if u == 1:
        return ("sc", 6, rng.randrange(3), 0)
    if u == 2:
        return ("sc", rng.choice([14, 15, 16, 17]), 0, 0)
    if u == 3:
        return ("txt", 12, rng.choice(STRINGS))
    if u == 4:
        return ("dec", rng.choice(DECIMALS))
    return ("txt", 27, rng.choice(ABSTRACT))


def rand_value(rng, depth=0):
    u = rng.randrange(10 if depth < 3 else 4)
    if u < 4:
        return rand_scalar(rng)
    if u < 6:
        return ("arr", [rand_value(rng, depth + 1) for _ in range(rng.randrange(3))])
    if u < 8:
        keys = sorted(set(rng.randrange(3) for _ in range(rng.randrange(3))))
        return ("map", [(("sc", 6, k, 0), rand_value(rng, depth + 1)) for k in keys])
    if u == 8:
        return ("err", ("txt", 12, rng.choice(STRINGS)))  # Error(String) as tag 22 + child
    return ("err", rand_value(rng, depth + 1))


def nested(depth, leaf=("sc", 6, 1, 0)):
    v = leaf
    for _ in range(depth):
        v = ("arr", [v])
    return v


# ---- the restatement of the commit ------------------------------------------------------------
def commit(rows, kind, to_client, by_id, n_clients):
    """rows: [(id, value)]; by_id: {id: [clients, current value]}. Returns ({client: [(id, row)]},
    {id: row that became current}); raises TooDeep."""
    batch, became = {}, {}
    current = {i: v[1] for i, v in by_id.items()}
    for i, (idv, v) in enumerate(rows):
        if kind[i] == nxo.PUB_UPDATE_CLIENT:
            if to_client[i] < n_clients:
                batch.setdefault(to_client[i], []).append((idv, i))
            continue
        pbl = by_id.get(idv)
        if pbl is None:
            continue
        if kind[i] == nxo.PUB_UPDATE_CHANGED and value_eq(current[idv], v):
            continue
        for cl in pbl[0]:
            batch.setdefault(cl, []).append((idv, i))
        current[idv] = v
        became[idv] = i
    return batch, became


def random_case(rng, n_rows, n_ids, n_clients):
    by_id, slot_ids = {}, []
    for i in range(n_ids):
        if rng.random() < 0.85:
            by_id[i] = [rng.sample(range(n_clients), rng.randint(0, min(3, n_clients))),
                        rand_value(rng)]
            slot_ids.append(i)
    rows = [(rng.randrange(n_ids + 1), rand_value(rng)) for _ in range(n_rows)]
    kind = [rng.choice([0, 1, 1, 1, 2]) for _ in range(n_rows)]
    to_client = [rng.randrange(n_clients + 1) for _ in range(n_rows)]
    return rows, kind, to_client, by_id, slot_ids


def case_arrays(rows, kind, to_client, by_id, slot_ids, n_ids):
    """The case in columns: batch (ids, tag, fixed, aux, children, heap), table (slot_of_id,
    client CSR, current values with their children and heap)."""
    bl, cl_ = Layout(), Layout()
    tag, fixed, aux = bl.top([v for _, v in rows])
    slot_of_id = np.full(n_ids, nxo.NO_SLOT, np.uint32)
    off, cl = [0], []
    for s, i in enumerate(slot_ids):
        slot_of_id[i] = s
        cl.extend(by_id[i][0])
        off.append(len(cl))
    ctag, cfix, caux = cl_.top([by_id[i][1] for i in slot_ids])
    return dict(ids=np.array([r[0] for r in rows], np.uint64), tag=tag, fixed=fixed, aux=aux,
                children=bl.children(), heap=bl.heap_array(), kind=np.array(kind, np.uint8),
                to=np.array(to_client, np.uint32), soi=slot_of_id, off=np.array(off, np.uint32),
                cl=np.array(cl, np.uint32), cur_tag=ctag, cur_fixed=cfix, cur_aux=caux,
                cur_children=cl_.children(), cur_heap=cl_.heap_array())


def run_oracle(a, n_clients):
    co, eid, erow, cur, um = nxo.publish_commit(
        a["ids"], a["tag"], a["fixed"], a["aux"], a["heap"], a["kind"], a["to"], a["soi"],
        a["off"], a["cl"], n_clients, a["cur_tag"], a["cur_fixed"], a["cur_aux"], a["cur_heap"],
        children=a["children"], cur_children=a["cur_children"])
    return co, eid, erow, cur, um


def as_dicts(co, eid, erow, cur, slot_ids, n_clients):
    got = {c: list(zip(eid[co[c]:co[c + 1]].tolist(), erow[co[c]:co[c + 1]].tolist()))
           for c in range(n_clients) if co[c + 1] > co[c]}
    became = {slot_ids[s]: int(cur[s]) - 1 for s in range(len(slot_ids)) if cur[s]}
    return got, became


# ---- tests -----------------------------------------------------------------------------------
def test_decimal_eq_known_answers():
    eq = nxo.decimal_eq
    assert eq(dec_bytes(0, 0, False), dec_bytes(0, 28, True))
    assert eq(dec_bytes(15, 1, False), dec_bytes(150, 2, False))
    assert not eq(dec_bytes(15, 1, False), dec_bytes(15, 1, True))
    assert not eq(dec_bytes(15, 1, False), dec_bytes(151, 2, False))
    assert eq(dec_bytes(3, 0, False), dec_bytes(3 * 10 ** 28, 28, False))
    assert not eq(dec_bytes(2 ** 96 - 1, 0, False), dec_bytes(2 ** 96 - 1, 28, False))
    assert not eq(dec_bytes(1, 0, False), dec_bytes(1, 29, False))
    assert eq(dec_bytes(7, 40, False), dec_bytes(7, 40, False))
    rng = random.Random(5)
    for _ in range(3000):
        a = dec_bytes(rng.choice([0, 1, 10, 100, rng.randrange(2 ** 96)]), rng.randrange(30),
                      rng.random() < 0.5)
        b = dec_bytes(rng.choice([0, 1, 10, 100, rng.randrange(2 ** 96)]), rng.randrange(30),
                      rng.random() < 0.5)
        assert eq(a, b) == (dec_value(a) == dec_value(b))
        assert eq(a, a)


@pytest.mark.parametrize("seed,n_rows,n_ids,n_clients", [
    (41, 0, 3, 2), (42, 1, 1, 1), (43, 400, 10, 3), (44, 3000, 40, 6), (45, 3000, 3, 4),
])
def test_oracle_container_equality_matches_commit(seed, n_rows, n_ids, n_clients):
    rng = random.Random(seed)
    rows, kind, to_client, by_id, slot_ids = random_case(rng, n_rows, n_ids, n_clients)
    want, want_became = commit(rows, kind, to_client, by_id, n_clients)
    a = case_arrays(rows, kind, to_client, by_id, slot_ids, n_ids)
    co, eid, erow, cur, um = run_oracle(a, n_clients)
    got, became = as_dicts(co, eid, erow, cur, slot_ids, n_clients)
    assert got == want and became == want_became
    # the comparisons really happened: some UpdateChanged rows were dropped as equal
    if n_rows > 100:
        pushed = {r for v in want.values() for _, r in v}
        dropped = [i for i, k in enumerate(kind)
                   if k == 1 and rows[i][0] in by_id and i not in pushed]
        assert dropped


def test_oracle_depth_limit():
    for d, ok in ((DEPTH_LIMIT, True), (DEPTH_LIMIT + 1, False)):
        by_id = {0: [[0], nested(d)]}
        rows = [(0, nested(d))]
        a = case_arrays(rows, [nxo.PUB_UPDATE_CHANGED], [0], by_id, [0], 1)
        if ok:
            co, eid, erow, cur, um = run_oracle(a, 1)
            assert len(eid) == 0  # equal: not pushed
            # a difference found before the limit is a plain difference
            a = case_arrays([(0, nested(d + 5))], [nxo.PUB_UPDATE_CHANGED], [0], by_id, [0], 1)
            assert len(run_oracle(a, 1)[1]) == 1
        else:
            with pytest.raises(ValueError) as e:
                run_oracle(a, 1)
            assert e.value.args[0] == nxo.UNSUPPORTED
            with pytest.raises(TooDeep):
                commit(rows, [nxo.PUB_UPDATE_CHANGED], [0], by_id, 1)


def test_oracle_containers_without_child_columns_refused():
    by_id = {0: [[0], ("arr", [("sc", 6, 1, 0)])]}
    a = case_arrays([(0, ("arr", [("sc", 6, 1, 0)]))], [nxo.PUB_UPDATE_CHANGED], [0], by_id, [0], 1)
    with pytest.raises(ValueError):
        nxo.publish_commit(a["ids"], a["tag"], a["fixed"], a["aux"], a["heap"], a["kind"], a["to"],
                           a["soi"], a["off"], a["cl"], 1, a["cur_tag"], a["cur_fixed"],
                           a["cur_aux"], a["cur_heap"])
    # a scalar never needs them
    a = case_arrays([(0, ("sc", 6, 1, 0))], [nxo.PUB_UPDATE_CHANGED], [0], by_id, [0], 1)
    assert len(run_oracle(a, 1)[1]) == 1


def unsubscribes(ids, clients, n_clients):
    out = {}
    for i, c in zip(ids, clients):
        if c < n_clients:
            out.setdefault(c, []).append(i)
    return out


@pytest.mark.parametrize("seed,n,n_clients", [(51, 0, 3), (52, 1, 1), (53, 5000, 7),
                                               (54, 20000, 1500)])
def test_oracle_unsubscribes(seed, n, n_clients):
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, 1000, n, dtype=np.uint64)
    cl = rng.integers(0, n_clients + 2, n, dtype=np.uint32)
    off, ent = nxo.publish_unsubscribes(ids, cl, n_clients)
    got = {c: ent[off[c]:off[c + 1]].tolist() for c in range(n_clients) if off[c + 1] > off[c]}
    assert got == unsubscribes(ids.tolist(), cl.tolist(), n_clients)
