"""Publisher commit on the CPU: the C oracle (nxo_publish_commit) against a line-by-line Python
restatement of UpdateBatch::commit (netidx/src/publisher/mod.rs:776-845) with Value::eq
(netidx-value/src/op.rs:133-172) on the column representation. The restatement is the pin for the
oracle (the reference has no commit vectors); the oracle checks the GPU
(tests/test_gpu_publish.py)."""
import math
import random
import struct

import numpy as np
import pytest

import nxo

def value_eq(a, b, heap_a, heap_b):
    """Value::eq on (tag, fixed, aux) triples of the scalar and text tags (the values this file
    draws; containers, Decimal and Abstract: tests/test_publish_values_cpu.py)."""
    (ta, fa, aa), (tb, fb, ab) = a, b
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
    if ta in (12, 13, 18):
        return aa == ab and bytes(heap_a[fa:fa + aa]) == bytes(heap_b[fb:fb + ab])
    if ta in (14, 15, 16):
        return True
    return fa == fb


def commit(rows, kind, to_client, by_id, n_clients, heap, cur_heap):
    """rows: [(id, tag, fixed, aux)]; by_id: {id: [clients, current (tag, fixed, aux), from_batch]}.
    Returns ({client: [(id, row)]}, {id: row that became current})."""
    batch = {}
    current = {i: (v[1], False) for i, v in by_id.items()}
    became = {}
    for i, (idv, t, f, a) in enumerate(rows):
        v = (t, f, a)
        if kind[i] == nxo.PUB_UPDATE_CLIENT:
            if to_client[i] < n_clients:
                batch.setdefault(to_client[i], []).append((idv, i))
            continue
        pbl = by_id.get(idv)
        if pbl is None:
            continue
        if kind[i] == nxo.PUB_UPDATE_CHANGED:
            cur, in_batch = current[idv]
            if value_eq(cur, v, heap if in_batch else cur_heap, heap):
                continue
        for cl in pbl[0]:
            batch.setdefault(cl, []).append((idv, i))
        current[idv] = (v, True)
        became[idv] = i
    return batch, became


def random_values(rng, n, heap_words):
    """(tag, fixed, aux) values drawn to collide often: a few f64s incl. NaNs and +-0, small
    ints, bools, nulls, strings from a small pool (offsets into heap)."""
    f64 = [0.0, -0.0, 1.5, float("nan"), struct.unpack("<d", struct.pack("<Q", 0x7FF8000000000123))[0]]
    vals = []
    for _ in range(n):
        u = rng.randrange(7)
        if u == 0:
            vals.append((9, struct.unpack("<Q", struct.pack("<d", rng.choice(f64)))[0], 0))
        elif u == 1:
            vals.append((6, rng.randrange(3), 0))
        elif u == 2:
            vals.append((rng.choice([14, 15]), 0, 0))
        elif u == 3:
            vals.append((16, 0, 0))
        elif u == 4:
            off, ln = rng.choice(heap_words)
            vals.append((12, off, ln))
        elif u == 5:
            vals.append((10, rng.randrange(2), rng.randrange(2)))
        else:
            vals.append((8, struct.unpack("<I", struct.pack("<f", rng.choice([0.0, -0.0, 2.0])))[0], 0))
    return vals


def make_heap():
    words = [b"", b"a", b"ab", b"ab", b"xyz"]
    heap, idx = b"", []
    for w in words:
        idx.append((len(heap), len(w)))
        heap += w
    return np.frombuffer(heap + b"\0", np.uint8), idx


def random_case(rng, n_rows, n_ids, n_clients, p_pub=0.8):
    heap, words = make_heap()
    by_id, slot_ids = {}, []
    for i in range(n_ids):
        if rng.random() < p_pub:
            cls = rng.sample(range(n_clients), rng.randint(0, min(3, n_clients)))
            by_id[i] = [cls, random_values(rng, 1, words)[0]]
            slot_ids.append(i)
    vals = random_values(rng, n_rows, words)
    rows = [(rng.randrange(n_ids + 2), t, f, a) for (t, f, a) in vals]
    kind = [rng.choice([0, 1, 1, 2]) for _ in range(n_rows)]
    to_client = [rng.randrange(n_clients + 1) for _ in range(n_rows)]
    return rows, kind, to_client, by_id, slot_ids, heap


def arrays(rows, kind, to_client, by_id, slot_ids, n_ids):
    slot_of_id = np.full(n_ids, nxo.NO_SLOT, np.uint32)
    off, cl, ctag, cfix, caux = [0], [], [], [], []
    for s, i in enumerate(slot_ids):
        slot_of_id[i] = s
        cl.extend(by_id[i][0])
        off.append(len(cl))
        t, f, a = by_id[i][1]
        ctag.append(t)
        cfix.append(f)
        caux.append(a)
    ids = np.array([r[0] for r in rows], np.uint64)
    tag = np.array([r[1] for r in rows], np.uint8)
    fixed = np.array([r[2] for r in rows], np.uint64)
    aux = np.array([r[3] for r in rows], np.uint32)
    return (ids, tag, fixed, aux, np.array(kind, np.uint8), np.array(to_client, np.uint32),
            slot_of_id, np.array(off, np.uint32), np.array(cl, np.uint32),
            np.array(ctag, np.uint8), np.array(cfix, np.uint64), np.array(caux, np.uint32))


def run_oracle(rows, kind, to_client, by_id, slot_ids, n_ids, n_clients, heap):
    (ids, tag, fixed, aux, kd, to, soi, off, cl, ctag, cfix, caux) = arrays(
        rows, kind, to_client, by_id, slot_ids, n_ids)
    co, eid, erow, cur, um = nxo.publish_commit(ids, tag, fixed, aux, heap, kd, to, soi, off, cl,
                                                n_clients, ctag, cfix, caux, heap)
    got = {c: list(zip(eid[co[c]:co[c + 1]].tolist(), erow[co[c]:co[c + 1]].tolist()))
           for c in range(n_clients) if co[c + 1] > co[c]}
    became = {slot_ids[s]: int(cur[s]) - 1 for s in range(len(slot_ids)) if cur[s]}
    return got, became, um


@pytest.mark.parametrize("seed,n_rows,n_ids,n_clients", [
    (1, 0, 5, 2), (2, 1, 1, 1), (3, 300, 20, 4), (4, 2000, 50, 7), (5, 3000, 5, 3),
    (6, 1000, 400, 30),
])
def test_oracle_matches_commit(seed, n_rows, n_ids, n_clients):
    rng = random.Random(seed)
    rows, kind, to_client, by_id, slot_ids, heap = random_case(rng, n_rows, n_ids, n_clients)
    want, want_became = commit(rows, kind, to_client, by_id, n_clients, heap, heap)
    got, became, um = run_oracle(rows, kind, to_client, by_id, slot_ids, n_ids, n_clients, heap)
    assert got == want
    assert became == want_became
    assert um == sum(1 for r, k in zip(rows, kind) if k != nxo.PUB_UPDATE_CLIENT and r[0] not in by_id)


def test_oracle_container_vs_scalar_differs():
    """An Array current value (no children: empty) against an F64 row: different Typ, pushed.
    Container equality proper is covered by tests/test_publish_values_cpu.py."""
    by_id = {0: [[0], (19, 0, 0)]}  # current value is an empty Array
    rows = [(0, 9, 0, 0)]
    heap, _ = make_heap()
    got, became, _ = run_oracle(rows, [nxo.PUB_UPDATE_CHANGED], [0], by_id, [0], 1, 1, heap)
    assert got == {0: [(0, 0)]} and became == {0: 0}
