"""GPU parity of the publisher commit (nxg_publish_commit, include/nxg_codec.h) against the CPU
oracle (nxo_publish_commit, a restatement of UpdateBatch::commit, publisher/mod.rs:776-845):
identical per-client batches (Id, row) in identical order, identical new `current` rows and
unmatched counts, and NXG_UNSUPPORTED exactly where the oracle refuses. Bit-exact."""
import random

import numpy as np
import pytest

import nxo
from test_publish_cpu import arrays, make_heap, random_case

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import torch
    import netidx_amd
    assert torch.cuda.is_available()
    c = netidx_amd.Codec(0)
    yield c
    c.close()


def gpu_commit(codec, a, heap, n_clients):
    import torch
    import netidx_amd
    (ids, tag, fixed, aux, kd, to, soi, off, cl, ctag, cfix, caux) = a
    batch = netidx_amd.columns_from_arrays(ids, fixed, tag, aux)
    tab = netidx_amd.PubTable(soi, off, cl, n_clients, ctag, cfix, caux, heap)
    dheap = torch.from_numpy(heap.copy()).cuda()
    kind = torch.from_numpy(kd.copy()).cuda()
    to_client = torch.from_numpy(to.view(np.int32).copy()).cuda()
    return codec.publish_commit(tab, batch, kind, to_client, heap=dheap)


def check(codec, rows, kind, to_client, by_id, slot_ids, n_ids, n_clients, heap):
    a = arrays(rows, kind, to_client, by_id, slot_ids, n_ids)
    (ids, tag, fixed, aux, kd, to, soi, off, cl, ctag, cfix, caux) = a
    w = nxo.publish_commit(ids, tag, fixed, aux, heap, kd, to, soi, off, cl, n_clients, ctag,
                           cfix, caux, heap)
    d = gpu_commit(codec, a, heap, n_clients)
    assert np.array_equal(d.chan_off.cpu().numpy().view(np.uint64), w[0])
    assert d.n_entries == len(w[1])
    assert np.array_equal(d.ent_sub[: d.n_entries].cpu().numpy().view(np.uint64), w[1])
    assert np.array_equal(d.ent_row[: d.n_entries].cpu().numpy().view(np.uint64), w[2])
    assert np.array_equal(d.last_row.cpu().numpy().view(np.uint64), w[3])
    assert d.n_unmatched == w[4]


@pytest.mark.parametrize("seed,n_rows,n_ids,n_clients", [
    (21, 0, 5, 2),
    (22, 1, 1, 1),
    (23, 300, 20, 4),        # many repeats per Id: prev() by the radix sort
    (24, 5000, 50, 7),
    (25, 20000, 5, 3),       # every Id repeated thousands of times
    (26, 3000, 4000, 30),    # mostly distinct Ids
    (27, 100000, 70000, 1025),  # more clients than the LDS counters
])
def test_publish_matches_oracle(codec, seed, n_rows, n_ids, n_clients):
    rng = random.Random(seed)
    rows, kind, to_client, by_id, slot_ids, heap = random_case(rng, n_rows, n_ids, n_clients)
    check(codec, rows, kind, to_client, by_id, slot_ids, n_ids, n_clients, heap)


def test_publish_distinct_ids_no_sort(codec):
    """Each Id once (the common batch): prev() is the table's current, no radix sort."""
    rng = random.Random(31)
    heap, words = make_heap()
    n = 50000
    by_id = {i: [[i % 5], (9, rng.choice([0, 1 << 63, 0x7FF8000000000000]), 0)] for i in range(n)}
    rows = [(i, 9, rng.choice([0, 1 << 63, 0x7FF8000000000001, 4607182418800017408]), 0)
            for i in rng.sample(range(n), n)]
    kind = [1] * n
    check(codec, rows, kind, [0] * n, by_id, list(range(n)), n, 5, heap)


def test_publish_only_updates_and_directed(codec):
    rng = random.Random(32)
    rows, kind, to_client, by_id, slot_ids, heap = random_case(rng, 5000, 300, 6)
    kind = [0 if k == 1 else k for k in kind]  # no UpdateChanged: the kinds route as they are
    check(codec, rows, kind, to_client, by_id, slot_ids, 300, 6, heap)


def test_publish_container_vs_scalar(codec):
    """A Map current value (empty) against an F64 row: different Typ, pushed, as the oracle."""
    heap, _ = make_heap()
    by_id = {0: [[0], (21, 0, 0)]}
    check(codec, [(0, 9, 0, 0)], [nxo.PUB_UPDATE_CHANGED], [0], by_id, [0], 1, 1, heap)


def test_publish_deep_value_unsupported(codec):
    """Values nested past NXG_MAX_DEPTH: NXG_UNSUPPORTED where the oracle refuses."""
    import netidx_amd
    from test_publish_values_cpu import case_arrays, nested, DEPTH_LIMIT
    by_id = {0: [[0], nested(DEPTH_LIMIT + 1)]}
    a = case_arrays([(0, nested(DEPTH_LIMIT + 1))], [nxo.PUB_UPDATE_CHANGED], [0], by_id, [0], 1)
    with pytest.raises(netidx_amd.CodecError, match="UNSUPPORTED"):
        gpu_commit_values(codec, a, 1)


def gpu_commit_values(codec, a, n_clients):
    import torch
    import netidx_amd
    ct, cf, ca = a["children"]
    batch = netidx_amd.columns_from_arrays(a["ids"], a["fixed"], a["tag"], a["aux"], ct, cf, ca)
    qt, qf, qa = a["cur_children"]
    tab = netidx_amd.PubTable(a["soi"], a["off"], a["cl"], n_clients, a["cur_tag"],
                              a["cur_fixed"], a["cur_aux"], a["cur_heap"], cur_ctag=qt,
                              cur_cfixed=qf, cur_caux=qa)
    dheap = torch.from_numpy(a["heap"].copy()).cuda()
    kind = torch.from_numpy(a["kind"].copy()).cuda()
    to_client = torch.from_numpy(a["to"].view(np.int32).copy()).cuda()
    return codec.publish_commit(tab, batch, kind, to_client, heap=dheap)


@pytest.mark.parametrize("seed,n_rows,n_ids,n_clients", [
    (61, 1, 1, 1),
    (62, 2000, 30, 5),      # repeats: prev() rows compared with each other
    (63, 20000, 4000, 40),  # mostly against the table's current values
])
def test_publish_container_decimal_abstract_equality(codec, seed, n_rows, n_ids, n_clients):
    """UpdateChanged over Arrays, Maps, Error(Value), Decimal (numeric) and Abstract values,
    nested up to 3 deep, batch rows against batch rows and against the table: identical to the
    oracle."""
    from test_publish_values_cpu import case_arrays, random_case, run_oracle
    rng = random.Random(seed)
    rows, kind, to_client, by_id, slot_ids = random_case(rng, n_rows, n_ids, n_clients)
    a = case_arrays(rows, kind, to_client, by_id, slot_ids, n_ids)
    w = run_oracle(a, n_clients)
    d = gpu_commit_values(codec, a, n_clients)
    assert np.array_equal(d.chan_off.cpu().numpy().view(np.uint64), w[0])
    assert d.n_entries == len(w[1])
    assert np.array_equal(d.ent_sub[: d.n_entries].cpu().numpy().view(np.uint64), w[1])
    assert np.array_equal(d.ent_row[: d.n_entries].cpu().numpy().view(np.uint64), w[2])
    assert np.array_equal(d.last_row.cpu().numpy().view(np.uint64), w[3])
    assert d.n_unmatched == w[4]


@pytest.mark.parametrize("seed,n,n_clients", [(71, 0, 3), (72, 1, 1), (73, 100000, 9),
                                               (74, 300000, 2000)])
def test_publish_unsubscribes(codec, seed, n, n_clients):
    """The commit's unsubscribes (publisher/mod.rs:820-832): per client, in queue order."""
    import torch
    rng = np.random.default_rng(seed)
    ids = rng.integers(0, 10 ** 6, n, dtype=np.uint64)
    cl = rng.integers(0, n_clients + 2, n, dtype=np.uint32)
    off, ent = nxo.publish_unsubscribes(ids, cl, n_clients)
    d = codec.publish_unsubscribes(torch.from_numpy(ids.view(np.int64).copy()).cuda(),
                                   torch.from_numpy(cl.view(np.int32).copy()).cuda(), n_clients)
    assert np.array_equal(d.chan_off.cpu().numpy().view(np.uint64), off)
    assert d.n_entries == len(ent)
    assert np.array_equal(d.ent_sub[: d.n_entries].cpu().numpy().view(np.uint64), ent)
