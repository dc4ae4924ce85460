"""GPU parity of the subscriber update dispatch (nxg_dispatch_updates, include/nxg_codec.h)
against the CPU oracle (nxo_dispatch, a restatement of process_updates_batch,
netidx/src/subscriber/connection.rs:546-567): identical per-channel batches (SubId, row) in
identical order, identical last rows and unmatched counts. Bit-exact (index work)."""
import random

import numpy as np
import pytest

import nxo
from test_dispatch_cpu import random_case, table_arrays

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import torch
    import netidx_amd
    assert torch.cuda.is_available()
    c = netidx_amd.Codec(0)
    yield c
    c.close()


def run_both(codec, ids, subs, n_ids, n_chans):
    import torch
    import netidx_amd
    order, slot_of_id, sub_id, off, chan, keep = table_arrays(subs, n_ids)
    ids = np.asarray(ids, np.uint64)
    tab = netidx_amd.SubTable(slot_of_id, sub_id, off, chan, keep, n_chans)
    did = torch.from_numpy(ids.view(np.int64).copy()).cuda()
    d = codec.dispatch_updates(tab, did)
    w_off, w_sub, w_row, w_last, w_um = nxo.dispatch(ids, slot_of_id, sub_id, off, chan, keep,
                                                     n_chans)
    g_off = d.chan_off.cpu().numpy().view(np.uint64)
    assert np.array_equal(g_off, w_off)
    assert d.n_entries == len(w_sub)
    assert np.array_equal(d.ent_sub[: d.n_entries].cpu().numpy().view(np.uint64), w_sub)
    assert np.array_equal(d.ent_row[: d.n_entries].cpu().numpy().view(np.uint64), w_row)
    assert np.array_equal(d.last_row.cpu().numpy().view(np.uint64), w_last)
    assert d.n_unmatched == w_um
    return d


@pytest.mark.parametrize("seed,n_rows,n_ids,n_chans,max_fan", [
    (11, 0, 10, 3, 2),          # empty batch
    (12, 1, 1, 1, 1),
    (13, 63, 50, 4, 3),         # one partial step
    (14, 64, 50, 4, 3),
    (15, 1025, 300, 17, 4),     # segment edge
    (16, 20000, 2000, 1, 1),    # one channel: every row in one batch
    (17, 50000, 5000, 1024, 3),  # largest LDS-counter case
    (18, 30000, 3000, 1025, 3),  # global-memory counters
    (19, 20000, 20000, 5000, 2),
    (20, 100000, 1000, 64, 8),  # repeated ids: last = the final occurrence
    (21, 129, 100, 5, 2),       # one row past a 128-row segment
    (22, 5000, 3000, 70000, 2),  # more channels than the count pass's row cache names
])
def test_dispatch_matches_oracle(codec, seed, n_rows, n_ids, n_chans, max_fan):
    rng = random.Random(seed)
    subs, ids = random_case(rng, n_rows, n_ids, n_chans, max_fan=max_fan)
    run_both(codec, ids, subs, n_ids, n_chans)


def test_dispatch_large_dense(codec):
    """10^6 distinct ids, each subscribed once on one of 16 channels (the bench shape)."""
    rng = np.random.default_rng(5)
    n = 1_000_000
    n_chans = 16
    slot_of_id = np.arange(n, dtype=np.uint32)
    sub_id = rng.integers(0, 2**63, n, dtype=np.uint64)
    off = np.arange(n + 1, dtype=np.uint32)
    chan = rng.integers(0, n_chans, n, dtype=np.uint32)
    keep = (rng.random(n) < 0.5).astype(np.uint8)
    ids = rng.permutation(n).astype(np.uint64)
    import torch
    import netidx_amd
    tab = netidx_amd.SubTable(slot_of_id, sub_id, off, chan, keep, n_chans)
    d = codec.dispatch_updates(tab, torch.from_numpy(ids.view(np.int64).copy()).cuda())
    w = nxo.dispatch(ids, slot_of_id, sub_id, off, chan, keep, n_chans)
    assert np.array_equal(d.chan_off.cpu().numpy().view(np.uint64), w[0])
    assert np.array_equal(d.ent_sub[: d.n_entries].cpu().numpy().view(np.uint64), w[1])
    assert np.array_equal(d.ent_row[: d.n_entries].cpu().numpy().view(np.uint64), w[2])
    assert np.array_equal(d.last_row.cpu().numpy().view(np.uint64), w[3])


def test_decode_then_dispatch(codec):
    """The decoded id column feeds the dispatch directly (the decode_task -> process_updates_batch
    path of connection.rs:209-242, 546-567)."""
    import torch
    import netidx_amd
    rng = np.random.default_rng(9)
    n = 200_000
    ids = rng.permutation(n).astype(np.uint64)
    vals = rng.integers(0, 2**64, n, dtype=np.uint64)
    wire = nxo.encode_f64(ids, vals)
    cols, st = codec.decode_batch(torch.from_numpy(wire.copy()).cuda(), layout=netidx_amd.LAYOUT_F64)
    assert st.err_kind == 0 and cols.n_rows == n
    subs = {int(i): (int(i) * 3 + 1, [int(i) % 5] if i % 7 else [], bool(i % 2)) for i in
            range(0, n, 2)}
    order, slot_of_id, sub_id, off, chan, keep = table_arrays(subs, n)
    tab = netidx_amd.SubTable(slot_of_id, sub_id, off, chan, keep, 5)
    d = codec.dispatch_updates(tab, cols.id, cols.n_rows)
    w = nxo.dispatch(ids, slot_of_id, sub_id, off, chan, keep, 5)
    assert np.array_equal(d.ent_row[: d.n_entries].cpu().numpy().view(np.uint64), w[2])
    assert np.array_equal(d.ent_sub[: d.n_entries].cpu().numpy().view(np.uint64), w[1])
    assert d.n_unmatched == w[4] == n // 2


def test_dispatch_capacity_error(codec):
    import torch
    import netidx_amd
    subs = {0: (5, [0, 1], False)}
    order, slot_of_id, sub_id, off, chan, keep = table_arrays(subs, 1)
    tab = netidx_amd.SubTable(slot_of_id, sub_id, off, chan, keep, 2)
    ids = torch.zeros(10, dtype=torch.int64, device="cuda")
    with pytest.raises(netidx_amd.CodecError, match="needs 20 entries"):
        codec.dispatch_updates(tab, ids, cap=19)
