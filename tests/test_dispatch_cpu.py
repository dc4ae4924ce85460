"""Subscriber update dispatch on the CPU: the C oracle (oracle/nx_oracle.c nxo_dispatch) against a
line-by-line Python restatement of ConnectionCtx::process_updates_batch
(netidx/src/subscriber/connection.rs:546-567), and the host-side table builder.

Parity anchor: the reference has no dispatch test vectors; the restatement
below follows the cited loop and is the pin for the oracle, which in turn checks the GPU path
(tests/test_gpu_dispatch.py).
"""
import random

import numpy as np
import pytest

import nxo


def process_updates_batch(ids, subscriptions, n_chans):
    """subscriptions: {id: (sub_id, [chan, ...], keeps_last)}. For m in batch.drain(..): if the
    id has a subscription, push (sub.sub_id, Update(m)) onto each stream's channel batch (by_chan,
    first use creates it), then set sub.last if kept. Returns ({chan: [(sub_id, row)]},
    {id: last row})."""
    by_chan = {}
    last = {}
    for row, i in enumerate(ids):
        sub = subscriptions.get(i)
        if sub is None:
            continue
        sub_id, streams, keeps_last = sub
        for chan_id in streams:
            by_chan.setdefault(chan_id, []).append((sub_id, row))
        if keeps_last:
            last[i] = row
    return by_chan, last


def table_arrays(subs, n_ids):
    slot_of_id = np.full(n_ids, nxo.NO_SLOT, np.uint32)
    sub_ids, offs, chans, keep = [], [0], [], []
    order = sorted(subs)
    for slot, i in enumerate(order):
        sid, streams, k = subs[i]
        if i < n_ids:
            slot_of_id[i] = slot
        sub_ids.append(sid)
        chans.extend(streams)
        offs.append(len(chans))
        keep.append(1 if k else 0)
    return (order, slot_of_id, np.array(sub_ids, np.uint64), np.array(offs, np.uint32),
            np.array(chans, np.uint32), np.array(keep, np.uint8))


def random_case(rng, n_rows, n_ids, n_chans, p_sub=0.8, max_fan=3):
    subs = {}
    for i in range(n_ids):
        if rng.random() < p_sub:
            fan = rng.randint(0, max_fan)
            subs[i] = (rng.getrandbits(64), rng.sample(range(n_chans), min(fan, n_chans)),
                       rng.random() < 0.5)
    # ids: mostly in range, some repeated, some past the table, some huge
    ids = []
    for _ in range(n_rows):
        u = rng.random()
        ids.append(rng.randrange(n_ids) if u < 0.9 else
                   (n_ids + rng.randrange(5) if u < 0.95 else rng.getrandbits(64)))
    return subs, ids


def oracle_batches(ids, subs, n_ids, n_chans):
    order, slot_of_id, sub_id, off, chan, keep = table_arrays(subs, n_ids)
    chan_off, ent_sub, ent_row, last_row, um = nxo.dispatch(ids, slot_of_id, sub_id, off, chan,
                                                            keep, n_chans)
    got = {c: list(zip(ent_sub[chan_off[c]:chan_off[c + 1]].tolist(),
                       ent_row[chan_off[c]:chan_off[c + 1]].tolist()))
           for c in range(n_chans) if chan_off[c + 1] > chan_off[c]}
    last = {order[s]: int(last_row[s]) - 1 for s in range(len(order)) if last_row[s]}
    return got, last, um


@pytest.mark.parametrize("seed,n_rows,n_ids,n_chans", [
    (1, 0, 10, 3), (2, 1, 1, 1), (3, 200, 50, 4), (4, 1000, 300, 17), (5, 5000, 40, 64),
    (6, 3000, 2000, 1), (7, 777, 100, 300),
])
def test_oracle_matches_process_updates_batch(seed, n_rows, n_ids, n_chans):
    rng = random.Random(seed)
    subs, ids = random_case(rng, n_rows, n_ids, n_chans)
    want_batches, want_last = process_updates_batch(ids, subs, n_chans)
    got, last, um = oracle_batches(ids, subs, n_ids, n_chans)
    assert got == want_batches
    assert last == want_last
    assert um == sum(1 for i in ids if i not in subs)


def test_oracle_empty_table_drops_everything():
    got, last, um = oracle_batches([0, 1, 2, 2**63], {}, 0, 2)
    assert got == {} and last == {} and um == 4


def test_subtable_builder_on_cpu():
    import netidx_amd
    subs = {0: (7, [1], True), 3: (9, [0, 1], False), 5: (11, [], True)}
    t = netidx_amd.SubTable.from_subscriptions(subs, n_chans=2, device="cpu")
    assert t.slot_of_id.numpy().view(np.uint32).tolist() == [0, netidx_amd.NO_SLOT,
                                                             netidx_amd.NO_SLOT, 1,
                                                             netidx_amd.NO_SLOT, 2]
    assert t.slot_sub_id.numpy().view(np.uint64).tolist() == [7, 9, 11]
    assert t.slot_stream_off.numpy().view(np.uint32).tolist() == [0, 1, 3, 3]
    assert t.stream_chan.numpy().view(np.uint32).tolist() == [1, 0, 1]
    assert t.slot_has_last.numpy().tolist() == [1, 0, 1]
