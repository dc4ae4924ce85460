"""Multi-rank path of bench.py on the CPU: gloo, world size 2 (and 3), one process per rank.

bench.py --gpus N runs one process per GPU over RCCL. Its data path has no collective (each rank
decodes its own shard); config 5 all-gathers the ranks' encoded shards. The helpers that do this
(netidx_amd/shard.py) are device-agnostic, so here they run over gloo on CPU tensors, with the
oracle standing in for the per-rank GPU encoder. Checked: the shards partition the batch, the
gathered frame is exactly the whole batch's frame (decoded by the oracle, every id and value in
order), and the timing reduction takes the slowest rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import nxo
from netidx_amd import shard, synth


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, total, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b, e = shard.shard_range(total, world, rank)
        ids, vals = synth.f64_columns(e - b, synth.SEED_8GPU, id_offset=b)
        wire = nxo.encode_f64(ids, vals)
        # pad the local buffer: only the first len(wire) bytes are payload
        local = torch.zeros(len(wire) + 97, dtype=torch.uint8)
        local[:len(wire)] = torch.from_numpy(wire)
        full, lengths = shard.gather_frames(local, len(wire), world)
        slowest = shard.max_over_ranks(0.25 + rank, world)
        np.save(os.path.join(outdir, f"full{rank}.npy"), full.numpy())
        np.save(os.path.join(outdir, f"meta{rank}.npy"),
                np.array([b, e, len(wire), slowest] + lengths, dtype=np.float64))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 20_011), (3, 9_999)])
def test_gather_frames_rebuilds_the_whole_batch(tmp_path, world, total):
    mp.spawn(_rank_main, args=(world, _free_port(), total, str(tmp_path)), nprocs=world,
             join=True)
    ids, vals = synth.f64_columns(total, synth.SEED_8GPU)
    want = nxo.encode_f64(ids, vals)
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    # shards partition [0, total) in rank order
    assert [int(m[0]) for m in metas] == [shard.shard_range(total, world, r)[0]
                                          for r in range(world)]
    assert int(metas[0][0]) == 0 and int(metas[-1][1]) == total
    for r in range(world - 1):
        assert int(metas[r][1]) == int(metas[r + 1][0])
    for r in range(world):
        full = np.load(tmp_path / f"full{r}.npy")
        # every rank holds the same frame, byte-identical to the single-process encode
        assert full.tobytes() == want.tobytes()
        assert float(metas[r][3]) == 0.25 + (world - 1)  # max over ranks
        assert [int(x) for x in metas[r][4:]] == [int(m[2]) for m in metas]
    d = nxo.decode(want, cap_rows=total + 1, cap_children=1, cap_ctl=1)
    assert d.s.err_kind == 0 and d.s.n_rows == total
    t = d.trim()
    assert np.array_equal(t["id"], ids) and np.array_equal(t["fixed"], vals)


def test_shard_range_partitions():
    for total in (0, 1, 7, 10_000_000, 100_000_000):
        for world in (1, 2, 3, 4, 8):
            spans = [shard.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1
            assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_max_over_ranks_single_process():
    assert shard.max_over_ranks(3.5, 1) == 3.5
