"""The torch.distributed transport of the multi-rank calls on the CPU: gloo, world size 2 and 3,
one process per rank.

The protocols (nxg_encode_allgather, nxg_decode_sharded) live only in the library and are tested
in test_multirank_lib_cpu.py (CPU) and test_gpu_multirank.py (GPU). Here: the transport that
netidx_amd/shard.py hands them through nxg_comm_init_ops where RCCL cannot serve --
- the grouped send/recv of shards at their byte offsets (config 5's all-gather): shards encoded
  in rank order end up as exactly the whole batch's frame on every rank (the oracle decodes it:
  every id and value in order);
- the timing reduction takes the slowest rank; the record / byte split.
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


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _rank_encode(rank, world, port, total, outdir):
    _init(rank, world, port)
    try:
        b, e = shard.shard_range(total, world, rank)
        ids, vals = synth.f64_columns(e - b, synth.SEED_8GPU, id_offset=b)
        wire = nxo.encode_f64(ids, vals)
        lens = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(lens, torch.tensor([len(wire)], dtype=torch.int64))
        off = np.concatenate([[0], np.cumsum([int(x) for x in lens])])
        out = torch.zeros(int(off[-1]), dtype=torch.uint8)
        out[int(off[rank]):int(off[rank + 1])] = torch.from_numpy(wire)  # the shard in place
        shard.allgather_at_offsets(out, off, rank, world)
        slowest = shard.max_over_ranks(0.25 + rank, world)
        np.save(os.path.join(outdir, f"full{rank}.npy"), out.numpy())
        np.save(os.path.join(outdir, f"meta{rank}.npy"),
                np.array([b, e, len(wire), slowest] + list(np.diff(off)), dtype=np.float64))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 20_011), (3, 9_999)])
def test_encode_allgather_at_offsets_rebuilds_the_whole_batch(tmp_path, world, total):
    mp.spawn(_rank_encode, args=(world, _free_port(), total, str(tmp_path)), nprocs=world,
             join=True)
    ids, vals = synth.f64_columns(total, synth.SEED_8GPU)
    want = nxo.encode_f64(ids, vals)
    metas = [np.load(tmp_path / f"meta{r}.npy") for r in range(world)]
    assert [int(m[0]) for m in metas] == [shard.shard_range(total, world, r)[0]
                                          for r in range(world)]
    assert int(metas[0][0]) == 0 and int(metas[-1][1]) == total
    for r in range(world):
        full = np.load(tmp_path / f"full{r}.npy")
        assert full.tobytes() == want.tobytes()  # every rank: the single-process frame
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
