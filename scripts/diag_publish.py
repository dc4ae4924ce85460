"""Timing of the publisher commit (nxg_publish_commit) at 10^7 rows, 16 clients, half
UpdateChanged: run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import netidx_amd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
n_cl = 16
rng = np.random.default_rng(2)
ids = np.arange(n, dtype=np.uint64)
vals = rng.integers(0, 2**63, n, dtype=np.uint64)
fan = 1 + (rng.random(n) < 0.5).astype(np.int64)
off = np.concatenate([[0], np.cumsum(fan)]).astype(np.uint32)
# a client subscribes to an Id once (pb.by_id[id].subscribed is a set): distinct per row
first = rng.integers(0, n_cl, n)
second = (first + 1 + rng.integers(0, n_cl - 1, n)) % n_cl
client = np.empty(int(off[-1]), np.uint32)
client[off[:-1]] = first
client[off[:-1][fan == 2] + 1] = second[fan == 2]
kind = np.where(np.arange(n) % 2 == 0, 1, 0).astype(np.uint8)
cur = np.where(rng.random(n) < 0.5, vals, vals ^ np.uint64(1))
codec = netidx_amd.Codec(0)
tab = netidx_amd.PubTable(np.arange(n, dtype=np.uint32), off, client, n_cl, None, cur)
batch = netidx_amd.columns_from_arrays(ids, vals)
dkind = torch.from_numpy(kind).cuda()
to = torch.zeros(n, dtype=torch.int32, device="cuda")
for _ in range(3):
    d = codec.publish_commit(tab, batch, dkind, to, cap=int(off[-1]))
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    d = codec.publish_commit(tab, batch, dkind, to, cap=int(off[-1]))
torch.cuda.synchronize()
print(f"n={n} call={(time.perf_counter() - t0) / 10 * 1e3:.3f} ms entries={d.n_entries}", flush=True)
