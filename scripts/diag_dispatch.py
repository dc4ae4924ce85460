"""Timing of the subscriber dispatch (nxg_dispatch_updates) at 10^7 rows, 16 channels: run under
rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import netidx_amd

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
n_chans = int(sys.argv[2]) if len(sys.argv) > 2 else 16
codec = netidx_amd.Codec(0)
rng = np.random.default_rng(1)
order = sys.argv[3] if len(sys.argv) > 3 else "random"
ids = torch.from_numpy((np.arange(n) if order == "seq" else rng.permutation(n)).astype(np.int64)).cuda()
tab = netidx_amd.SubTable(np.arange(n, dtype=np.uint32), rng.integers(0, 2**63, n, dtype=np.uint64),
                          np.arange(n + 1, dtype=np.uint32),
                          rng.integers(0, n_chans, n, dtype=np.uint32),
                          (rng.random(n) < 0.5).astype(np.uint8), n_chans)
for _ in range(3):
    d = codec.dispatch_updates(tab, ids, n, cap=n)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    d = codec.dispatch_updates(tab, ids, n, cap=n)
torch.cuda.synchronize()
print(f"n={n} chans={n_chans} call={(time.perf_counter() - t0) / 10 * 1e3:.3f} ms "
      f"entries={d.n_entries} ids={order}", flush=True)
