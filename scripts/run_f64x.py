"""Driver for profiling: f64 frames with ids in random order decoded on the single-pass decoder
(NXG_F64_PATH=x), checked once against the batch. Usage: run_f64x.py [records] [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NXG_F64_PATH"] = "x"
import torch  # noqa: E402

import netidx_amd  # noqa: E402
from netidx_amd import synth  # noqa: E402
from netidx_amd.codec import Columns  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
c = netidx_amd.Codec(0)
ids, vals = synth.f64_columns(n, synth.SEED_F64)
ids = np.random.default_rng(0x5EED0003).permutation(n).astype(np.uint64)
cols = netidx_amd.columns_from_arrays(ids, vals)
wire = c.encode_batch(cols)
out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
for _ in range(reps):
    c.decode_async(wire.data_ptr(), wire.numel(), out)
st = c.sync()
ok = torch.equal(out.id[:n], cols.id[:n]) and torch.equal(out.fixed[:n], cols.fixed[:n])
print(f"n={n} path {st.path} rows {st.n_rows} ok {ok}", flush=True)
