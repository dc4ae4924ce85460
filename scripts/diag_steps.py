"""Diagnostic: f64 decode status after K back-to-back async decodes (bench.py's timing loop)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import netidx_amd  # noqa: E402
from netidx_amd.codec import Codec, Columns  # noqa: E402

codec = Codec(0)
stream = torch.cuda.Stream()
codec.set_stream(stream.cuda_stream)
n = 10_000_000
cols, wire = bench.make_f64_wire(codec, n, 0)
out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
for k in (20, 100, 200, 400, 499, 500, 501):
    wall, kms, st = bench.time_decode(codec, wire, out, n, k, 2, 1, stream)
    print(k, "err", st.err_kind, "path", st.path, "rows", st.n_rows, "kms", round(kms, 4),
          "wall/step", round(wall / k * 1e3, 4), flush=True)
