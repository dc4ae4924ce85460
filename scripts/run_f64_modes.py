"""Driver: 10^8 (or N) sequential-id f64 records decoded k times as one stream of frames
(nxg_decode_frames_async) and k times one call per frame (nxg_decode_updates_async); HIP-event
times per frame for both. Usage: run_f64_modes.py [records] [k]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import netidx_amd  # noqa: E402
from netidx_amd import synth  # noqa: E402
from netidx_amd.codec import Columns  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
c = netidx_amd.Codec(0)
s = torch.cuda.Stream()
c.set_stream(s.cuda_stream)
ids, vals = synth.f64_columns(n, synth.SEED_F64)
cols = netidx_amd.columns_from_arrays(ids, vals)
wire = c.encode_batch(cols)
out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")


def run(mode):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    if mode == "stream":
        c.decode_frames_async([wire.data_ptr()] * k, [wire.numel()] * k, [out] * k)
    else:
        for _ in range(k):
            c.decode_async(wire.data_ptr(), wire.numel(), out)
    e1.record(s)
    st = c.sync()
    torch.cuda.synchronize()
    assert st.path == 1 and st.n_rows == n
    return e0.elapsed_time(e1) / k


for rep in range(3):
    for mode in ("stream", "call"):
        print(f"{mode} {n} rep {rep}: {run(mode):.4f} ms/frame", flush=True)
