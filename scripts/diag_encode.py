"""Mixed (config-3) encode timing at n records: k back-to-back async encodes, HIP events."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import netidx_amd
from netidx_amd import synth

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
codec = netidx_amd.Codec(0)
stream = torch.cuda.Stream()
codec.set_stream(stream.cuda_stream)
m = synth.mixed_columns(n)
mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
heap = torch.from_numpy(m.heap.copy()).cuda()
try:
    wire = codec.encode_batch(mc, heap)
except Exception as e:  # a timing-only variant (scripts/ab_variants.sh) may size frames wrongly
    print("encode_batch:", e, flush=True)
    wire = torch.zeros(n * 40 + heap.numel(), dtype=torch.uint8, device="cuda")
dout = torch.empty(wire.numel() + 64, dtype=torch.uint8, device="cuda")
for _ in range(2):
    codec.encode_async(mc, heap, dout.data_ptr(), dout.numel())
    codec.sync()
s = stream
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
k = 20
torch.cuda.synchronize()
e0.record(s)
for _ in range(k):
    codec.encode_async(mc, heap, dout.data_ptr(), dout.numel())
e1.record(s)
codec.sync()
torch.cuda.synchronize()
same = torch.equal(dout[: wire.numel()], wire)
print(f"n={n} W={wire.numel()} encode={e0.elapsed_time(e1) / k:.4f} ms identical={same}", flush=True)
