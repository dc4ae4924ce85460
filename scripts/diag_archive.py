"""Archive batch decode/encode timing at n items (config-3 mix, 5 % Unsubscribed)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import netidx_amd
from netidx_amd import synth
from netidx_amd.codec import Columns

codec = netidx_amd.Codec(0)
for n in [int(x) for x in (sys.argv[1:] or ["10000000"])]:
    m = synth.archive_columns(n)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    buf = codec.encode_archive(mc, heap)
    out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
    for rep in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        codec.encode_archive(mc, heap, buf)
        torch.cuda.synchronize()
        te = time.perf_counter() - t0
        t0 = time.perf_counter()
        st, used = codec.decode_archive(buf, buf.numel(), out)
        torch.cuda.synchronize()
        td = time.perf_counter() - t0
    print(f"n={n} bytes={buf.numel()} enc={te*1e3:.3f}ms dec={td*1e3:.3f}ms rows={st.n_rows} "
          f"err={st.err_kind} used={used}", flush=True)
