"""Driver for profiling: 10^7 archive items of the config-3 mix (5 % Unsubscribed) encoded and
decoded on the fast path, checked once against the generator's ids and tags.
Usage: run_archive.py [items] [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import netidx_amd  # noqa: E402
from netidx_amd import synth  # noqa: E402
from netidx_amd.codec import Columns  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
c = netidx_amd.Codec(0)
m = synth.archive_columns(n)
mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
heap = torch.from_numpy(m.heap.copy()).cuda()
buf = c.encode_archive(mc, heap)
out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
for _ in range(reps):
    st, used = c.decode_archive(buf, buf.numel(), out)
ok = torch.equal(out.id[:n].cpu(), mc.id[:n].cpu()) and torch.equal(out.tag[:n].cpu(), mc.tag[:n].cpu())
import ctypes as C  # noqa: E402
from netidx_amd import codec as cm  # noqa: E402
fa = (C.c_ulonglong * 8)()
cm.lib().nxg_debug_fa(C.c_void_p(c.ctx), fa)
tiles = (buf.numel() + 4095) // 4096
print(f"n={n} path {st.path} rows {st.n_rows} used {used} ok {ok}; tiles {tiles}, recounted by "
      f"the resolve pass {fa[5]}", flush=True)
