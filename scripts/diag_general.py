"""Diagnostics of the general decode kernel on config-3 data (timing + DevStatus.diag)."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import torch

import netidx_amd
from netidx_amd import synth
from netidx_amd.codec import Columns, lib

NAMES = ["run_fixes", "rep_exhausted", "repair_rounds", "rep_wrong_guess", "spec_tries", "rep_missed", "rep_spurious", "fix_entries"]


def diag(codec):
    a = (C.c_ulonglong * 8)()
    lib().nxg_debug_diag(C.c_void_p(codec.ctx), a)
    return dict(zip(NAMES, list(a)))


codec = netidx_amd.Codec(0)
for n in [int(x) for x in (sys.argv[1:] or ["100000", "1000000", "10000000"])]:
    m = synth.mixed_columns(n)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    t0 = time.perf_counter()
    wire = codec.encode_batch(mc, heap)
    torch.cuda.synchronize()
    t_enc = time.perf_counter() - t0
    out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = codec.decode_into(wire, wire.numel(), out, netidx_amd.HINT_MIXED)
        t = time.perf_counter() - t0
    # text / bytes rows hold byte offsets (heap on encode, wire on decode) and arrays child
    # bases: compare every other value exactly
    tag = mc.tag[:n]
    plain = (tag != 12) & (tag != 13) & (tag != 18) & (tag != 19) & (tag != 20) & (tag != 21)
    ok = (torch.equal(out.id[:n], mc.id[:n]) and torch.equal(out.tag[:n], tag)
          and torch.equal(out.aux[:n], mc.aux[:n])
          and torch.equal(out.fixed[:n][plain], mc.fixed[:n][plain]))
    tiles = (wire.numel() + 4095) // 4096
    print(f"n={n} W={wire.numel()} tiles={tiles} enc={t_enc*1e3:.1f}ms dec={t*1e3:.2f}ms "
          f"rows={st.n_rows} err={st.err_kind} ok={ok} {diag(codec)}", flush=True)
