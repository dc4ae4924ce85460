#!/usr/bin/env python3
"""Diagnostics of nxg_decode_range on a random-order f64 frame: per range the NxgRange and the
last attempt's DevStatus (fast_fail, irregular, path, rows, err, timeout; diag[0..7])."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
assert torch.cuda.is_available()
import netidx_amd
from netidx_amd import shard, synth
from netidx_amd.codec import Columns, lib
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import nxo

codec = netidx_amd.Codec(0)
L = lib()
for kind in ("perm", "mixed"):
    n = 300_007
    ids, vals = synth.f64_columns(n, 111)
    ids = np.random.default_rng(2).permutation(ids)
    wire = nxo.encode_f64(ids, vals)
    W = len(wire)
    dw = torch.from_numpy(np.ascontiguousarray(wire)).cuda()
    for world in (2, 3):
        for r in range(world):
            b, e = shard.shard_range(W, world, r)
            cols = Columns(max((e - b) // 12 + 2, 1), 0, 0, netidx_amd.LAYOUT_F64, "cuda")
            rng = codec.decode_range(dw, W, b, e, cols)
            st = (C.c_ulonglong * 6)()
            L.nxg_debug_status(C.c_void_p(codec.ctx), st)
            print(kind, world, r, (b, e), "ok", rng.ok, "entry", rng.entry, "exit", rng.exit, "rows",
                  rng.n_rows, "status", list(st), "diag", codec.last_diag(), flush=True)
    break
