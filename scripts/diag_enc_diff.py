"""Encode config-3 columns of n rows (seed) and report the first byte where the library's frame
differs from the oracle's, with the tile (1024 rows) it falls in. usage: diag_enc_diff.py n seed"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import torch
assert torch.cuda.is_available()
import netidx_amd
import nxo
from netidx_amd import synth

n = int(sys.argv[1]); seed = int(sys.argv[2])
m = synth.mixed_columns(n, seed)
d = nxo.Decoded(n, len(m.ctag) + 1, 1)
for name in ("id", "tag", "fixed", "aux"):
    getattr(d, name)[:n] = getattr(m, name)
d.ctag[:len(m.ctag)] = m.ctag
d.cfixed[:len(m.ctag)] = m.cfixed
d.caux[:len(m.ctag)] = m.caux
d.s.n_rows, d.s.n_children, d.s.n_ctl = n, len(m.ctag), 0
wire = np.frombuffer(nxo.encode(d, m.heap), np.uint8)
codec = netidx_amd.Codec(0)
cols = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
heap = torch.from_numpy(m.heap.copy()).cuda()
for rep in range(3):
    out = codec.encode_batch(cols, heap).cpu().numpy()
    if len(out) != len(wire):
        print("length", len(out), len(wire)); continue
    bad = np.flatnonzero(out != wire)
    if not len(bad):
        print("identical"); continue
    b0 = int(bad[0]) & ~15
    print(f"{len(bad)} bad bytes, first {bad[0]}; block {b0}: got {out[b0:b0+16].tobytes().hex()} want {wire[b0:b0+16].tobytes().hex()}")
    print("  want around:", wire[b0-16:b0+48].tobytes().hex())
