#!/usr/bin/env python3
"""Phase timeline of the general encoder's rows kernel from a diagnostic build (-DNXG_ENC_PROF=1,
s_memrealtime stamps at 100 MHz per tile): encodes the config-3 mixed batch of N rows a few times,
then prints percentiles over the last encode's tiles of each phase's duration (us).
usage: NXG_LIB=.../encp/libnxg_codec.so python3 scripts/stamps_enc.py [N]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import lib
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    c = netidx_amd.Codec(0)
    m = synth.mixed_columns(n)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    W = c.encoded_len(mc, heap)
    out = torch.empty(W + 64, dtype=torch.uint8, device="cuda")
    for _ in range(5):
        c.encode_into(mc, heap, out.data_ptr(), W)
    torch.cuda.synchronize()
    buf = np.zeros(7 * 16384, np.uint64)
    f = lib().nxg_debug_enc_stamps
    f.restype = C.c_int
    f.argtypes = [C.c_void_p]
    assert f(buf.ctypes.data) == 0
    nt = min((n + 1023) // 1024, 16384)
    t = buf.reshape(7, 16384)[:, :nt].astype(np.int64)
    t0 = t[0].min()
    us = lambda x: x / 100.0

    def pct(name, x):
        q = np.percentile(x, [0, 10, 50, 90, 100])
        print(f"{name:10s} " + " ".join(f"{us(v):8.2f}" for v in q), flush=True)
    print(f"tiles {nt}, kernel span {us(t[6].max() - t0):.2f} us; percentiles 0/10/50/90/100 (us)")
    pct("start", t[0] - t0)
    for k, name in enumerate(["classify", "size", "scan", "stage", "lookback", "store"]):
        pct(name, t[k + 1] - t[k])
    pct("total", t[6] - t[0])
    for frac in (0.25, 0.5, 0.75):
        tt = t0 + frac * (t[6].max() - t0)
        print(f"at {frac:.2f} of the span: {int(((t[0] <= tt) & (t[6] > tt)).sum())} resident")
    c.close()


if __name__ == "__main__":
    main()
