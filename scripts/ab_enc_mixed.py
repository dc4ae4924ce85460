#!/usr/bin/env python3
"""A/B timing of the general encoder (nxg_enc_rows_kernel) for one library build (NXG_LIB):
config 3's columns at 10^7 rows encoded K times (async, HIP events on the codec stream), plus the
archive-batch encode of the same mix; the frame checked against the oracle's encoder once.
usage: NXG_LIB=... python3 scripts/ab_enc_mixed.py tag"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch
    import netidx_amd
    import nxo
    from netidx_amd import synth
    n = 10_000_000
    codec = netidx_amd.Codec(0)
    stream = torch.cuda.Stream()
    codec.set_stream(stream.cuda_stream)
    m = synth.mixed_columns(n)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    W = codec.encoded_len(mc, heap)
    dout = torch.empty(W + 64, dtype=torch.uint8, device="cuda")
    codec.encode_async(mc, heap, dout.data_ptr(), dout.numel())
    codec.sync()
    d = nxo.Decoded(n, len(m.ctag) + 1, 1)
    for name in ("id", "tag", "fixed", "aux"):
        getattr(d, name)[:n] = getattr(m, name)
    d.ctag[:len(m.ctag)] = m.ctag
    d.cfixed[:len(m.ctag)] = m.cfixed
    d.caux[:len(m.ctag)] = m.caux
    d.s.n_rows, d.s.n_children, d.s.n_ctl = n, len(m.ctag), 0
    ok = bool(np.array_equal(dout[:W].cpu().numpy(), np.frombuffer(nxo.encode(d, m.heap), np.uint8)))
    res = {"tag": sys.argv[1], "ok": ok, "W": W}
    for rep in range(3):
        k = 20
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            codec.encode_async(mc, heap, dout.data_ptr(), dout.numel())
        e1.record(stream)
        codec.sync()
        torch.cuda.synchronize()
        res[f"ms{rep}"] = round(e0.elapsed_time(e1) / k, 4)
    print(json.dumps(res), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
