#!/usr/bin/env python3
"""Timing of the type-partitioned view (nxg_partition_by_tag) on config 3's decoded columns at
10^7 rows: K synchronous calls, HIP events on the codec stream; the view checked against its
numpy restatement once. usage: [NXG_LIB=...] python3 scripts/ab_partition.py tag"""
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
    from netidx_amd.codec import Columns
    n = 10_000_000
    codec = netidx_amd.Codec(0)
    stream = torch.cuda.Stream()
    codec.set_stream(stream.cuda_stream)
    m = synth.mixed_columns(n)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    wire = codec.encode_batch(mc, heap)
    out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
    codec.decode_into(wire, wire.numel(), out, netidx_amd.HINT_MIXED)
    view = codec.partition_by_tag(out)
    g = out.numpy()
    want = nxo.partition_by_tag(g["tag"], g["fixed"], g["aux"])
    got = view.numpy()
    ok = all(np.array_equal(got[k], want[k]) for k in want)
    res = {"tag": sys.argv[1], "ok": ok}
    for rep in range(3):
        k = 20
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(k):
            view = codec.partition_by_tag(out, view)
        e1.record(stream)
        torch.cuda.synchronize()
        res[f"ms{rep}"] = round(e0.elapsed_time(e1) / k, 4)
    print(json.dumps(res), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
