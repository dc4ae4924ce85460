#!/usr/bin/env python3
"""Does the config-3 decode time depend on what ran before it? Times the mixed decode (20 frames,
HIP events), then runs ~10 s of 10^8-record f64 decodes, then times the mixed decode again, on one
codec and on a fresh one."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    stream = torch.cuda.Stream()
    codec = netidx_amd.Codec(0)
    codec.set_stream(stream.cuda_stream)
    n = 10_000_000
    m = synth.mixed_columns(n)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    wire = codec.encode_batch(mc, heap)
    out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")

    def tmix(c, tag):
        for _ in range(2):
            c.decode_async(wire.data_ptr(), wire.numel(), out, netidx_amd.HINT_MIXED)
            c.sync()
        res = {"tag": tag}
        for rep in range(3):
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(20):
                c.decode_async(wire.data_ptr(), wire.numel(), out, netidx_amd.HINT_MIXED)
            e1.record(stream)
            c.sync()
            torch.cuda.synchronize()
            res[f"ms{rep}"] = round(e0.elapsed_time(e1) / 20, 4)
        print(json.dumps(res), flush=True)

    tmix(codec, "cold")
    nf = 100_000_000
    ids, vals = synth.f64_columns(nf)
    fc = netidx_amd.columns_from_arrays(ids, vals)
    fw = codec.encode_batch(fc)
    fo = Columns(nf, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    t0 = time.time()
    while time.time() - t0 < 10:
        for _ in range(20):
            codec.decode_async(fw.data_ptr(), fw.numel(), fo)
        codec.sync()
    tmix(codec, "after 10 s of 10^8 decodes")
    c2 = netidx_amd.Codec(0)
    c2.set_stream(stream.cuda_stream)
    tmix(c2, "fresh codec")
    time.sleep(5)
    tmix(c2, "after 5 s idle")


if __name__ == "__main__":
    main()
