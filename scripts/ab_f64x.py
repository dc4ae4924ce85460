#!/usr/bin/env python3
"""A/B timing of the single-pass f64 decoder (NXG_F64_PATH=x) on random-order ids for one library
build (NXG_LIB): 10^7 (3 frames in rotation) and 10^8 (2 frames), K decodes each, HIP events on
the codec stream; every output checked against the batch.
usage: NXG_LIB=... python3 scripts/ab_f64x.py tag [sizes...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NXG_F64_PATH"] = "x"


def main():
    import numpy as np
    import torch
    assert torch.cuda.is_available()
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    tag = sys.argv[1]
    sizes = [int(x) for x in sys.argv[2:]] or [10_000_000, 100_000_000]
    for n in sizes:
        nf = 3 if n <= 10_000_000 else 2
        c = netidx_amd.Codec(0)
        stream = torch.cuda.Stream()
        c.set_stream(stream.cuda_stream)
        ids, vals = synth.f64_columns(n, synth.SEED_F64)
        wires, refs = [], []
        for j in range(nf):
            ids = np.random.default_rng(0x5EED0003 + j).permutation(n).astype(np.uint64)
            cols = netidx_amd.columns_from_arrays(ids, vals)
            wires.append(c.encode_batch(cols))
            refs.append(cols)
        outs = [Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda") for _ in range(nf)]
        for j in range(nf):
            c.decode_async(wires[j].data_ptr(), wires[j].numel(), outs[j])
        st = c.sync()
        ok = all(torch.equal(outs[j].id[:n], refs[j].id[:n]) and torch.equal(outs[j].fixed[:n], refs[j].fixed[:n])
                 for j in range(nf))
        res = {"tag": tag, "n": n, "path": st.path, "ok": bool(ok)}
        k = 30 if n <= 10_000_000 else 10
        for rep in range(2):
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for i in range(k):
                c.decode_async(wires[i % nf].data_ptr(), wires[i % nf].numel(), outs[i % nf])
            e1.record(stream)
            st = c.sync()
            torch.cuda.synchronize()
            res[f"ms{rep}"] = round(e0.elapsed_time(e1) / k, 4)
        W = wires[0].numel()
        res["frac"] = round((W + 16 * n) / (res["ms1"] * 1e-3) / 8e12, 4)
        print(json.dumps(res), flush=True)
        c.close()
        del wires, outs, refs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
