#!/usr/bin/env python3
"""A/B timing of the f64 decode for one library build (NXG_LIB selects it): per record count,
K back-to-back decodes one call each (nxg_decode_updates_async) and as one stream of frames
(nxg_decode_frames_async), HIP events on the codec stream; every variant's columns are compared
with the encoder's input columns (bit-exact) before timing.
usage: NXG_LIB=... python3 scripts/ab_f64.py tag N [N ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    tag = sys.argv[1]
    codec = netidx_amd.Codec(0)
    stream = torch.cuda.Stream()
    codec.set_stream(stream.cuda_stream)
    perm = os.environ.get("AB_PERM") == "1"
    for n in [int(x) for x in sys.argv[2:]]:
        ids, vals = synth.f64_columns(n, synth.SEED_F64)
        if perm:
            import numpy as np
            ids = np.random.default_rng(0x5EED0003).permutation(n).astype(np.uint64)
        cols = netidx_amd.columns_from_arrays(ids, vals)
        wire = codec.encode_batch(cols)
        W = wire.numel()
        out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        res = {"tag": tag, "n": n, "W": W}
        for mode in ("call", "stream"):
            k = 40 if n <= 10**7 else 12
            for rep in range(2):
                out.id.zero_()
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                if mode == "call":
                    for _ in range(k):
                        codec.decode_async(wire.data_ptr(), W, out)
                else:
                    codec.decode_frames_async([wire.data_ptr()] * k, [W] * k, [out] * k)
                e1.record(stream)
                st = codec.sync()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / k
                ok = st.n_rows == n and torch.equal(out.id[:n], cols.id[:n]) and \
                    torch.equal(out.fixed[:n], cols.fixed[:n])
                res[f"{mode}_ms"] = round(ms, 4)
                res[f"{mode}_frac"] = round((W + 16 * n) / (ms / 1e3) / 8e12, 4)
                res[f"{mode}_ok"] = bool(ok)
                res[f"{mode}_path"] = st.path
        print(json.dumps(res), flush=True)
        del cols, wire, out
        torch.cuda.empty_cache()
    codec.close()


if __name__ == "__main__":
    main()
