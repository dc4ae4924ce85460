#!/usr/bin/env python3
"""A/B of the f64 encoders (config 4): the sequential-id kernel (nxg_encode_f64_seq.hip, the
default) against the tiled look-back kernel (NXG_F64_ENC=tile), per record count: K async encodes
of one column set into one output buffer (the bench's encode_f64 leg), HIP events on the codec
stream. Both outputs are compared with the oracle's encoder first (10^7) or with each other (10^8,
plus the oracle on the first and last 10^6 records' bytes).
usage: [NXG_LIB=...] python3 scripts/ab_enc_f64.py tag N [N ...]"""
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
    tag = sys.argv[1]
    stream = torch.cuda.Stream()
    for n in [int(x) for x in sys.argv[2:]]:
        ids, vals = synth.f64_columns(n, synth.SEED_F64)
        cols = netidx_amd.columns_from_arrays(ids, vals)
        outs = {}
        for path in os.environ.get("AB_ENC_PATHS", "seq,tile").split(","):
            os.environ["NXG_F64_ENC"] = "" if path == "seq" else "tile"
            codec = netidx_amd.Codec(0)
            codec.set_stream(stream.cuda_stream)
            # (sized on the host, so that a kernel trace holds writing launches only)
            W = int((11 + 1 + (ids >= 2**7).astype(np.int64) + (ids >= 2**14) + (ids >= 2**21) +
                     (ids >= 2**28)).sum())
            dout = torch.empty(W + 64, dtype=torch.uint8, device="cuda")
            res = {"tag": tag, "path": path, "n": n, "W": W, "alg_bytes": W + 16 * n}
            for _ in range(2):
                codec.encode_async(cols, None, dout.data_ptr(), dout.numel())
                codec.sync()
            res["kernel"] = codec.last_encode_kernel()
            k = 40 if n <= 10**7 else 10
            for rep in range(3):
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(k):
                    codec.encode_async(cols, None, dout.data_ptr(), dout.numel())
                e1.record(stream)
                codec.sync()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / k
                res[f"ms{rep}"] = round(ms, 4)
                res[f"frac{rep}"] = round((W + 16 * n) / (ms / 1e3) / 8e12, 4)
            outs[path] = dout[:W].cpu().numpy()
            codec.close()
            print(json.dumps(res), flush=True)
        os.environ.pop("NXG_F64_ENC", None)
        if len(outs) < 2:
            continue
        same = bool(np.array_equal(outs["seq"], outs["tile"]))
        if n <= 10**7:
            ok = same and bool(np.array_equal(outs["seq"], nxo.encode_f64(ids, vals)))
        else:
            m = 10**6
            head = nxo.encode_f64(ids[:m], vals[:m])
            ok = same and bool(np.array_equal(outs["seq"][: len(head)], head))
        print(json.dumps({"tag": tag, "n": n, "seq_equals_tile": same, "oracle_ok": ok}), flush=True)
        del cols, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
