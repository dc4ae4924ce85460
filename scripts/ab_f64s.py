#!/usr/bin/env python3
"""A/B of the f64 decoders for one library build (NXG_LIB selects it): the sequential-id decoder
(default) against the length-run decoder (NXG_F64_PATH=run), per record count: K decodes of ONE
frame into one column set, and K decodes rotating over 3 distinct frames and column sets (working
set > 3x the 256 MiB Infinity Cache at 10^8; at 10^7 3 x 308 MB), HIP events on the codec stream.
Every variant's columns are compared with the encoder's input columns (bit-exact) first.
usage: NXG_LIB=... python3 scripts/ab_f64s.py tag N [N ...]"""
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
    paths = os.environ.get("AB_PATHS", "seq,run").split(",")
    stream = torch.cuda.Stream()
    for n in [int(x) for x in sys.argv[2:]]:
        enc = netidx_amd.Codec(0)
        ids, vals = synth.f64_columns(n, synth.SEED_F64)
        cols = netidx_amd.columns_from_arrays(ids, vals)
        w0 = enc.encode_batch(cols)
        enc.close()
        W = w0.numel()
        wires = [w0] + [w0.clone() for _ in range(2)]
        outs = [Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda") for _ in range(3)]
        for path in paths:
            os.environ["NXG_F64_PATH"] = "" if path == "seq" else path
            codec = netidx_amd.Codec(0)
            codec.set_stream(stream.cuda_stream)
            res = {"tag": tag, "path": path, "n": n, "W": W}
            for o in outs:
                o.id.zero_()
            torch.cuda.synchronize()  # (the zeroing runs on torch's stream, the decode on ours)
            st = codec.decode_into(wires[0].data_ptr(), W, outs[0])
            res["diag1"] = codec.last_diag()[1]
            res["ok"] = bool(st.n_rows == n and torch.equal(outs[0].id[:n], cols.id[:n])
                             and torch.equal(outs[0].fixed[:n], cols.fixed[:n]))
            modes = ["same", "rot3"] + (["stream_same", "stream_rot3"] if path == "run" else [])
            for mode in modes:
                k = 60 if n <= 10**7 else 12
                rot = mode.endswith("rot3")
                for rep in range(3):
                    torch.cuda.synchronize()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    if mode.startswith("stream"):
                        sel = [j % 3 if rot else 0 for j in range(k)]
                        codec.decode_frames_async([wires[j].data_ptr() for j in sel], [W] * k,
                                                  [outs[j] for j in sel])
                    else:
                        for j in range(k):
                            i = j % 3 if rot else 0
                            codec.decode_async(wires[i].data_ptr(), W, outs[i])
                    e1.record(stream)
                    st = codec.sync()
                    torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1) / k
                    if rep == 0:
                        continue  # warm-up
                    key = f"{mode}_ms{rep}"
                    res[key] = round(ms, 4)
                res[f"{mode}_frac"] = round((W + 16 * n) / (min(res[f'{mode}_ms1'], res[f'{mode}_ms2']) / 1e3) / 8e12, 4)
            res["ok_after"] = bool(all(torch.equal(o.id[:n], cols.id[:n]) for o in outs))
            print(json.dumps(res), flush=True)
            codec.close()
        del cols, wires, outs, w0
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
