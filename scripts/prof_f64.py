#!/usr/bin/env python3
"""Profiling driver for the f64 decoders: K decodes of an N-record sequential-id frame, rotating
over 3 distinct frames and column sets, on each decoder named (seq: the sequential-id kernel;
run: the length-run probe + emit, NXG_F64_PATH=run; x: the single-pass decoder). Every decode's
columns are checked against the encoder's input once at the end.
usage: python3 scripts/prof_f64.py N K path [path ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n, k = int(sys.argv[1]), int(sys.argv[2])
    enc = netidx_amd.Codec(0)
    ids, vals = synth.f64_columns(n, synth.SEED_F64)
    cols = netidx_amd.columns_from_arrays(ids, vals)
    w0 = enc.encode_batch(cols)
    enc.close()
    W = w0.numel()
    wires = [w0] + [w0.clone() for _ in range(2)]
    outs = [Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda") for _ in range(3)]
    for path in sys.argv[3:]:
        os.environ["NXG_F64_PATH"] = "" if path == "seq" else path
        c = netidx_amd.Codec(0)
        for j in range(k):
            c.decode_async(wires[j % 3].data_ptr(), W, outs[j % 3])
        st = c.sync()
        ok = st.n_rows == n and all(torch.equal(o.id[:n], cols.id[:n]) and
                                    torch.equal(o.fixed[:n], cols.fixed[:n]) for o in outs)
        print(path, n, "ok" if ok else "MISMATCH", "diag1", c.last_diag()[1], flush=True)
        c.close()


if __name__ == "__main__":
    main()
