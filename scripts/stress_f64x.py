#!/usr/bin/env python3
"""Stress of the single-pass f64 decoder (NXG_F64_PATH=x): K decodes of 2 random-order frames of N
records, each checked on the GPU against the batch; on a mismatch prints the first bad row, the
number of bad rows and the decode's status.
usage: NXG_LIB=... python3 scripts/stress_f64x.py N K"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NXG_F64_PATH"] = "x"


def main():
    import torch
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n, k = int(sys.argv[1]), int(sys.argv[2])
    c = netidx_amd.Codec(0)
    ids, vals = synth.f64_columns(n, synth.SEED_F64)
    wires, refs = [], []
    for j in range(2):
        ids = np.random.default_rng(0x5EED0003 + j).permutation(n).astype(np.uint64)
        cols = netidx_amd.columns_from_arrays(ids, vals)
        wires.append(c.encode_batch(cols))
        refs.append(cols)
    out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    bad = 0
    for i in range(k):
        j = i % 2
        out.id.zero_()
        st = c.decode_into(wires[j].data_ptr(), wires[j].numel(), out, 0, check=False)
        diff = (out.id[:n] != refs[j].id[:n]) | (out.fixed[:n] != refs[j].fixed[:n])
        nb = int(diff.sum())
        if nb or st.n_rows != n:
            bad += 1
            first = int(torch.nonzero(diff)[0]) if nb else -1
            print(f"decode {i}: {nb} bad rows, first {first}, n_rows {st.n_rows}, path {st.path}, "
                  f"err {st.err_kind}, status {c.last_status()}", flush=True)
    print(f"n={n} decodes={k} bad={bad}", flush=True)
    c.close()


if __name__ == "__main__":
    main()
