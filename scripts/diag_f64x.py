"""Diagnostics (GPU): the single-pass f64 decoder (nxg_f64x_kernel, NXG_F64_PATH=x) and the
stream-of-frames decode on sequential and random-order ids at growing sizes: path, rows, and
whether the columns match the batch."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    plain = netidx_amd.Codec(0)
    os.environ["NXG_F64_PATH"] = "x"
    forced = netidx_amd.Codec(0)
    del os.environ["NXG_F64_PATH"]
    for n in (1000, 100_000, 1_000_000, 3_000_000, 10_000_000):
        for order in ("seq", "rand"):
            ids, vals = synth.f64_columns(n, synth.SEED_F64)
            if order == "rand":
                ids = np.random.default_rng(3).permutation(n).astype(np.uint64)
            cols = netidx_amd.columns_from_arrays(ids, vals)
            wire = plain.encode_batch(cols)
            for name, c in (("x", forced), ("auto", plain)):
                out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
                out.id.zero_()
                c.decode_async(wire.data_ptr(), wire.numel(), out)
                st = c.sync()
                ok = torch.equal(out.id[:n], cols.id[:n]) and torch.equal(out.fixed[:n], cols.fixed[:n])
                print(f"n={n} {order} {name}: path {st.path} rows {st.n_rows} ok {ok}", flush=True)
            fresh = netidx_amd.Codec(0)
            out = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
            out.id.zero_()
            fresh.decode_frames_async([wire.data_ptr()] * 4, [wire.numel()] * 4, [out] * 4)
            st = fresh.sync()
            ok = torch.equal(out.id[:n], cols.id[:n]) and torch.equal(out.fixed[:n], cols.fixed[:n])
            print(f"n={n} {order} stream(fresh ctx): path {st.path} rows {st.n_rows} ok {ok}",
                  flush=True)
            fresh.close()


if __name__ == "__main__":
    main()
