#!/usr/bin/env python3
"""The bench's 10^8 leg alone, for a clean rocprofv3 trace of the north-star kernel: 10^8
sequential-id f64 records, 2 frames and column sets in rotation, W warmup decodes and then K
decodes as one backlog (nxg_decode_frames_async), as bench.py's extras.decode_f64_1e8 times
them. Every decode is a full decode by the sequential-id kernel (checked: the connection's
status says the kernel decoded each one, diag[1]); the columns are checked against the encoder's
input at the end. Prints the HIP-event time per decode for comparison with the trace.
usage: python3 scripts/prof_f64_1e8.py [K] [W]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    w = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    n = 100_000_000
    c = netidx_amd.Codec(0)
    ids, vals = synth.f64_columns(n, synth.SEED_F64)
    cols = netidx_amd.columns_from_arrays(ids, vals)
    del ids, vals
    w0 = c.encode_batch(cols)
    W = w0.numel()
    wires = [w0, w0.clone()]
    outs = [Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda") for _ in range(2)]
    s = torch.cuda.Stream()
    c.set_stream(s.cuda_stream)

    def backlog(m):
        c.decode_frames_async([wires[j % 2].data_ptr() for j in range(m)], [W] * m,
                              [outs[j % 2] for j in range(m)])

    backlog(w)
    st = c.sync()
    assert st.n_rows == n and st.path == 1
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    backlog(k)
    e1.record(s)
    st = c.sync()
    ok = st.n_rows == n and c.last_diag()[1] == 1 and all(
        torch.equal(o.id[:n], cols.id[:n]) and torch.equal(o.fixed[:n], cols.fixed[:n])
        for o in outs)
    ms = e0.elapsed_time(e1) / k
    print(f"10^8 seq decode: {k} frames, {ms:.4f} ms per decode (HIP events), "
          f"{(W + 16 * n) / ms / 1e6:.1f} GB/s, {'ok' if ok else 'MISMATCH'}", flush=True)
    c.close()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
