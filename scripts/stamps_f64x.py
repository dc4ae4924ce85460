#!/usr/bin/env python3
"""Phase timeline of the single-pass f64 decoder from a diagnostic build (-DNXG_F64X_PROF=1,
s_memrealtime stamps at 100 MHz per workgroup): decodes random-order frames of N records (3 in
rotation), then prints, over the last decode's workgroups, percentiles of the start time, phase 1,
block scan, look-back and emit durations (us), and the kernel span.
usage: NXG_LIB=.../xprof/libnxg_codec.so python3 scripts/stamps_f64x.py [N]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NXG_F64_PATH"] = "x"


def main():
    import torch
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns, lib
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    c = netidx_amd.Codec(0)
    _, vals = synth.f64_columns(n, synth.SEED_F64)
    wires = []
    for j in range(3):
        ids = np.random.default_rng(0x5EED0003 + j).permutation(n).astype(np.uint64)
        wires.append(c.encode_batch(netidx_amd.columns_from_arrays(ids, vals)))
    outs = [Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda") for _ in range(3)]
    for i in range(12):
        c.decode_async(wires[i % 3].data_ptr(), wires[i % 3].numel(), outs[i % 3])
    c.sync()
    buf = np.zeros(6 * 16384, np.uint64)
    f = lib().nxg_debug_f64x_stamps
    f.restype = C.c_int
    f.argtypes = [C.c_void_p]
    assert f(buf.ctypes.data) == 0
    st = buf.reshape(6, 16384)
    ng = (wires[0].numel() + 65535) // 65536
    ng = min(ng, 16384)
    t = st[:5, :ng].astype(np.int64)
    t0 = t[0].min()
    us = lambda x: x / 100.0  # 100 MHz ticks
    def pct(name, x):
        q = np.percentile(x, [0, 10, 50, 90, 100])
        print(f"{name:10s} " + " ".join(f"{us(v):8.2f}" for v in q), flush=True)
    print(f"workgroups {ng}, kernel span {us(t[4].max() - t0):.2f} us; percentiles 0/10/50/90/100 (us)")
    pct("start", t[0] - t0)
    pct("phase1", t[1] - t[0])
    pct("scan", t[2] - t[1])
    pct("lookback", t[3] - t[2])
    pct("emit", t[4] - t[3])
    pct("total", t[4] - t[0])
    pct("end", t[4] - t0)
    hw = st[5, :ng]
    xcc = (hw >> np.uint64(32)).astype(np.int64)
    print("workgroups per XCC:", np.bincount(xcc, minlength=8).tolist())
    # generations: how many workgroups run at once (sampled)
    for frac in (0.1, 0.3, 0.5, 0.7, 0.9):
        tt = t0 + frac * (t[4].max() - t0)
        print(f"at {frac:.1f} of the span: {int(((t[0] <= tt) & (t[4] > tt)).sum())} resident")
    c.close()


if __name__ == "__main__":
    main()
