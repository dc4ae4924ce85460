#!/usr/bin/env python3
"""A/B timing of the fast mixed decoder for one library build (NXG_LIB selects it): config 3 at
10^7 records (plain, and with 1 % Heartbeats + 1 % 200-byte strings), K decodes each, HIP events
on the codec stream; every variant's columns checked against the oracle once.
usage: NXG_LIB=... python3 scripts/ab_mixed.py tag [n]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch
    assert torch.cuda.is_available()
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    tag = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
    codec = netidx_amd.Codec(0)
    stream = torch.cuda.Stream()
    codec.set_stream(stream.cuda_stream)
    kinds = {"ctlonly": ("ctl",), "plainonly": ("plain",)}.get(tag, ("plain", "ctl"))
    for kind in kinds:
        if kind == "plain":
            m = synth.mixed_columns(n)
            cr = np.zeros(0, np.uint64)
            mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
        else:
            m, cr, co, cl, cv = synth.mixed_columns_ctl(n)
            mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed,
                                                m.caux, cr, co, cl, cv)
        heap = torch.from_numpy(m.heap.copy()).cuda()
        wire = codec.encode_batch(mc, heap)
        out = Columns(n + 1, len(m.ctag) + 1, len(cr) + 1, netidx_amd.LAYOUT_MIXED, "cuda")
        st = codec.decode_into(wire, wire.numel(), out, netidx_amd.HINT_MIXED)
        o = nxo.decode(wire.cpu().numpy(), cap_rows=n + 1, cap_children=len(m.ctag) + 1,
                       cap_ctl=len(cr) + 1).trim()
        g = out.numpy()
        ok = all(np.array_equal(g[k], o[k]) for k in ("id", "tag", "fixed", "aux", "ctag",
                                                      "cfixed", "caux", "ctl_row", "ctl_off"))
        res = {"tag": tag, "kind": kind, "path": st.path, "ok": bool(ok), "diag": [int(x) for x in codec.last_diag()],
               "tiles": (wire.numel() + 4095) // 4096}
        for rep in range(3):
            k = 20
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(k):
                codec.decode_async(wire.data_ptr(), wire.numel(), out, netidx_amd.HINT_MIXED)
            e1.record(stream)
            st = codec.sync()
            torch.cuda.synchronize()
            if rep:
                res[f"ms{rep}"] = round(e0.elapsed_time(e1) / k, 4)
        res["path_after"] = st.path
        res["diag_after"] = [int(x) for x in codec.last_diag()]
        print(json.dumps(res), flush=True)
        del mc, heap, wire, out
        torch.cuda.empty_cache()
    codec.close()


if __name__ == "__main__":
    main()
