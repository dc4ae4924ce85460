"""Section clocks of the archive count pass from a diagnostic build (-DNXG_FA_PROF=1): one decode
of 10^7 items after a warm-up, the accumulators read before and after it.
usage: NXG_LIB=.../fap/libnxg_codec.so python3 scripts/prof_fa.py [items]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns, lib
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    c = netidx_amd.Codec(0)
    m = synth.archive_columns(n)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    buf = c.encode_archive(mc, heap)
    out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
    c.decode_archive(buf, buf.numel(), out)
    torch.cuda.synchronize()
    f = lib().nxg_debug_fa_prof
    a = (C.c_ulonglong * 16)()
    b = (C.c_ulonglong * 16)()
    f(a)
    st, used = c.decode_archive(buf, buf.numel(), out)
    torch.cuda.synchronize()
    f(b)
    d = [b[i] - a[i] for i in range(16)]
    waves = max(d[8], 1)
    names = ["image", "own spec walk", "walk before tile", "own exact walk", "chain"]
    tot = sum(d[:5])
    print(f"n={n} path {st.path} waves {d[8]}: clocks per wave (s_memtime) and share")
    for i, nm in enumerate(names):
        print(f"  {nm:18s} {d[i] / waves:10.0f}  {100 * d[i] / max(tot, 1):5.1f} %")
    print(f"  lanes re-walked per wave {d[9] / waves:.2f}; waves off the ballot path "
          f"{d[10]} ({100 * d[10] / waves:.1f} %); chunks walked by the wave {d[11]}", flush=True)


main()
