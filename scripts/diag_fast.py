"""Diagnostics (GPU): which path the fast mixed decoder (config-3 mix) and the fast archive
decoder take at growing sizes, each on a fresh context, with the columns checked against the
general decoder's."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    os.environ["NXG_MIXED_PATH"] = "general"
    gen = netidx_amd.Codec(0)
    del os.environ["NXG_MIXED_PATH"]
    for n in (10_000, 100_000, 1_000_000, 3_000_000, 10_000_000):
        m = synth.mixed_columns(n)
        mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
        heap = torch.from_numpy(m.heap.copy()).cuda()
        c = netidx_amd.Codec(0)
        wire = c.encode_batch(mc, heap)
        out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
        ref = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
        st = c.decode_into(wire, wire.numel(), out, netidx_amd.HINT_MIXED, check=False)
        sr = gen.decode_into(wire, wire.numel(), ref, netidx_amd.HINT_MIXED, check=False)
        same = all(torch.equal(out.t[k][:n], ref.t[k][:n]) for k in ("id", "tag", "fixed", "aux"))
        print(f"mixed n={n}: path {st.path} rows {st.n_rows} err {st.err_kind}; general path "
              f"{sr.path}; columns equal {same}", flush=True)
        c.close()
    for n in (100_000, 1_000_000, 10_000_000):
        m = synth.archive_columns(n)
        mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
        heap = torch.from_numpy(m.heap.copy()).cuda()
        c = netidx_amd.Codec(0)
        buf = c.encode_archive(mc, heap)
        out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
        st, used = c.decode_archive(buf, buf.numel(), out)
        print(f"archive n={n}: path {st.path} rows {st.n_rows} err {st.err_kind} used {used} of "
              f"{buf.numel()}", flush=True)
        c.close()


def long_text():
    """The GPU test's long_text archive batch, with the fast path's decline reasons."""
    import ctypes as C
    import random
    import zlib
    import importlib.util
    import netidx_amd
    from netidx_amd import codec as cm
    from netidx_amd.codec import Columns
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    spec = importlib.util.spec_from_file_location(
        "mg", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)

    def varint(x):
        o = bytearray()
        while x >= 0x80:
            o.append((x & 0x7f) | 0x80)
            x >>= 7
        o.append(x)
        return bytes(o)
    for sizes in ([100, 300, 4000, 20000], [100, 300], [4000], [20000]):
        rng = random.Random(zlib.crc32(b"long_text"))
        items = []
        for i in range(6000):
            iid = rng.getrandbits(rng.choice([7, 14, 21, 28, 32]))
            if rng.random() < 0.05:
                s = bytes(rng.randrange(0x61, 0x7b) for _ in range(rng.choice(sizes)))
                if rng.random() < 0.5:
                    s = s[:50] + "\u00e9".encode() + s[52:]
                v = (12, s)
            else:
                v = mg.rand_value(rng)
                while v[0] in (19, 21, 22):
                    v = mg.rand_value(rng)
            items.append(varint(iid) + mg.enc_value(v))
        buf = np.frombuffer(varint(len(items)) + b"".join(items), np.uint8)
        import torch
        c = netidx_amd.Codec(0)
        d = torch.from_numpy(buf.copy()).cuda()
        out = Columns(len(items) + 1, len(buf) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
        st, used = c.decode_archive(d, d.numel(), out, check=False)
        fa = (C.c_ulonglong * 8)()
        cm.lib().nxg_debug_fa(C.c_void_p(c.ctx if isinstance(c.ctx, int) else c.ctx.value), fa)
        print(f"long_text sizes {sizes}: {len(buf)} bytes, path {st.path} err {st.err_kind}; "
              f"FaHead fast_fail {fa[0] & 0xffffffff} end {fa[1]} items {fa[3]} recounts {fa[5]} "
              f"why {fa[6]:#x}; first declining tile {(~(fa[7] >> 16)) & 0xffffffffffff} "
              f"(why {fa[7] & 0xffff:#x}) of {(len(buf) + 4095) // 4096}", flush=True)
        # the items around that tile: where each item starts (host walk of the batch)
        ft = (~(fa[7] >> 16)) & 0xffffffffffff
        pos, lens = len(varint(len(items))), []
        for it in items:
            lens.append((pos, len(it)))
            pos += len(it)
        near = [(p, l) for p, l in lens if p + l > (ft - 1) * 4096 and p < (ft + 1) * 4096]
        print("  items near it (start, len):", [(p - ft * 4096, l) for p, l in near][:40])
        c.close()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "long_text":
        long_text()
    else:
        main()
