"""Self-help look-backs (nxg_device.h lookback_selfhelp_fn): no kernel of the f64 encoder, the
general encoder or the single-pass f64 decoder waits on a workgroup that may not be running --
an unpublished predecessor's aggregate is computed by the waiting workgroup itself. With
NXG_LOOKBACK_PATIENCE=0 (read at context creation) every predecessor not yet published when a
workgroup looks back is computed that way, so the self-help path runs on many tiles; the results
must stay bit-exact against the oracle. Then two processes share the GPU, each running a mixed
encode and a random-order f64 decode back to back (the case where an XCD falls behind), and
every output is checked.
Reference rules: netidx-core/src/pack.rs:504-555, netidx/src/publisher/server.rs:604-629.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _codec(patience):
    import torch
    import netidx_amd
    assert torch.cuda.is_available()  # torch's HIP runtime first (netidx_amd.codec.lib)
    os.environ["NXG_LOOKBACK_PATIENCE"] = str(patience)
    try:
        return netidx_amd.Codec(0)
    finally:
        del os.environ["NXG_LOOKBACK_PATIENCE"]


def _mixed(n, seed):
    import nxo
    from netidx_amd import synth
    m = synth.mixed_columns(n, seed)
    d = nxo.Decoded(n, len(m.ctag) + 1, 1)
    for name in ("id", "tag", "fixed", "aux"):
        getattr(d, name)[:n] = getattr(m, name)
    d.ctag[:len(m.ctag)] = m.ctag
    d.cfixed[:len(m.ctag)] = m.cfixed
    d.caux[:len(m.ctag)] = m.caux
    d.s.n_rows, d.s.n_children, d.s.n_ctl = n, len(m.ctag), 0
    return m, np.frombuffer(nxo.encode(d, m.heap), np.uint8)


def _random_f64(n, seed):
    import nxo
    from netidx_amd import synth
    ids, vals = synth.f64_columns(n, seed)
    ids = np.random.default_rng(seed).permutation(ids)
    return ids, vals, nxo.encode_f64(ids, vals)


def _check_all(c, seed):
    import torch
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    # f64 encode (nxg_enc_f64_kernel)
    ids, vals = synth.f64_columns(2_000_000, seed)
    out = c.encode_batch(netidx_amd.columns_from_arrays(ids, vals)).cpu().numpy()
    assert np.array_equal(out, nxo.encode_f64(ids, vals)), "f64 encode"
    # general encode (nxg_enc_rows_kernel)
    m, want = _mixed(1_000_000, seed)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    got = c.encode_batch(mc, heap).cpu().numpy()
    assert np.array_equal(got, want), "mixed encode"
    # single-pass f64 decode (nxg_f64x_kernel): random-order ids
    rids, rvals, wire = _random_f64(2_000_000, seed + 1)
    cols = Columns(len(rids), 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    dw = torch.from_numpy(wire).cuda()
    for _ in range(2):  # the second call goes straight to the single-pass decoder
        st = c.decode_into(dw, dw.numel(), cols)
        g = cols.numpy()
        assert st.path == 1 and np.array_equal(g["id"], rids) and np.array_equal(g["fixed"], rvals)


def test_selfhelp_everywhere_is_bit_exact():
    c = _codec(0)
    try:
        _check_all(c, 501)
    finally:
        c.close()
    _codec(128).close()  # back to the default patience for the tests after this one


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _proc(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        c = _codec(128)
        dist.barrier()  # both processes start their kernels together
        ok = 1
        try:
            for k in range(3):
                _check_all(c, 600 + 10 * rank + k)
        except AssertionError as e:
            print(f"rank {rank}: {e}", flush=True)
            ok = 0
        np.save(os.path.join(outdir, f"ok{rank}.npy"), np.array([ok]))
        c.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_processes_share_the_gpu():
    """Mixed encode and random-order decode in two processes at once: bit-exact, no watchdog."""
    import tempfile
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_proc, args=(2, _free_port(), d), nprocs=2, join=True)
        for r in range(2):
            assert int(np.load(os.path.join(d, f"ok{r}.npy"))[0]) == 1, f"rank {r}"
