"""Full-size parity at the BASELINE.json configs: the HIP path through the C ABI against the CPU
oracle (oracle/nx_oracle.c) on EVERY column and EVERY byte -- no sampling, no self-comparison.

  configs[1]  decode 10^7 all-f64 records          (product decode vs nxo.decode of the same bytes)
  configs[2]  decode 10^7 mixed records            (every column, children, control spans)
  configs[3]  encode 10^7 records, f64 and mixed   (product encode vs the oracle encoder's bytes)

plus a frame past the Infinity Cache (the XCD-ordered emit) and the f64 decoders' robustness
cases: ids whose varints cross 2^28 (5-byte ids), ids in random order (record lengths vary record
to record: the single-pass decoder of any f64 frame takes it), that decoder forced on every shape,
the length-run decoder's exact path on every tile, and two decodes running at once on two streams
(sequential ids, and ids in random order).
Reference rules: netidx-core/src/pack.rs:504-555, netidx-value/src/lib.rs:470-506.
"""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import torch
    import netidx_amd
    assert torch.cuda.is_available()
    c = netidx_amd.Codec(0)
    yield c
    c.close()


@pytest.fixture(scope="module", params=["seq", "run"])
def f64codec(request):
    """The f64 front ends: the sequential-id kernel (default) and the length-run decoder
    (NXG_F64_PATH=run)."""
    import netidx_amd
    os.environ["NXG_F64_PATH"] = "" if request.param == "seq" else "run"
    try:
        c = netidx_amd.Codec(0)
    finally:
        del os.environ["NXG_F64_PATH"]
    c.front = request.param
    yield c
    c.close()


def _decode_dev(codec, wire, cols, flags=0):
    import torch
    dw = torch.from_numpy(np.ascontiguousarray(wire)).cuda()
    st = codec.decode_into(dw, dw.numel(), cols, flags, check=False)
    return st


def _assert_f64(cols, st, wire, n):
    import nxo
    assert st.err_kind == 0 and st.n_rows == n and st.path == 1
    o = nxo.decode(wire, cap_rows=n + 1, cap_children=1, cap_ctl=1).trim()
    assert o["err_kind"] == 0 and len(o["id"]) == n and (o["tag"] == 9).all()
    g = cols.numpy()
    assert np.array_equal(g["id"], o["id"])
    assert np.array_equal(g["fixed"], o["fixed"])


def test_config2_f64_decode_10m_every_row(f64codec):
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n = 10_000_000
    ids, vals = synth.f64_columns(n)
    wire = nxo.encode_f64(ids, vals)
    assert len(wire) == 147_886_336
    cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    st = _decode_dev(f64codec, wire, cols)
    _assert_f64(cols, st, wire, n)
    assert (f64codec.last_diag()[1] == 1) == (f64codec.front == "seq")


def test_f64_decode_past_the_infinity_cache_every_row(f64codec):
    """A 2 * 10^7-record frame (296 MB, past the 256 MiB Infinity Cache): both f64 front ends
    take their XCD-contiguous workgroup order there; every row against the oracle."""
    import netidx_amd
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n = 20_000_000
    ids, vals = synth.f64_columns(n)
    import nxo
    wire = nxo.encode_f64(ids, vals)
    assert len(wire) > 256 << 20
    cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    st = _decode_dev(f64codec, wire, cols)
    _assert_f64(cols, st, wire, n)


def test_config4_f64_encode_10m_every_byte(codec):
    import netidx_amd
    import nxo
    from netidx_amd import synth
    n = 10_000_000
    ids, vals = synth.f64_columns(n)
    out = codec.encode_batch(netidx_amd.columns_from_arrays(ids, vals)).cpu().numpy()
    assert np.array_equal(out, nxo.encode_f64(ids, vals))


def _mixed(n, seed=None):
    import nxo
    from netidx_amd import synth
    m = synth.mixed_columns(n) if seed is None else synth.mixed_columns(n, seed)
    d = nxo.Decoded(n, len(m.ctag) + 1, 1)
    for name in ("id", "tag", "fixed", "aux"):
        getattr(d, name)[:n] = getattr(m, name)
    d.ctag[:len(m.ctag)] = m.ctag
    d.cfixed[:len(m.ctag)] = m.cfixed
    d.caux[:len(m.ctag)] = m.caux
    d.s.n_rows, d.s.n_children, d.s.n_ctl = n, len(m.ctag), 0
    return m, np.frombuffer(nxo.encode(d, m.heap), np.uint8)


def test_config3_mixed_decode_10m_every_column(codec):
    import netidx_amd
    import nxo
    from netidx_amd.codec import Columns
    n = 10_000_000
    m, wire = _mixed(n)
    nc = len(m.ctag)
    cols = Columns(n + 1, nc + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
    st = _decode_dev(codec, wire, cols, netidx_amd.HINT_MIXED)
    assert st.err_kind == 0 and st.path == 4 and st.n_rows == n
    o = nxo.decode(wire, cap_rows=n + 1, cap_children=nc + 1, cap_ctl=1).trim()
    assert o["err_kind"] == 0 and len(o["id"]) == n and len(o["ctag"]) == nc
    g = cols.numpy()
    for k in ("id", "tag", "fixed", "aux", "ctag", "cfixed", "caux", "ctl_row", "ctl_off",
              "ctl_len", "ctl_variant"):
        assert np.array_equal(g[k], o[k]), k
    assert st.n_heartbeat == o["n_heartbeat"] == 0
    # and the generator's own columns (strings are zero-copy offsets into the frame, so only
    # the non-text columns are compared with the generator)
    assert np.array_equal(g["id"], m.id) and np.array_equal(g["tag"], m.tag)
    assert np.array_equal(g["ctag"], m.ctag) and np.array_equal(g["cfixed"], m.cfixed)


def test_config4_mixed_encode_10m_every_byte(codec):
    import netidx_amd
    import torch
    n = 10_000_000
    m, wire = _mixed(n)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    out = codec.encode_batch(mc, heap).cpu().numpy()
    assert np.array_equal(out, wire)


def test_f64_ids_across_2_28_on_the_fast_path(f64codec):
    """Ids grow from a per-process counter (netidx-core/src/utils.rs:130-134): a long-lived
    publisher crosses 2^28, where ids take 5 varint bytes. 10^6 records straddling it."""
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n = 1_000_000
    ids, vals = synth.f64_columns(n, 71, id_offset=2**28 - n // 2)
    wire = nxo.encode_f64(ids, vals)
    cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    _assert_f64(cols, _decode_dev(f64codec, wire, cols), wire, n)
    # 5-byte ids everywhere (random order within [2^28, 2^35))
    rng = np.random.default_rng(72)
    ids = rng.integers(2**28, 2**35, n, dtype=np.uint64)
    wire = nxo.encode_f64(ids, vals)
    _assert_f64(cols, _decode_dev(f64codec, wire, cols), wire, n)


def test_f64_ids_in_random_order(codec):
    """Record lengths that vary record to record: the length-run decoder hands the frame to the
    single-pass decoder (DevStatus.irregular), still on path 1 and bit-exact."""
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n = 2_000_000
    ids, vals = synth.f64_columns(n, 73)
    ids = np.random.default_rng(74).permutation(ids)
    wire = nxo.encode_f64(ids, vals)
    cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    for _ in range(2):  # the second frame goes straight to the single-pass decoder
        _assert_f64(cols, _decode_dev(codec, wire, cols), wire, n)


def test_f64_run_decoder_exact_path_everywhere():
    """NXG_F64R_FLAGS=1 (read at ctx creation) routes every tile of the length-run decoder
    through its exact path (merge points): bit-exact on sequential, random-order and wide ids."""
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    os.environ["NXG_F64R_FLAGS"] = "3"
    os.environ["NXG_F64_PATH"] = "run"
    try:
        c = netidx_amd.Codec(0)
    finally:
        del os.environ["NXG_F64R_FLAGS"]
        del os.environ["NXG_F64_PATH"]
    try:
        n = 300_000
        cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        for k, off in enumerate((0, 2**28 - n // 2)):
            ids, vals = synth.f64_columns(n, 80 + k, id_offset=off)
            if k == 1:
                ids = np.random.default_rng(81).permutation(ids)
            wire = nxo.encode_f64(ids, vals)
            _assert_f64(cols, _decode_dev(c, wire, cols), wire, n)
    finally:
        c.close()


def test_f64_decodes_on_two_streams_at_once():
    """Co-residency: two decodes in flight on two streams of one GPU (no workgroup of the f64
    path waits on one that may not be resident). Both bit-exact; the pair completes within
    2.5x the time of one decode alone."""
    import netidx_amd
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n = 10_000_000
    ids, vals = synth.f64_columns(n)
    import nxo
    wire = torch.from_numpy(nxo.encode_f64(ids, vals)).cuda()
    cs = [netidx_amd.Codec(0) for _ in range(2)]
    ss = [torch.cuda.Stream() for _ in range(2)]
    outs = [Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda") for _ in range(2)]
    try:
        for c, s in zip(cs, ss):
            c.set_stream(s.cuda_stream)

        def run(k_ctx, reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                for k in range(k_ctx):
                    cs[k].decode_async(wire.data_ptr(), wire.numel(), outs[k])
            sts = [cs[k].sync() for k in range(k_ctx)]
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps, sts

        run(1, 3)
        run(2, 3)
        solo, _ = run(1, 20)
        pair, sts = run(2, 20)
        for st, o in zip(sts, outs):
            assert st.path == 1 and st.n_rows == n
            assert torch.equal(o.fixed[:n].cpu(), torch.from_numpy(vals.view(np.int64)))
        assert pair < 2.5 * solo, (pair, solo)
    finally:
        for c in cs:
            c.close()


def _codec_env(name, value):
    import netidx_amd
    os.environ[name] = value
    try:
        return netidx_amd.Codec(0)
    finally:
        del os.environ[name]


def test_f64_single_pass_decoder_everywhere():
    """NXG_F64_PATH=x (read at ctx creation) puts every f64 frame on the single-pass decoder
    (nxg_decode_f64_x.hip): sequential ids, random order, 5-byte ids in random order, frames of a
    few records, frames ending on either side of its 4 KiB and 16 KiB boundaries, and malformed
    frames (the fallback reports the oracle's first error)."""
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    c = _codec_env("NXG_F64_PATH", "x")
    rng = np.random.default_rng(90)
    try:
        cases = []
        ids, vals = synth.f64_columns(1_000_000, 91)
        cases.append((ids, vals))
        cases.append((rng.permutation(ids), vals))
        cases.append((rng.integers(2**28, 2**35, 300_000, dtype=np.uint64), vals[:300_000]))
        cases.append((rng.integers(0, 2**35, 300_000, dtype=np.uint64), vals[:300_000]))
        for n in (1, 2, 3, 5, 64, 341, 342, 343, 1365, 1366, 1367, 4000):
            i2, v2 = synth.f64_columns(n, 92 + n, id_offset=int(rng.integers(0, 2**20)))
            cases.append((rng.permutation(i2), v2))
        for ids_, vals_ in cases:
            n = len(ids_)
            wire = nxo.encode_f64(ids_, vals_)
            cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
            _assert_f64(cols, _decode_dev(c, wire, cols), wire, n)
        # frames of exactly 4096 / 16384 bytes +- one record
        for target in (4096, 16384, 65536):
            i3, v3 = synth.f64_columns(target // 12 + 2, 93, id_offset=200)  # 13-byte records
            wire = nxo.encode_f64(i3, v3)
            for n in range(target // 13 - 1, target // 13 + 2):
                w = wire[: 13 * n]
                cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
                _assert_f64(cols, _decode_dev(c, w, cols), w, n)
        # the last 64 KiB workgroup holds rows in its first wave only: its empty waves start at an
        # odd row for odd n (the paired emit must not index the empty start list)
        i4, v4 = synth.f64_columns(5300, 95, id_offset=300)  # 13-byte records
        rng4 = np.random.default_rng(96)  # (its own: `rng` sets up the malformed frames below)
        for n in range(5200, 5208):
            w = nxo.encode_f64(rng4.permutation(i4[:n]), v4[:n])
            assert 65536 < len(w) < 65536 + 4096
            cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
            _assert_f64(cols, _decode_dev(c, w, cols), w, n)
        # malformed: a record cut short, a wrong value tag: the oracle's (kind, offset)
        ids, vals = synth.f64_columns(20_000, 94)
        wire = nxo.encode_f64(rng.permutation(ids), vals)
        for bad in (wire[:-3], np.concatenate([wire[:13 * 777 + 3], [0x77], wire[13 * 777 + 4:]])):
            bad = np.ascontiguousarray(bad, np.uint8)
            cols = Columns.for_frame(len(bad), netidx_amd.LAYOUT_MIXED, "cuda")
            st = _decode_dev(c, bad, cols)
            o = nxo.decode(bad)
            assert st.err_kind == o.s.err_kind != 0 and st.err_offset == o.s.err_offset
    finally:
        c.close()


def _false_record(L, rng):
    """8 value bytes whose bytes 1.. read as a record of length L: `L 04 varint(L - 11 bytes) 09`
    (L <= 14: the varint and the tag fit in the value)."""
    nb = L - 11
    b = [0x41, L, 0x04] + [0x80 | int(rng.integers(0, 128)) for _ in range(nb - 1)] + \
        [int(rng.integers(1, 128)), 0x09]
    b += [int(x) for x in rng.integers(0, 256, 8 - len(b))]
    return np.frombuffer(bytes(b), ">u8")[0]


def _record_lengths(ids):
    return 11 + np.where(ids < 128, 1, np.where(ids < 1 << 14, 2, np.where(ids < 1 << 21, 3, 4)))


def _plant_false_starts(ids, vals, frac, rng):
    """f64 values whose bytes read as a record (`L 04 id 09 ...`, L the value's own record
    length), so that the frame holds positions that pass every record check but are not starts.
    Returns the planted values and the row indices."""
    rows = np.nonzero(rng.random(len(ids)) < frac)[0]
    lens = _record_lengths(ids)
    vals = vals.copy()
    for k in rows:
        if lens[k] <= 14:
            vals[k] = _false_record(int(lens[k]), rng)
    return vals, rows


@pytest.mark.parametrize("path", ["x", "auto"])
def test_f64_false_record_starts(path):
    """Values whose bytes look like records (a false start passes every per-record check): the
    single-pass decoder drops the starts no record leads to and stays on path 1, bit-exact, for
    sparse false starts (random rows, and rows at the 4 KiB sub-tile edges); a frame where every
    value hides a false start (a false chain beside the true one through the whole frame) is still
    decoded exactly (on whichever path the decoders settle)."""
    import netidx_amd
    import nxo
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    c = _codec_env("NXG_F64_PATH", "x") if path == "x" else netidx_amd.Codec(0)
    rng = np.random.default_rng(97)
    try:
        n = 400_000
        ids, vals = synth.f64_columns(n, 98)
        ids = rng.permutation(ids)
        for frac in (0.001, 0.02):
            v2, rows = _plant_false_starts(ids, vals, frac, rng)
            assert len(rows) > 100
            wire = nxo.encode_f64(ids, v2)
            cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
            for _ in range(2):  # (auto: the second frame goes straight to the single-pass decoder)
                _assert_f64(cols, _decode_dev(c, wire, cols), wire, n)
        # false starts in the records that straddle each 4 KiB sub-tile edge, and their neighbours
        lens = _record_lengths(ids)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
        edge = np.nonzero((starts // 4096) != ((starts + lens - 1) // 4096))[0]
        near = np.unique(np.concatenate([edge, edge - 1, edge + 1]).clip(0, n - 1))
        v3 = vals.copy()
        for k in near:
            if lens[k] <= 14:
                v3[k] = _false_record(int(lens[k]), rng)
        wire = nxo.encode_f64(ids, v3)
        assert wire[starts[-1]] == lens[-1]
        cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        _assert_f64(cols, _decode_dev(c, wire, cols), wire, n)
        # every value hides a false start: exact on any path
        v4, _ = _plant_false_starts(ids, vals, 1.0, rng)
        wire = nxo.encode_f64(ids, v4)
        cols = Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
        st = _decode_dev(c, wire, cols)
        o = nxo.decode(wire, cap_rows=n + 1, cap_children=1, cap_ctl=1).trim()
        g = cols.numpy()
        assert st.err_kind == 0 and st.n_rows == n
        assert np.array_equal(g["id"], o["id"]) and np.array_equal(g["fixed"], o["fixed"])
    finally:
        c.close()


def test_f64_random_order_decodes_on_two_streams_at_once():
    """The two-stream co-residency test on a frame with ids in random order (the single-pass
    decoder: its workgroups wait only on lower-numbered ones)."""
    import netidx_amd
    import nxo
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n = 10_000_000
    ids, vals = synth.f64_columns(n, 95)
    ids = np.random.default_rng(96).permutation(ids)
    wire = torch.from_numpy(nxo.encode_f64(ids, vals)).cuda()
    cs = [_codec_env("NXG_F64_PATH", "x") for _ in range(2)]
    ss = [torch.cuda.Stream() for _ in range(2)]
    outs = [Columns(n, 0, 0, netidx_amd.LAYOUT_F64, "cuda") for _ in range(2)]
    try:
        for c, s in zip(cs, ss):
            c.set_stream(s.cuda_stream)

        def run(k_ctx, reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                for k in range(k_ctx):
                    cs[k].decode_async(wire.data_ptr(), wire.numel(), outs[k])
            sts = [cs[k].sync() for k in range(k_ctx)]
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps, sts

        run(1, 3)
        run(2, 3)
        solo, _ = run(1, 20)
        pair, sts = run(2, 20)
        for st, o in zip(sts, outs):
            assert st.path == 1 and st.n_rows == n
            assert torch.equal(o.id[:n].cpu(), torch.from_numpy(ids.view(np.int64)))
            assert torch.equal(o.fixed[:n].cpu(), torch.from_numpy(vals.view(np.int64)))
        assert pair < 2.5 * solo, (pair, solo)
    finally:
        for c in cs:
            c.close()
