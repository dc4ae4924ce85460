"""The type-partitioned view of decoded mixed columns (nxg_partition.hip, SURVEY.md 8a's optional
output; BASELINE configs[2]'s "LDS histogram + scan") against its numpy restatement
(tests/nxo.py partition_by_tag: a stable sort by tag).

Pinned: config 3 decoded by the product decoder at 10^7 rows (the view of its own columns), every
tag value 0..255 in random order, runs of one tag across tile edges, 1..5000 rows around the
4096-row tile and 64-row round edges, an empty batch, and the API errors (F64-only columns, a
view too small). Integer bookkeeping only: bit-exact.
"""
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


def _cols(tag, fixed, aux):
    import netidx_amd
    from netidx_amd.codec import Columns
    n = len(tag)
    c = Columns(max(n, 1), 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
    import torch
    c.tag[:n] = torch.from_numpy(np.asarray(tag, np.uint8))
    c.fixed[:n] = torch.from_numpy(np.asarray(fixed, np.uint64).view(np.int64))
    c.aux[:n] = torch.from_numpy(np.asarray(aux, np.uint32).view(np.int32))
    torch.cuda.synchronize()
    c.s.n_rows = n
    return c


def _check(view, tag, fixed, aux):
    import nxo
    want = nxo.partition_by_tag(tag, fixed, aux)
    got = view.numpy()
    assert view.n_rows == len(tag)
    for k in ("count", "off", "row_of", "fixed", "aux", "rank"):
        assert np.array_equal(got[k], want[k]), k


def test_partition_config3_decoded_columns(codec):
    """Config 3 through the product decoder, then its view: every array bit-exact."""
    import netidx_amd
    import torch
    from netidx_amd import synth
    from netidx_amd.codec import Columns
    n = 10_000_000
    m = synth.mixed_columns(n)
    mc = netidx_amd.columns_from_arrays(m.id, m.fixed, m.tag, m.aux, m.ctag, m.cfixed, m.caux)
    heap = torch.from_numpy(m.heap.copy()).cuda()
    wire = codec.encode_batch(mc, heap)
    out = Columns(n + 1, len(m.ctag) + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
    st = codec.decode_into(wire, wire.numel(), out, netidx_amd.HINT_MIXED)
    assert st.n_rows == n
    view = codec.partition_by_tag(out)
    g = out.numpy()
    _check(view, g["tag"], g["fixed"], g["aux"])
    assert set(np.flatnonzero(view.count).tolist()) == {6, 9, 10, 12, 19}


def test_partition_shapes(codec):
    rng = np.random.default_rng(61)
    cases = []
    for n in (1, 2, 63, 64, 65, 1023, 1024, 4095, 4096, 4097, 5000):
        cases.append(rng.integers(0, 28, n).astype(np.uint8))
    cases.append(rng.integers(0, 256, 300_000).astype(np.uint8))  # every tag value
    runs = np.repeat(rng.integers(0, 256, 400).astype(np.uint8), rng.integers(1, 3000, 400))
    cases.append(runs)  # runs of one tag across tile and round edges
    cases.append(np.full(70_000, 12, np.uint8))  # one tag
    view = None
    for tag in cases:
        n = len(tag)
        fixed = rng.integers(0, 2**64, n, dtype=np.uint64)
        aux = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        view = codec.partition_by_tag(_cols(tag, fixed, aux), view)
        _check(view, tag, fixed, aux)


def test_partition_empty_and_errors(codec):
    import netidx_amd
    from netidx_amd.codec import Columns
    empty = _cols(np.zeros(0, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint32))
    v = codec.partition_by_tag(empty)
    assert v.n_rows == 0 and int(v.off[-1]) == 0 and not v.count.any()
    f64 = Columns(10, 0, 0, netidx_amd.LAYOUT_F64, "cuda")
    f64.s.n_rows = 10
    with pytest.raises(netidx_amd.CodecError, match="mixed-layout"):
        codec.partition_by_tag(f64)
    big = _cols(np.ones(100, np.uint8), np.zeros(100, np.uint64), np.zeros(100, np.uint32))
    small = netidx_amd.TagView(50)
    with pytest.raises(netidx_amd.CodecError, match="capacity"):
        _too_small(codec, big, small)


def _too_small(codec, cols, view):
    """partition_by_tag reallocates a view that is too small; call the ABI directly instead."""
    import ctypes as C
    from netidx_amd.codec import NetidxError, NxgTagView, _check, lib
    v = NxgTagView()
    v.cap_rows = view.cap
    v.rank, v.row_of = view.rank.data_ptr(), view.row_of.data_ptr()
    v.fixed, v.aux = view.fixed.data_ptr(), view.aux.data_ptr()
    err = NetidxError()
    _check(lib().nxg_partition_by_tag(codec.ctx, C.byref(cols.s), C.byref(v), C.byref(err)), err)
