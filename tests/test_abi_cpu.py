"""CPU-only checks of the product library: it loads, and exports every symbol that
include/nxg_codec.h declares. Host framing is checked against the reference rules
(netidx/src/channel.rs:107-126, 177-257, 379-443). No GPU compute is called here."""
import os
import re

import numpy as np

import netidx_amd
from netidx_amd import codec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nxg_codec.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nxg_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    for f in ["nxg_ctx_new", "nxg_decode_updates", "nxg_encode_updates", "nxg_encoded_len",
              "nxg_columns_alloc", "nxg_frame_split"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    L = netidx_amd.lib()
    missing = [f for f in declared_functions() if not hasattr(L, f)]
    assert not missing, missing
    assert set(declared_functions()) == set(codec.SIGNATURES), \
        "ctypes signatures out of sync with the header"


def test_version():
    assert netidx_amd.lib().nxg_version().startswith(b"nxg ")


def test_frame_header_roundtrip():
    # flush_buf: u32 BE, bit 31 = encrypted (channel.rs:110-118)
    assert netidx_amd.frame_header(0x0102, False) == b"\x00\x00\x01\x02"
    assert netidx_amd.frame_header(5, True) == b"\x80\x00\x00\x05"
    assert netidx_amd.frame_parse_header(b"\x80\x00\x00\x05") == (5, True)
    assert netidx_amd.frame_parse_header(b"\x3f\xff\xff\xff") == (0x3FFFFFFF, False)
    assert netidx_amd.frame_parse_header(b"\x00\x01") is None


def ref_frame_split(lens):
    """Literal restatement of queue_send + try_flush (channel.rs:177-202, 237-257)."""
    MAX_BATCH = 0x3FFFFFFF
    buf_len, boundries = 0, []
    for ln in lens:
        last = boundries[-1] if boundries else 0
        if (buf_len - last) + ln > MAX_BATCH:
            boundries.append(buf_len - sum(boundries))
        buf_len += ln
    chunks, rem = [], buf_len
    for b in boundries:
        chunks.append(b)
        rem -= b
    if rem:
        chunks.append(rem)
    return chunks


def test_frame_split_matches_queue_send():
    assert list(netidx_amd.frame_split([12] * 10)) == [120]
    # 10^8 f64 records (1,497,886,336 B) split into two frames, as SURVEY 8d notes
    rng = np.random.default_rng(3)
    for lens in ([0x3FFFFFFF, 1, 5], [0x20000000] * 7, list(rng.integers(1, 300_000_000, 40))):
        assert list(netidx_amd.frame_split(lens)) == ref_frame_split(lens)


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        return
    try:
        netidx_amd.Codec(0)
    except netidx_amd.CodecError:
        return
    raise AssertionError("Codec() must fail loudly without a gfx950 GPU")
