"""GPU zstd decompression of compressed archive records (nxg_archive_decompress, nxg_zstd.hip)
against the committed libzstd fixtures (tests/golden/make_zstd.py): every record's bytes equal
libzstd's output (dictionary frames at level 19 as the reference writes them, frames without a
dictionary at levels 1-19, several blocks, raw and RLE blocks, a checksum, no content size, an
empty payload, matches far back), then every batch decoded on the GPU (nxg_decode_archive_batch)
against the oracle's decode. Errors: a record's own error code, the others unaffected."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def codec():
    import torch
    import netidx_amd
    assert torch.cuda.is_available()
    c = netidx_amd.Codec(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def fx():
    m = json.load(open(os.path.join(G, "zstd_manifest.json")))
    rec = np.frombuffer(open(os.path.join(G, "zstd_records.bin"), "rb").read(), np.uint8)
    plain = open(os.path.join(G, "zstd_plain.bin"), "rb").read()
    d = open(os.path.join(G, "zstd_dict.bin"), "rb").read()
    return m["records"], rec, plain, d


def _run(codec, zd, rec, ents, indexed):
    return codec.archive_decompress(rec, [(e["rec_off"], e["rec_len"]) for e in ents], indexed, zd)


def test_decompress_every_fixture(codec, fx):
    ents, rec, plain, d = fx
    zd = codec.zstd_dict(d)
    groups = {}
    for e in ents:
        groups.setdefault((e["dict"], e["indexed"]), []).append(e)
    seen = 0
    for (use_dict, indexed), es in groups.items():
        out, res = _run(codec, zd if use_dict else None, rec, es, indexed)
        host = out.cpu().numpy()
        for e, (oo, ol, er) in zip(es, res):
            want = plain[e["plain_off"]:e["plain_off"] + e["plain_len"]]
            assert er == 0, (e["kind"], er)
            assert ol == len(want) and host[oo:oo + ol].tobytes() == want, e["kind"]
            seen += 1
    assert seen == len(ents)
    zd.close()


def test_decompressed_batches_decode_on_the_gpu(codec, fx):
    import nxo
    import netidx_amd
    from netidx_amd.codec import Columns
    ents, rec, plain, d = fx
    zd = codec.zstd_dict(d)
    es = [e for e in ents if e["batch"] and e["dict"]]
    for indexed in (False, True):
        part = [e for e in es if e["indexed"] == indexed]
        out, res = _run(codec, zd, rec, part, indexed)
        for e, (oo, ol, er) in zip(part, res):
            assert er == 0
            cols = Columns(ol + 1, ol + 1, 1, netidx_amd.LAYOUT_MIXED, "cuda")
            st, used = codec.decode_archive(out[oo:oo + ol], ol, cols)
            o, used_o = nxo.decode_archive(np.frombuffer(plain[e["plain_off"]:e["plain_off"] + ol],
                                                         np.uint8))
            o = o.trim()
            assert used == used_o == ol and st.n_rows == len(o["id"])
            g = cols.numpy()
            for k in ("id", "tag", "aux", "ctag", "cfixed", "caux"):
                assert np.array_equal(g[k], o[k]), k
            # text offsets index the batch itself: compare as offsets
            assert np.array_equal(g["fixed"], o["fixed"])
    zd.close()


def test_errors_are_per_record(codec, fx):
    ents, rec, plain, d = fx
    zd = codec.zstd_dict(d)
    es = [e for e in ents if e["dict"] and not e["indexed"]][:6]
    buf = bytearray(rec.tobytes())
    # record 1: a corrupt byte in its frame's block data; record 3: not a zstd frame; record 4:
    # an uncompressed length too small for its payload
    e1, e3, e4 = es[1], es[3], es[4]
    buf[e1["rec_off"] + e1["rec_len"] - 3] ^= 0xFF
    buf[e3["rec_off"] + 4] ^= 0x55
    if e4["plain_len"] > 1:
        buf[e4["rec_off"]:e4["rec_off"] + 4] = (e4["plain_len"] - 1).to_bytes(4, "big")
    out, res = _run(codec, zd, np.frombuffer(bytes(buf), np.uint8), es, False)
    host = out.cpu().numpy()
    assert res[3][2] == 1  # not a zstd frame
    if e4["plain_len"] > 1:
        assert res[4][2] == 3  # the batch is longer than the record says
    for k in (0, 2, 5):
        oo, ol, er = res[k]
        want = plain[es[k]["plain_off"]:es[k]["plain_off"] + es[k]["plain_len"]]
        assert er == 0 and host[oo:oo + ol].tobytes() == want
    # without the dictionary: dictionary frames are refused
    out, res = _run(codec, None, rec, es[:2], False)
    assert all(r[2] == 4 for r in res)
    zd.close()


def test_crafted_frames_rejected_on_the_device(codec):
    """crafted frames libzstd rejects (tests/golden/make_zstd_crafted.py) -- a Huffman
    tree description of 256 weights, one without two weight-1 symbols, four-stream literals of
    fewer than 6 bytes -- fail their record on the GPU too (a per-record error, never output), and
    a good fixture record decompressed in the same call is unaffected."""
    m = json.load(open(os.path.join(G, "zstd_crafted.json")))["cases"]
    ents = json.load(open(os.path.join(G, "zstd_manifest.json")))["records"]
    rec = open(os.path.join(G, "zstd_records.bin"), "rb").read()
    plain = open(os.path.join(G, "zstd_plain.bin"), "rb").read()
    good = [e for e in ents if not e["dict"] and not e["indexed"] and e["plain_len"]][0]
    parts, recs = [], []
    off = 0
    for c in m:
        f = bytes.fromhex(c["frame"])
        r = (len(f) + 64).to_bytes(4, "big") + f  # generous plain length: the frame must fail
        parts.append(r)
        recs.append((off, len(r)))
        off += len(r)
    g = rec[good["rec_off"]:good["rec_off"] + good["rec_len"]]
    parts.append(g)
    recs.append((off, len(g)))
    src = np.frombuffer(b"".join(parts), np.uint8)
    out, res = codec.archive_decompress(src, recs, False, None)
    for c, (oo, ol, er) in zip(m, res):
        assert er != 0, c["name"]
    oo, ol, er = res[-1]
    assert er == 0 and out.cpu().numpy()[oo:oo + ol].tobytes() == \
        plain[good["plain_off"]:good["plain_off"] + good["plain_len"]]
