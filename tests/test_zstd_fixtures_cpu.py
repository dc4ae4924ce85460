"""The zstd fixtures of compressed archive batches (tests/golden/make_zstd.py), checked on the CPU
without libzstd: every record's layout (u32 BE uncompressed record length | the index when
indexed | one zstd frame, netidx-archive/src/logfile/reader.rs:453-477, 737-801), the frame
headers (RFC 8878 3.1.1.1), and every batch payload against the oracle's archive decoder. The GPU
decompressor is checked against the same fixtures in tests/test_gpu_zstd.py."""
import json
import os

import numpy as np

import nxo

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    m = json.load(open(os.path.join(G, "zstd_manifest.json")))
    rec = open(os.path.join(G, "zstd_records.bin"), "rb").read()
    plain = open(os.path.join(G, "zstd_plain.bin"), "rb").read()
    d = open(os.path.join(G, "zstd_dict.bin"), "rb").read()
    return m, rec, plain, d


def varint(b, i):
    v, k = 0, 0
    while True:
        v |= (b[i + k] & 0x7F) << (7 * k)
        if b[i + k] < 0x80:
            return v, k + 1
        k += 1


def test_records_layout_and_frame_headers():
    m, rec, plain, d = load()
    assert d[:4] == bytes.fromhex("37a430ec")  # the dictionary magic EC30A437, little-endian
    dict_id = int.from_bytes(d[4:8], "little")
    kinds = set()
    for e in m["records"]:
        r = rec[e["rec_off"]:e["rec_off"] + e["rec_len"]]
        assert int.from_bytes(r[:4], "big") == e["uncomp_len"] == e["index_len"] + e["plain_len"]
        if e["indexed"]:
            v, _ = varint(r, 4)
            assert v == e["index_len"]  # the index's varint prefix is its own length
        f = r[4 + e["index_len"]:]
        assert len(f) == e["frame_len"] and f[:4] == bytes.fromhex("28b52ffd")
        fhd = f[4]
        did_flag = fhd & 3
        if e["dict"]:
            assert did_flag == 3
            assert int.from_bytes(f[5 + (0 if fhd & 0x20 else 1):][:4], "little") == dict_id
        else:
            assert did_flag == 0
        kinds.add(e["kind"])
    assert {"dict_l19", "multiblock_dict", "raw_blocks", "rle", "checksum", "empty",
            "no_content_size", "long_distance"} <= kinds


def test_batch_payloads_decode_with_the_oracle():
    m, rec, plain, d = load()
    n = 0
    for e in m["records"]:
        if not e["batch"]:
            continue
        p = np.frombuffer(plain[e["plain_off"]:e["plain_off"] + e["plain_len"]], np.uint8)
        o, used = nxo.decode_archive(p)
        assert o.s.err_kind == 0 and used == len(p)
        n += 1
    assert n >= 40


def _crafted():
    return json.load(open(os.path.join(G, "zstd_crafted.json")))["cases"]


def test_crafted_tree_descriptions_rejected_on_the_host():
    """the Huffman tree reader shared by the host dictionary parser and the device
    (nxg_zstd.h read_huf_weights) rejects what libzstd rejects -- a weight description that decodes
    to 256 weights (libzstd stops at 255) and one without two weight-1 symbols -- and a dictionary
    built on either fails to load. The fixture's own libzstd verdicts are asserted too; the real
    archive dictionary's tree is the positive control."""
    import ctypes as C
    from netidx_amd.codec import lib
    L = lib()
    L.nxg_debug_huf_weights.restype = C.c_uint32
    L.nxg_debug_huf_weights.argtypes = [C.c_char_p, C.c_uint32, C.POINTER(C.c_uint32)]
    L.nxg_debug_zstd_dict_ok.restype = C.c_bool
    L.nxg_debug_zstd_dict_ok.argtypes = [C.c_char_p, C.c_uint64]
    ns = C.c_uint32(0)
    d = load()[3]
    assert L.nxg_debug_huf_weights(d[8:], len(d) - 8, C.byref(ns)) > 0 and ns.value > 1
    assert L.nxg_debug_zstd_dict_ok(d, len(d))
    seen = 0
    for c in _crafted():
        if c["dict"] is None:
            continue
        db = bytes.fromhex(c["dict"])
        tree = db[8:]
        assert L.nxg_debug_huf_weights(tree, len(tree), C.byref(ns)) == 0, c["name"]
        assert not L.nxg_debug_zstd_dict_ok(db, len(db)), c["name"]
        assert c["libzstd_dict"] in ("rejected", None) and c["libzstd_frame"] in ("rejected", None)
        seen += 1
    assert seen == 2


def test_crafted_256_weight_description_is_what_it_says():
    """The crafted FSE description really decodes to 256 weights whose sum rule holds (the case
    the old bound let through), by the generator's independent restatement."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mzc", os.path.join(G, "make_zstd_crafted.py"))
    mzc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mzc)
    c = [x for x in _crafted() if x["name"] == "huf_256_weights"][0]
    tree = bytes.fromhex(c["dict"])[8:]
    hb = tree[0]
    norm, log, used = mzc.read_ncount(tree[1:1 + hb], 15)
    cells = mzc.build_fse(norm, log)
    w = mzc.fse_weights(tree[1 + used:1 + hb], cells, log, 10**6)
    assert len(w) == 256 and mzc.weights_ok(w)
