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
