#!/usr/bin/env python3
"""Generate the committed zstd fixtures for compressed archive batches (tests/golden/zstd_*).

A compressed archive (netidx-archive/src/logfile/reader.rs:737-801, `compress`) stores each batch
record, after its RecordHeader, as
    u32 BE uncompressed record length | the record's index (indexed files; a length-wrapped
    RecordIndex whose varint prefix is its own length) | one zstd frame of the batch,
compressed at level 19 with a dictionary trained over the archive's records
(zstd::dict::from_continuous, max size end / 10; zstd::bulk::Compressor::with_prepared_dictionary)
and read back with zstd::bulk::Decompressor::with_dictionary + decompress_to_buffer
(reader.rs:243-244, 453-477). The reference pins zstd = "0.13" (Cargo.toml:97; libzstd 1.5.x);
the zstd frame format (RFC 8878) is the same in the libzstd 1.4.8 of this image, whose
ZDICT_trainFromBuffer / ZSTD_compress_usingCDict / ZSTD_compress2 make these frames through
ctypes. The frames are the golden vectors of the GPU decompressor: their plain bytes are stored
next to them, and libzstd decompresses every frame back to them before anything is written.

Records:
  * archive batches (the oracle's encoder over netidx_amd.synth.archive_columns) of 1 .. 3000
    items, compressed with a trained dictionary at level 19 (the reference's setting), half of
    them in an indexed file;
  * the same batches without a dictionary at levels 1, 3, 9 and 19, and with a content checksum;
  * frames that stress the format: a batch past 128 KiB (several blocks), incompressible bytes
    (raw blocks), one repeated byte (RLE block), an empty payload, a frame without its content
    size, and a long-distance repeat (matches far back).
Non-batch payloads are marked `batch: false` (decompression-only vectors).

Usage: python tests/golden/make_zstd.py  (rewrites tests/golden/zstd_*.bin and zstd_manifest.json)
"""
import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

Z = C.CDLL("libzstd.so.1")
Z.ZSTD_compressBound.restype = C.c_size_t
Z.ZSTD_compressBound.argtypes = [C.c_size_t]
Z.ZSTD_isError.argtypes = [C.c_size_t]
Z.ZSTD_getErrorName.restype = C.c_char_p
Z.ZSTD_getErrorName.argtypes = [C.c_size_t]
Z.ZDICT_trainFromBuffer.restype = C.c_size_t
Z.ZDICT_trainFromBuffer.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_uint]
Z.ZDICT_isError.argtypes = [C.c_size_t]
Z.ZSTD_createCCtx.restype = C.c_void_p
Z.ZSTD_createDCtx.restype = C.c_void_p
Z.ZSTD_createCDict.restype = C.c_void_p
Z.ZSTD_createCDict.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
Z.ZSTD_createDDict.restype = C.c_void_p
Z.ZSTD_createDDict.argtypes = [C.c_void_p, C.c_size_t]
Z.ZSTD_compress_usingCDict.restype = C.c_size_t
Z.ZSTD_compress_usingCDict.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                       C.c_size_t, C.c_void_p]
Z.ZSTD_compressCCtx.restype = C.c_size_t
Z.ZSTD_compressCCtx.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                C.c_int]
Z.ZSTD_CCtx_setParameter.restype = C.c_size_t
Z.ZSTD_CCtx_setParameter.argtypes = [C.c_void_p, C.c_int, C.c_int]
Z.ZSTD_CCtx_reset.argtypes = [C.c_void_p, C.c_int]
Z.ZSTD_compress2.restype = C.c_size_t
Z.ZSTD_compress2.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
Z.ZSTD_decompress_usingDDict.restype = C.c_size_t
Z.ZSTD_decompress_usingDDict.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                         C.c_size_t, C.c_void_p]
Z.ZSTD_decompressDCtx.restype = C.c_size_t
Z.ZSTD_decompressDCtx.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
Z.ZSTD_compressStream2.restype = C.c_size_t

ZSTD_c_compressionLevel = 100
ZSTD_c_checksumFlag = 201
ZSTD_c_contentSizeFlag = 200
ZSTD_reset_session_and_parameters = 3


def chk(r):
    if Z.ZSTD_isError(r):
        raise RuntimeError(Z.ZSTD_getErrorName(r).decode())
    return r


def compress(data, level=19, cdict=None, checksum=False, content_size=True):
    cctx = Z.ZSTD_createCCtx()
    out = C.create_string_buffer(Z.ZSTD_compressBound(len(data)) + 64)
    src = C.create_string_buffer(bytes(data), len(data))
    if cdict is not None:
        n = chk(Z.ZSTD_compress_usingCDict(cctx, out, len(out), src, len(data), cdict))
    else:
        chk(Z.ZSTD_CCtx_setParameter(cctx, ZSTD_c_compressionLevel, level))
        chk(Z.ZSTD_CCtx_setParameter(cctx, ZSTD_c_checksumFlag, 1 if checksum else 0))
        chk(Z.ZSTD_CCtx_setParameter(cctx, ZSTD_c_contentSizeFlag, 1 if content_size else 0))
        n = chk(Z.ZSTD_compress2(cctx, out, len(out), src, len(data)))
    Z.ZSTD_freeCCtx(C.c_void_p(cctx))
    return out.raw[:n]


def decompress(frame, cap, ddict=None):
    dctx = Z.ZSTD_createDCtx()
    out = C.create_string_buffer(max(cap, 1))
    src = C.create_string_buffer(bytes(frame), len(frame))
    if ddict is not None:
        n = chk(Z.ZSTD_decompress_usingDDict(dctx, out, cap, src, len(frame), ddict))
    else:
        n = chk(Z.ZSTD_decompressDCtx(dctx, out, cap, src, len(frame)))
    Z.ZSTD_freeDCtx(C.c_void_p(dctx))
    return out.raw[:n]


def varint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def index_bytes(ids):
    """RecordIndex { index: Vec<Id> } (logfile/mod.rs): a length-wrapped struct, so the leading
    varint is the whole index's length (reader.rs:459 skips that many bytes)."""
    body = varint(len(ids)) + b"".join(varint(int(i)) for i in ids)
    n = len(body)
    for k in range(1, 4):
        if len(varint(n + k)) == k:
            L = n + k
            break
    return varint(L) + body


def batch(n, seed):
    import nxo
    from netidx_amd import synth
    m = synth.archive_columns(n, seed)
    d = nxo.Decoded(n, len(m.ctag) + 1, 1)
    for name in ("id", "tag", "fixed", "aux"):
        getattr(d, name)[:n] = getattr(m, name)
    d.ctag[:len(m.ctag)] = m.ctag
    d.cfixed[:len(m.ctag)] = m.cfixed
    d.caux[:len(m.ctag)] = m.caux
    d.s.n_rows, d.s.n_children = n, len(m.ctag)
    return nxo.encode_archive(d, m.heap), m.id


def main():
    rng = np.random.default_rng(0x5EED00F5)
    sizes = [1, 2, 7, 40, 150, 400, 900, 1500, 3000]
    batches = [batch(int(sizes[k % len(sizes)]), 0x5EED0100 + k) for k in range(36)]
    # the archive's dictionary, trained over its records (from_continuous: max size end / 10)
    samples = b"".join(b for b, _ in batches)
    lens = (C.c_size_t * len(batches))(*[len(b) for b, _ in batches])
    cap = min(16384, max(1024, len(samples) // 10))
    dbuf = C.create_string_buffer(cap)
    dlen = Z.ZDICT_trainFromBuffer(dbuf, cap, C.create_string_buffer(samples, len(samples)), lens,
                                   len(batches))
    if Z.ZDICT_isError(dlen):
        raise RuntimeError("dictionary training failed")
    dictionary = dbuf.raw[:dlen]
    cdict = Z.ZSTD_createCDict(C.create_string_buffer(dictionary, dlen), dlen, 19)
    ddict = Z.ZSTD_createDDict(C.create_string_buffer(dictionary, dlen), dlen)

    records, plain, manifest = bytearray(), bytearray(), []

    def add(payload, frame, kind, dict_used, is_batch, indexed=False, ids=()):
        got = decompress(frame, len(payload) + 16, ddict if dict_used else None)
        assert got == payload, kind  # libzstd agrees before anything is written
        idx = index_bytes(ids) if indexed else b""
        uncomp = len(idx) + len(payload)  # the uncompressed record's length (reader.rs:746)
        rec = uncomp.to_bytes(4, "big") + idx + frame
        manifest.append({"kind": kind, "rec_off": len(records), "rec_len": len(rec),
                         "plain_off": len(plain), "plain_len": len(payload),
                         "uncomp_len": uncomp, "index_len": len(idx), "indexed": indexed,
                         "dict": dict_used, "batch": is_batch, "frame_len": len(frame)})
        records.extend(rec)
        plain.extend(payload)

    for k, (b, ids) in enumerate(batches):
        add(b, compress(b, cdict=cdict), "dict_l19", True, True, indexed=bool(k % 2), ids=ids[:50])
    for k, lvl in enumerate((1, 3, 9, 19)):
        b, _ = batches[5 + k]
        add(b, compress(b, level=lvl), f"nodict_l{lvl}", False, True)
    b, _ = batches[7]
    add(b, compress(b, level=5, checksum=True), "checksum", False, True)
    add(b, compress(b, level=5, content_size=False), "no_content_size", False, True)
    big, _ = batch(12000, 0x5EED0200)  # past 128 KiB: several blocks
    assert len(big) > 3 * 131072 // 2
    add(big, compress(big, cdict=cdict), "multiblock_dict", True, True)
    add(big, compress(big, level=3), "multiblock_l3", False, True)
    noise = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    add(noise, compress(noise, level=19), "raw_blocks", False, False)
    add(b"\x5a" * 200000, compress(b"\x5a" * 200000, level=3), "rle", False, False)
    add(b"", compress(b"", level=3), "empty", False, False)
    # matches far back: a 40 KB random piece repeated after 60 KB of other bytes
    piece = rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()
    far = piece + rng.integers(0, 256, 60000, dtype=np.uint8).tobytes() + piece + piece[:5000]
    add(far, compress(far, level=19), "long_distance", False, False)

    open(os.path.join(HERE, "zstd_dict.bin"), "wb").write(dictionary)
    open(os.path.join(HERE, "zstd_records.bin"), "wb").write(bytes(records))
    open(os.path.join(HERE, "zstd_plain.bin"), "wb").write(bytes(plain))
    json.dump({"libzstd": int(C.CDLL("libzstd.so.1").ZSTD_versionNumber()),
               "dict_len": len(dictionary), "records": manifest},
              open(os.path.join(HERE, "zstd_manifest.json"), "w"), indent=0)
    print(f"dict {len(dictionary)} B, {len(manifest)} records, {len(records)} B compressed, "
          f"{len(plain)} B plain")


if __name__ == "__main__":
    main()
