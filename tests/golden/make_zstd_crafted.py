#!/usr/bin/env python3
"""Crafted (malformed) zstd inputs for the decompressor's table readers: each one is
rejected by libzstd, and must be rejected by nxg_zstd.h on the host (dictionary entropy tables) and
on the device (a compressed block's literals section).

  huf_256_weights  an FSE-compressed Huffman tree description that decodes to 256 weights before
                   its bitstream ends (libzstd's FSE_decompress stops at 255: `op > omax - 2`);
                   with the implied last weight that would be a 257th weight.
  huf_rank1_zero   direct 4-bit weights [2]: the implied weight is 2, so no symbol has weight 1
                   (HUF_readStats: at least two weight-1 symbols, an even number of them).
  lit4_small       a four-stream Huffman literals section of 5 literals (libzstd 1.5:
                   MIN_LITERALS_FOR_4_STREAMS = 6).

The FSE and Huffman rules restated here are RFC 8878 4.1.1 / 4.2.1 (the same rules as
netidx_amd/csrc/nxg_zstd.h, restated independently in Python). Writes tests/golden/zstd_crafted.json:
per case the bytes (hex) of a zstd frame, and of a dictionary for the host path where the case
is a tree description, with libzstd's verdict when the system libzstd is loadable.

Usage: python tests/golden/make_zstd_crafted.py
"""
import ctypes as C
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))


# ---- FSE table description (RFC 8878 4.1.1), writer and reader -------------------------------
def write_ncount(norm, log):
    """FSE_writeNCount: the normalized counts `norm` (sum 2^log, -1 = low probability)."""
    bits, nbits_total = 0, 0

    def put(v, n):
        nonlocal bits, nbits_total
        bits |= v << nbits_total
        nbits_total += n

    put(log - 5, 4)
    remaining = (1 << log) + 1
    threshold = 1 << log
    nb = log + 1
    sym = 0
    prev0 = False
    while remaining > 1:
        if prev0:
            start = sym
            while sym < len(norm) and norm[sym] == 0:
                sym += 1
            run = sym - start
            while run >= 3:
                put(3, 2)
                run -= 3
            put(run, 2)
        count = norm[sym]
        sym += 1
        mx = (2 * threshold - 1) - remaining
        remaining -= -count if count < 0 else count
        count += 1
        if count >= threshold:
            count += mx
        put(count, nb)
        if count < mx:
            nbits_total -= 1
        prev0 = count == 1
        while remaining < threshold:
            nb -= 1
            threshold >>= 1
    n = (nbits_total + 7) // 8
    return bits.to_bytes(n, "little")


def read_ncount(p, max_sym):
    """FSE_readNCount (the rules of nxg_zstd.h read_ncount): (norm, log, bytes used)."""
    pos = 0

    def peek(k):
        v = int.from_bytes(p[pos >> 3:(pos >> 3) + 5].ljust(5, b"\0"), "little")
        return (v >> (pos & 7)) & ((1 << k) - 1)

    log = peek(4) + 5
    pos += 4
    remaining = (1 << log) + 1
    threshold = 1 << log
    nb = log + 1
    norm = []
    prev0 = False
    while remaining > 1 and len(norm) <= max_sym:
        if prev0:
            n0 = len(norm)
            while peek(2) == 3:
                n0 += 3
                pos += 2
            n0 += peek(2)
            pos += 2
            norm += [0] * (n0 - len(norm))
        mx = (2 * threshold - 1) - remaining
        v = peek(nb)
        if (v & (threshold - 1)) < mx:
            count = v & (threshold - 1)
            pos += nb - 1
        else:
            count = v & (2 * threshold - 1)
            if count >= threshold:
                count -= mx
            pos += nb
        count -= 1
        remaining -= -count if count < 0 else count
        norm.append(count)
        prev0 = count == 0
        while remaining < threshold:
            nb -= 1
            threshold >>= 1
    assert remaining == 1
    return norm, log, (pos + 7) >> 3


def build_fse(norm, log):
    """FSE_buildDTable: cells (symbol, nbits, base)."""
    size = 1 << log
    sym = [0] * size
    high = size - 1
    nxt = []
    for s, c in enumerate(norm):
        if c == -1:
            sym[high] = s
            high -= 1
            nxt.append(1)
        else:
            nxt.append(max(c, 0))
    step = (size >> 1) + (size >> 3) + 3
    pos = 0
    for s, c in enumerate(norm):
        for _ in range(max(c, 0)):
            sym[pos] = s
            pos = (pos + step) & (size - 1)
            while pos > high:
                pos = (pos + step) & (size - 1)
    assert pos == 0
    cells = []
    for u in range(size):
        s = sym[u]
        ns = nxt[s]
        nxt[s] += 1
        nb = log - (ns.bit_length() - 1)
        cells.append((s, nb, (ns << nb) - size))
    return cells


def fse_weights(stream, cells, log, limit):
    """The two-state FSE decode of Huffman weights (HUF_readStats' FSE_decompress), until the
    bitstream is exhausted or `limit` weights are out. Returns the weights."""
    last = stream[-1]
    bp = len(stream) * 8 - 8 + last.bit_length() - 1

    def rd(k):
        nonlocal bp
        if k == 0:
            return 0
        bp -= k
        v = 0
        for i in range(k):
            q = bp + i
            if q >= 0:
                v |= ((stream[q >> 3] >> (q & 7)) & 1) << i
        return v

    s1, s2 = rd(log), rd(log)
    w = []
    while len(w) < limit:
        w.append(cells[s1][0])
        s1 = cells[s1][2] + rd(cells[s1][1])
        if bp < 0:
            w.append(cells[s2][0])
            break
        w.append(cells[s2][0])
        s2 = cells[s2][2] + rd(cells[s2][1])
        if bp < 0:
            w.append(cells[s1][0])
            break
    return w


def weights_ok(w):
    """The weight-sum rule: the implied last weight exists (a power-of-two remainder)."""
    total = sum(1 << (x - 1) for x in w if x)
    if total == 0:
        return False
    mb = total.bit_length()
    rest = (1 << mb) - total
    return mb <= 12 and rest & (rest - 1) == 0


def craft_256():
    """An FSE weight description whose bitstream yields exactly 256 weights (all 0 or 1, the
    weight-sum rule satisfied): symbols 0 and 1 with 16 cells each at accuracy 5, so every state
    update reads one bit and the stream length sets the weight count."""
    norm, log = [16, 16], 5
    desc = write_ncount(norm, log)
    back, _, used = read_ncount(desc, 15)
    assert back[:2] == norm and used == len(desc)
    cells = build_fse(norm, log)
    rng = random.Random(8878)
    for _ in range(20000):
        # 10 bits of initial states + 254 one-bit updates before the stream runs out
        nbits = 10 + 254
        body = [rng.getrandbits(1) for _ in range(nbits)]
        v = sum(b << i for i, b in enumerate(body)) | (1 << nbits)  # the stop bit on top
        stream = v.to_bytes((nbits + 8) // 8, "little")
        w = fse_weights(stream, cells, log, 10**6)
        if len(w) == 256 and weights_ok(w):
            hb = len(desc) + len(stream)
            assert hb < 128
            return bytes([hb]) + desc + stream
    raise RuntimeError("no stream found")


# ---- frames ----------------------------------------------------------------------------------
def frame_with_block(block, content_size):
    """A single-segment frame (content size in 1 byte) holding one compressed, last block."""
    fhd = 0x20  # Single_Segment_flag, FCS field 1 byte
    hdr = (0xFD2FB528).to_bytes(4, "little") + bytes([fhd, content_size])
    bh = (len(block) << 3) | (2 << 1) | 1  # Compressed_Block, Last_Block
    return hdr + bh.to_bytes(3, "little") + block


def lits_compressed(tree, streams_bytes, regen, four):
    """Literals section header type 2 (Compressed_Literals_Block), size format 00 (one stream)
    or 01 (four streams): 10-bit regenerated and compressed sizes, then the tree and streams."""
    payload = tree + streams_bytes
    cs = len(payload)
    sf = 1 if four else 0
    h = 2 | (sf << 2) | (regen << 4) | (cs << 14)
    return h.to_bytes(3, "little") + payload


def dictionary(tree):
    """A zstd dictionary (RFC 8878 5) whose Huffman table is `tree`; the FSE tables that follow
    are never reached (the tree fails first), so they are the predefined-like minimal ones."""
    magic = (0xEC30A437).to_bytes(4, "little")
    dict_id = (0x4E584731).to_bytes(4, "little")
    return magic + dict_id + tree + bytes(64)


def libzstd_verdict(frame, dict_bytes=None):
    try:
        Z = C.CDLL("libzstd.so.1")
    except OSError:
        return None
    Z.ZSTD_isError.argtypes = [C.c_size_t]
    Z.ZSTD_createDCtx.restype = C.c_void_p
    Z.ZSTD_createDDict.restype = C.c_void_p
    Z.ZSTD_createDDict.argtypes = [C.c_void_p, C.c_size_t]
    Z.ZSTD_decompressDCtx.restype = C.c_size_t
    Z.ZSTD_decompressDCtx.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
    out = C.create_string_buffer(4096)
    if dict_bytes is not None:
        db = C.create_string_buffer(dict_bytes, len(dict_bytes))
        dd = Z.ZSTD_createDDict(db, len(dict_bytes))
        return "rejected" if not dd else "accepted"
    dctx = Z.ZSTD_createDCtx()
    r = Z.ZSTD_decompressDCtx(dctx, out, 4096, frame, len(frame))
    return "rejected" if Z.ZSTD_isError(r) else "accepted"


def main():
    cases = []
    t256 = craft_256()
    blk = lits_compressed(t256, bytes(8), 16, False) + b"\x00"  # then 0 sequences
    f = frame_with_block(blk, 16)
    cases.append({"name": "huf_256_weights", "frame": f.hex(), "dict": dictionary(t256).hex(),
                  "libzstd_frame": libzstd_verdict(f),
                  "libzstd_dict": libzstd_verdict(None, dictionary(t256))})
    t_r1 = bytes([128, 0x20])  # one direct weight, 2 (high nibble)
    blk = lits_compressed(t_r1, bytes([0x80, 0x01]), 4, False) + b"\x00"
    f = frame_with_block(blk, 4)
    cases.append({"name": "huf_rank1_zero", "frame": f.hex(), "dict": dictionary(t_r1).hex(),
                  "libzstd_frame": libzstd_verdict(f),
                  "libzstd_dict": libzstd_verdict(None, dictionary(t_r1))})
    # a valid-looking tree (direct weights [1, 1, 1]: the implied weight 1, four 2-bit codes)
    # with a four-stream section of 5 literals: jump table + 4 one-byte streams
    t_ok = bytes([130, 0x11, 0x10])
    streams = bytes([1, 0, 1, 0, 1, 0]) + bytes([0x80, 0x80, 0x80, 0x80])
    blk = lits_compressed(t_ok, streams, 5, True) + b"\x00"
    f = frame_with_block(blk, 5)
    cases.append({"name": "lit4_small", "frame": f.hex(), "dict": None,
                  "libzstd_frame": libzstd_verdict(f), "libzstd_dict": None})
    json.dump({"cases": cases}, open(os.path.join(HERE, "zstd_crafted.json"), "w"), indent=1)
    for c in cases:
        print(c["name"], "libzstd frame:", c["libzstd_frame"], "dict:", c["libzstd_dict"])


if __name__ == "__main__":
    main()
