// nxg_zstd.h -- zstd frame decoding (RFC 8878) shared by the host (dictionary parsing) and the
// gfx950 decompressor (nxg_zstd.hip) of compressed archive batches.
//
// The reference reads a compressed archive record with zstd::bulk::Decompressor::with_dictionary
// + decompress_to_buffer (netidx-archive/src/logfile/reader.rs:243-244, 453-477; zstd = "0.13",
// Cargo.toml:97, libzstd 1.5.x). The format restated here:
//   FSE table descriptions and decoding tables        RFC 8878 4.1.1, libzstd FSE_readNCount /
//                                                     FSE_buildDTable
//   Huffman tree descriptions (FSE-compressed or direct 4-bit weights) and decoding tables
//                                                     RFC 8878 4.2.1, HUF_readStats / readDTableX1
//   literals / sequences sections, repeat offsets     RFC 8878 3.1.1.3, 3.1.1.5
//   dictionaries (entropy tables, repeat offsets, content)  RFC 8878 5
// Functions here are pure (no memory outside their arguments) so that the host parses a
// dictionary with exactly the code the device uses per block.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define NXZ_HD __host__ __device__ inline
#else
#define NXZ_HD inline
#endif

namespace nxz {

constexpr uint32_t kFrameMagic = 0xFD2FB528u;
constexpr uint32_t kDictMagic = 0xEC30A437u;
constexpr uint32_t kBlockMax = 128u * 1024u;
constexpr int kLLMax = 35, kMLMax = 52, kOFMax = 31;  // largest codes
constexpr int kLLLog = 9, kMLLog = 9, kOFLog = 8;      // largest table accuracy logs
constexpr int kHufMaxBits = 12;  // HUF_TABLELOG_MAX (libzstd); encoders use 11

// errors (NxgArchiveRecord.err)
enum : uint32_t {
    Z_OK = 0,
    Z_PREFIX = 1,      // not a zstd frame (magic), or a reserved bit set
    Z_CORRUPT = 2,     // malformed block / table / bitstream
    Z_DST_SMALL = 3,   // output larger than the record's uncompressed length
    Z_DICT = 4,        // dictionary missing or of another id
    Z_CHECKSUM = 5,    // content checksum mismatch
    Z_FRAME_SIZE = 6,  // frame content size differs from the output
    Z_SRC = 7,         // record shorter than its headers
};

// a decoding-table cell: symbol, bits to read, next-state baseline
struct FseCell {
    uint16_t base;
    uint8_t sym;
    uint8_t nbits;
};
struct HufCell {
    uint8_t sym;
    uint8_t nbits;
};

NXZ_HD uint32_t highbit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// LSB-first reader over [p, p + n) (table descriptions); bits past the end read as 0
struct FwdBits {
    const uint8_t* p;
    uint32_t n;
    uint32_t pos = 0;  // bit position
    NXZ_HD FwdBits(const uint8_t* p_, uint32_t n_) : p(p_), n(n_) {}
    NXZ_HD uint32_t peek(uint32_t k) const {  // k <= 24
        uint64_t v = 0;
        const uint32_t b = pos >> 3;
        for (uint32_t i = 0; i < 5; i++)
            if (b + i < n) v |= (uint64_t)p[b + i] << (8 * i);
        return (uint32_t)(v >> (pos & 7)) & ((1u << k) - 1u);
    }
    NXZ_HD void skip(uint32_t k) { pos += k; }
};

// FSE_readNCount: the normalized counts of a table description; returns the bytes used (0 on
// error), *al the accuracy log, *max_sym the last symbol.
NXZ_HD uint32_t read_ncount(const uint8_t* p, uint32_t n, int16_t* norm, uint32_t max_sym_allowed,
                            uint32_t max_log, uint32_t* al, uint32_t* max_sym) {
    if (n < 1) return 0;
    FwdBits in(p, n);
    const uint32_t log = in.peek(4) + 5;
    in.skip(4);
    if (log > max_log) return 0;
    int remaining = (1 << log) + 1;
    int threshold = 1 << log;
    uint32_t nb = log + 1;
    uint32_t sym = 0;
    bool prev0 = false;
    while (remaining > 1 && sym <= max_sym_allowed) {
        if (prev0) {
            uint32_t n0 = sym;
            while (in.peek(2) == 3) {
                n0 += 3;
                in.skip(2);
                if (n0 > max_sym_allowed + 1) return 0;
            }
            n0 += in.peek(2);
            in.skip(2);
            if (n0 > max_sym_allowed + 1) return 0;
            while (sym < n0) norm[sym++] = 0;
            if (sym > max_sym_allowed) break;
        }
        const int max = (2 * threshold - 1) - remaining;
        const uint32_t v = in.peek(nb);
        int count;
        if ((int)(v & (uint32_t)(threshold - 1)) < max) {
            count = (int)(v & (uint32_t)(threshold - 1));
            in.skip(nb - 1);
        } else {
            count = (int)(v & (uint32_t)(2 * threshold - 1));
            if (count >= threshold) count -= max;
            in.skip(nb);
        }
        count--;  // -1: a "less than one" probability
        remaining -= count < 0 ? -count : count;
        norm[sym++] = (int16_t)count;
        prev0 = count == 0;
        while (remaining < threshold) {
            nb--;
            threshold >>= 1;
        }
    }
    if (remaining != 1 || sym == 0) return 0;
    const uint32_t used = (in.pos + 7) >> 3;
    if (used > n) return 0;
    for (uint32_t s = sym; s <= max_sym_allowed; s++) norm[s] = 0;
    *al = log;
    *max_sym = sym - 1;
    return used;
}

// FSE_buildDTable: `tab` has 1 << al cells. `scratch` holds max_sym + 1 u16. False on a
// malformed distribution.
NXZ_HD bool build_fse(FseCell* tab, const int16_t* norm, uint32_t max_sym, uint32_t al,
                      uint16_t* next) {
    const uint32_t size = 1u << al;
    uint32_t high = size - 1;
    for (uint32_t s = 0; s <= max_sym; s++) {
        if (norm[s] == -1) {
            tab[high--].sym = (uint8_t)s;
            next[s] = 1;
        } else {
            next[s] = (uint16_t)(norm[s] > 0 ? norm[s] : 0);
        }
    }
    const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= max_sym; s++)
        for (int i = 0; i < norm[s]; i++) {
            tab[pos].sym = (uint8_t)s;
            do {
                pos = (pos + step) & mask;
            } while (pos > high);
        }
    if (pos != 0) return false;
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t s = tab[u].sym;
        const uint32_t ns = next[s]++;
        if (ns == 0) return false;
        const uint32_t nb = al - highbit(ns);
        tab[u].nbits = (uint8_t)nb;
        tab[u].base = (uint16_t)((ns << nb) - size);
    }
    return true;
}

// a table of one symbol (RLE mode): accuracy 0
NXZ_HD void build_rle(FseCell* tab, uint32_t sym) {
    tab[0].sym = (uint8_t)sym;
    tab[0].nbits = 0;
    tab[0].base = 0;
}

// predefined distributions (RFC 8878 3.1.1.3.2.2)
constexpr int16_t kLLDefault[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                    2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kMLDefault[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kOFDefault[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                    1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// code -> (baseline, extra bits) (RFC 8878 3.1.1.3.2.1.1)
NXZ_HD uint32_t ll_base(uint32_t c) {
    constexpr uint32_t b[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,    10,   11,
                                12, 13, 14, 15, 16, 18, 20,  22,  24,  28,   32,   40,
                                48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
    return b[c];
}
NXZ_HD uint32_t ll_bits(uint32_t c) {
    constexpr uint8_t b[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                               1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
    return b[c];
}
NXZ_HD uint32_t ml_base(uint32_t c) {
    constexpr uint32_t b[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16,
                                17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30,
                                31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51, 59, 67, 83,
                                99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
    return b[c];
}
NXZ_HD uint32_t ml_bits(uint32_t c) {
    constexpr uint8_t b[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                               0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                               2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
    return b[c];
}

// Huffman weights (HUF_readStats): `w` receives up to 256 weights; returns the bytes used (0 on
// error), *n_sym the symbols (the last weight included), *max_bits the longest code.
// `fse`: 64 cells of scratch, `norm`/`next`: 16 entries each.
NXZ_HD uint32_t read_huf_weights(const uint8_t* p, uint32_t n, uint8_t* w, uint32_t* n_sym,
                                 uint32_t* max_bits, FseCell* fse, int16_t* norm,
                                 uint16_t* next) {
    if (n < 1) return 0;
    const uint32_t hb = p[0];
    uint32_t nw = 0, used;
    if (hb >= 128) {  // direct: hb - 127 weights, 4 bits each, high nibble first
        nw = hb - 127;
        used = 1 + (nw + 1) / 2;
        if (used > n) return 0;
        for (uint32_t i = 0; i < nw; i++) {
            const uint32_t b = p[1 + i / 2];
            w[i] = (uint8_t)((i & 1) ? (b & 15) : (b >> 4));
        }
    } else {  // FSE-compressed weights: hb bytes, two interleaved states
        used = 1 + hb;
        if (used > n || hb == 0) return 0;
        uint32_t al, ms;
        const uint32_t tb = read_ncount(p + 1, hb, norm, 15, 6, &al, &ms);
        if (!tb || !build_fse(fse, norm, ms, al, next)) return 0;
        const uint8_t* s = p + 1 + tb;
        const uint32_t sn = hb - tb;
        if (sn == 0 || s[sn - 1] == 0) return 0;
        int64_t bp = (int64_t)sn * 8 - 8 + (int64_t)highbit(s[sn - 1]);  // unread bits below
        auto rd = [&](uint32_t k) -> uint32_t {
            if (k == 0) return 0;
            bp -= k;
            uint64_t v = 0;
            const int64_t lo = bp;
            for (uint32_t i = 0; i < k; i++) {
                const int64_t q = lo + i;
                if (q >= 0) v |= (uint64_t)((s[q >> 3] >> (q & 7)) & 1u) << i;
            }
            return (uint32_t)v;
        };
        uint32_t s1 = rd(al), s2 = rd(al);
        // FSE_decompress into 255 weights: libzstd fails a write past index 253 (`op > omax - 2`,
        // each write may be followed by the other state's final one), so at most 255 are decoded
        for (;;) {
            if (nw > 253) return 0;
            w[nw++] = fse[s1].sym;
            s1 = fse[s1].base + rd(fse[s1].nbits);
            if (bp < 0) {
                w[nw++] = fse[s2].sym;
                break;
            }
            if (nw > 253) return 0;
            w[nw++] = fse[s2].sym;
            s2 = fse[s2].base + rd(fse[s2].nbits);
            if (bp < 0) {
                w[nw++] = fse[s1].sym;
                break;
            }
        }
    }
    // the last weight is implied: the weights' sum must reach the next power of two
    uint32_t total = 0;
    for (uint32_t i = 0; i < nw; i++) {
        if (w[i] > kHufMaxBits) return 0;
        if (w[i]) total += 1u << (w[i] - 1);
    }
    if (total == 0) return 0;
    const uint32_t mb = highbit(total) + 1;
    if (mb > kHufMaxBits) return 0;
    const uint32_t rest = (1u << mb) - total;
    if (rest & (rest - 1)) return 0;  // not a power of two
    if (nw >= 256) return 0;          // no room for the implied weight (w holds 256)
    w[nw++] = (uint8_t)(highbit(rest) + 1);
    // HUF_readStats' tree check: at least two weight-1 symbols, an even number of them
    uint32_t r1 = 0;
    for (uint32_t i = 0; i < nw; i++) r1 += w[i] == 1;
    if (r1 < 2 || (r1 & 1)) return 0;
    *n_sym = nw;
    *max_bits = mb;
    return used;
}

// HUF_readDTableX1: 1 << max_bits cells; symbols of weight w take 2^(w-1) cells, weights in
// increasing order, symbols in order within a weight
NXZ_HD void build_huf(HufCell* tab, const uint8_t* w, uint32_t n_sym, uint32_t max_bits) {
    uint32_t start[kHufMaxBits + 2] = {0};
    uint32_t cnt[kHufMaxBits + 2] = {0};
    for (uint32_t s = 0; s < n_sym; s++) cnt[w[s]]++;
    uint32_t acc = 0;
    for (uint32_t k = 1; k <= max_bits; k++) {
        start[k] = acc;
        acc += cnt[k] << (k - 1);
    }
    for (uint32_t s = 0; s < n_sym; s++) {
        const uint32_t k = w[s];
        if (!k) continue;
        const uint32_t len = 1u << (k - 1);
        const uint8_t nb = (uint8_t)(max_bits + 1 - k);
        for (uint32_t i = 0; i < len; i++) tab[start[k] + i] = HufCell{(uint8_t)s, nb};
        start[k] += len;
    }
}

}  // namespace nxz
