// nxg_f64_rec16.h -- From::Update(Id, F64) records of 12..16 bytes (ids of 1..5 varint bytes,
// < 2^35) on the wire, and the record-boundary machinery shared by the homogeneous-f64 decoders
// (nxg_decode_f64_run.hip: length runs; nxg_decode_f64_x.hip: any f64 frame, single pass):
//     varint(L) 04 varint(id) 09 f64be     L = lw(10 + vl(id)) = 11 + vl(id)
// (len_wrapped_encode pack.rs:527-535, derive lib.rs:289-381, Value::encode lib.rs:404-407).
//
// Merge points: the first record at or after a position c lies in [c, c+16); every valid record
// start in that window starts a walk, and the walks are advanced in position order until they
// coincide. The true chain passes through the merge point, which depends only on the bytes, so
// the lane that owns the bytes before c computes the same position.
#pragma once
#include "nxg_device.h"

namespace f64rec16 {

// A frame whose ids count up by one from i0 (a publisher updating all of its values in
// publication order, netidx-core/src/utils.rs:130-134): record j is 12 + #{t in 1..4 :
// i0 + j >= 2^(7t)} bytes long (ids < 2^35), so record k starts at
//     seq_pos(i0, k) = 12 k + sum_t clamp(i0 + k - 2^(7t), 0, k).
// Shared by the sequential-id decoder and encoder; wave-uniform callers keep it in scalar registers.
NXG_DEV uint64_t seq_pos(uint64_t i0, uint64_t k) {
    uint64_t p = 12 * k;
#pragma unroll
    for (uint32_t t = 1; t <= 4; t++) {
        const uint64_t B = 1ull << (7 * t);
        const uint64_t x = i0 + k > B ? i0 + k - B : 0ull;
        p += x < k ? x : k;
    }
    return p;
}

NXG_DEV uint4 ld16r(const uint8_t* __restrict__ p) { return *reinterpret_cast<const uint4*>(p); }
// the bytes of [off, off+16) that lie inside the frame, zero-filled (out of line: rare)
__device__ __attribute__((noinline)) uint4 ld16_tail(const uint8_t* __restrict__ wire,
                                                    uint64_t off, uint64_t W) {
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; k++)
        if (off + k < W) v[k >> 2] |= (uint32_t)wire[off + k] << (8 * (k & 3));
    return make_uint4(v[0], v[1], v[2], v[3]);
}
NXG_DEV uint4 ld16g(const uint8_t* __restrict__ wire, uint64_t off, uint64_t W) {
    if (off + 16 <= W) return ld16r(wire + off);
    return ld16_tail(wire, off, W);
}

// 16 bytes at byte s (0..15) of the 32 bytes d[0..7] (little-endian dwords), no memory access
NXG_DEV void extract16(const uint32_t (&d)[8], uint32_t s, uint32_t& e0, uint32_t& e1,
                       uint32_t& e2, uint32_t& e3) {
    // two levels of selects on the dword offset q = s / 4 (masks, not a dynamic array index,
    // which the compiler would lower to scratch memory)
    const uint32_t r = s & 3u;
    const uint32_t m2 = 0u - ((s >> 3) & 1u), m1 = 0u - ((s >> 2) & 1u);
    uint32_t g[6], f[5];
#pragma unroll
    for (int j = 0; j < 6; j++) g[j] = d[j] ^ ((d[j] ^ d[j + 2]) & m2);
#pragma unroll
    for (int j = 0; j < 5; j++) f[j] = g[j] ^ ((g[j] ^ g[j + 1]) & m1);
    e0 = alignbyte(f[1], f[0], r);
    e1 = alignbyte(f[2], f[1], r);
    e2 = alignbyte(f[3], f[2], r);
    e3 = alignbyte(f[4], f[3], r);
}

// A valid f64 Update record (L in 12..16: 1..5 id bytes) at e0,e1? Returns L or 0.
// rem = bytes from the record start to the frame end.
NXG_DEV uint32_t rec_check16(uint32_t e0, uint32_t e1, uint64_t rem) {
    const uint32_t L = e0 & 0xffu;
    const bool head = (L - 12u <= 4u) && (((e0 >> 8) & 0xffu) == 4u);
    const uint32_t sh = 8u * ((L - 11u) & 7u);  // 8 * nb
    const uint64_t x = ((((uint64_t)e1) << 32) | e0) >> 16;  // bytes 2..7
    const uint64_t m = (1ull << sh) - 1ull;
    const uint64_t want = 0x8080808080ull & (m >> 8);
    const bool var = (x & 0x808080808080ull & m) == want;  // exactly nb varint bytes
    const uint32_t tag = (uint32_t)(x >> sh) & 0xffu;       // Value tag after the id
    return (head && var && tag == 9u && rem >= L) ? L : 0u;
}

// id and f64 bits of a record of length L (12..16) already checked by rec_check16
NXG_DEV void rec_decode16(uint32_t e0, uint32_t e1, uint32_t e2, uint32_t e3, uint32_t L,
                          uint64_t& id, uint64_t& val) {
    const uint32_t sh = 8u * ((L - 11u) & 7u);
    const uint64_t x = ((((uint64_t)e1) << 32) | e0) >> 16;
    const uint64_t y = x & ((1ull << sh) - 1ull) & 0x7f7f7f7f7full;
    id = (y & 0x7full) | ((y >> 1) & 0x3f80ull) | ((y >> 2) & 0x1fc000ull) |
         ((y >> 3) & 0xfe00000ull) | ((y >> 4) & 0x7f0000000ull);
    const uint32_t o = L - 8u;  // value offset, 4..8
    const uint32_t lo = o >= 8u ? e2 : alignbyte(e2, e1, o & 3u);
    const uint32_t hi = o >= 8u ? e3 : alignbyte(e3, e2, o & 3u);
    val = ((uint64_t)bswap32(lo) << 32) | bswap32(hi);  // big-endian f64 (pack.rs:592-598)
}

// SWAR: 0x80 in each byte of x whose value is in [12, 16] (record lengths)
NXG_DEV uint32_t len_bytes(uint32_t x) {
    const uint32_t y = x & 0x7f7f7f7fu;
    return (0x90909090u - y) & ~x & (y + 0x74747474u) & 0x80808080u;
}
// candidate starts in positions 0..15 of d[0..4]: a byte in 12..16 followed by 0x04
NXG_DEV uint32_t cand16(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t d4) {
    const uint32_t a = nib(len_bytes(d0)) | (nib(len_bytes(d1)) << 4) | (nib(len_bytes(d2)) << 8) |
                       (nib(len_bytes(d3)) << 12);
    const uint32_t b = nib(zero_bytes(d0 ^ 0x04040404u)) | (nib(zero_bytes(d1 ^ 0x04040404u)) << 4) |
                       (nib(zero_bytes(d2 ^ 0x04040404u)) << 8) |
                       (nib(zero_bytes(d3 ^ 0x04040404u)) << 12) |
                       (nib(zero_bytes(d4 ^ 0x04040404u)) << 16);
    return a & (b >> 1) & 0xffffu;
}

// 16 bytes at LDS byte offset rel (any alignment)
// LDS images of the wire. LinImg: bytes in order. SwzImg: dword i of the image kept at dword
// i ^ ((i >> 4) & 15), so that 64 lanes reading at 64-byte strides (one chunk each) hit 32
// different banks in pairs instead of two banks 16 deep (ds_read_b32 banks: (a / 4) mod 32,
// MI355X_MICROARCH.md LDS); reads are dword-wise, so any byte offset still works.
struct LinImg {
    const uint8_t* b;
    NXG_DEV uint32_t w(uint32_t i) const { return reinterpret_cast<const uint32_t*>(b)[i]; }
    NXG_DEV uint32_t byte(uint32_t p) const { return b[p]; }
};
struct SwzImg {
    const uint8_t* b;
    static NXG_DEV uint32_t sw(uint32_t i) { return i ^ ((i >> 4) & 15u); }
    NXG_DEV uint32_t w(uint32_t i) const { return reinterpret_cast<const uint32_t*>(b)[sw(i)]; }
    NXG_DEV uint32_t byte(uint32_t p) const { return b[(sw(p >> 2) << 2) | (p & 3u)]; }
};

// 16 bytes at image byte offset rel (any alignment)
template <typename Img>
NXG_DEV void lds16i(const Img& im, uint32_t rel, uint32_t& e0, uint32_t& e1, uint32_t& e2,
                   uint32_t& e3) {
    const uint32_t q = rel >> 2, s = rel & 3u;
    const uint32_t d0 = im.w(q), d1 = im.w(q + 1), d2 = im.w(q + 2), d3 = im.w(q + 3),
                   d4 = im.w(q + 4);
    e0 = alignbyte(d1, d0, s);
    e1 = alignbyte(d2, d1, s);
    e2 = alignbyte(d3, d2, s);
    e3 = alignbyte(d4, d3, s);
}
NXG_DEV void lds16(const uint8_t* buf, uint32_t rel, uint32_t& e0, uint32_t& e1, uint32_t& e2,
                   uint32_t& e3) {
    lds16i(LinImg{buf}, rel, e0, e1, e2, e3);
}

constexpr uint32_t FAILX = 0xffffffffu;
constexpr int WIN = 64;  // merge walks must coincide within 64 bytes of the chunk start

// Merge point of all record walks starting in [r, r+16) of the LDS image (r 4-aligned), as a
// position relative to the image; the END position (W - a0) for a chunk at or past the frame's
// end; FAILX if the walks do not merge.
template <typename Img>
NXG_DEV uint32_t merge16i(const Img& buf, uint32_t r, uint64_t a0, uint64_t W) {
    // positions are signed: an exact tile at the start of a byte range images 64 bytes before it
    const int64_t abs_r = (int64_t)a0 + (int64_t)r;
    if (abs_r >= (int64_t)W) return (uint32_t)((int64_t)W - (int64_t)a0);
    const uint64_t remr = (uint64_t)((int64_t)W - abs_r);
    const uint32_t q = r >> 2;
    uint32_t cand = cand16(buf.w(q), buf.w(q + 1), buf.w(q + 2), buf.w(q + 3), buf.w(q + 4));
    uint64_t S = 0;
    if (remr < 16) S |= 1ull << remr;  // the frame end is a valid (terminal) position
    while (cand) {
        const uint32_t p = __builtin_ctz(cand);
        cand &= cand - 1;
        uint32_t e0, e1, e2, e3;
        lds16i(buf, r + p, e0, e1, e2, e3);
        if (rec_check16(e0, e1, remr - p)) S |= 1ull << p;
    }
    for (int it = 0; it < WIN && __popcll(S) > 1; it++) {
        const uint32_t p = __builtin_ctzll(S);
        S &= S - 1;
        uint32_t e0, e1, e2, e3;
        lds16i(buf, r + p, e0, e1, e2, e3);
        const uint32_t L = rec_check16(e0, e1, remr - p);
        const uint32_t np = p + L;
        if (np >= (uint32_t)WIN) return FAILX;
        bool ok = (np == remr);
        if (!ok) {
            lds16i(buf, r + np, e0, e1, e2, e3);
            ok = rec_check16(e0, e1, remr - np) != 0;
        }
        if (ok) S |= 1ull << np;
    }
    if (__popcll(S) != 1) return FAILX;
    return r + (uint32_t)__builtin_ctzll(S);
}

NXG_DEV uint32_t merge16(const uint8_t* buf, uint32_t r, uint64_t a0, uint64_t W) {
    return merge16i(LinImg{buf}, r, a0, W);
}

// the bytes of the 16 at `pos` (signed, relative to wire) that lie in [-pre, W), zero-filled
__device__ __attribute__((noinline)) uint4 ld16_pre(const uint8_t* __restrict__ wire,
                                                   int64_t pos, uint64_t W, uint64_t pre) {
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int64_t q = pos + k;
        if (q >= -(int64_t)pre && q < (int64_t)W)
            v[k >> 2] |= (uint32_t)wire[q] << (8 * (k & 3));
    }
    return make_uint4(v[0], v[1], v[2], v[3]);
}

// The exact path of the f64 decoders: records counted (and, with EMIT, decoded) by the whole wave
// over 4 KiB sub-tiles whose LDS image holds kXImg bytes: [a0 - 64, a0 + 4096 + 128).
constexpr uint32_t kXSub = 4096;              // bytes per sub-tile
constexpr uint32_t kXHalo = 128;              // look-ahead past the sub-tile
constexpr uint32_t kXLo = 64;                 // image offset of a0
constexpr uint32_t kXHi = kXLo + kXSub;       // image offset of a0 + 4096
constexpr uint32_t kXImg = kXHi + kXHalo;     // image bytes

// Exact path for tile t (T bytes), by the whole wave, in 4 KiB sub-tiles. A sub-tile at a0 owns the
// records that START in [a0, a0 + 4096), like a uniform tile. Its LDS image holds the bytes
// [a0 - 64, a0 + 4096 + kXHalo) (image offset = position - a0 + 64). Lane j walks the chain from
// the merge point of chunk j to that of chunk j + 1; lane 0 starts one chunk earlier (the chunk
// before a0, whose merge point precedes a0: the frame start for a0 = 0), so the walks cover
// every record from before a0 to past a0 + 4096, and each record is counted by exactly one lane.
// Returns (wave-uniform) the record count, the entry (first start - t0), the exit x (first start
// at or past t0 + T, or the frame end, minus t0) and `bad`. With EMIT the records go to rows
// base + index (a rare path: plain stores).
// `pre`: bytes readable before wire[0] (a byte range that does not start the frame)
template <bool EMIT, uint32_t T>
NXG_DEV void exact_tile(const uint8_t* __restrict__ wire, uint64_t W, uint64_t R, bool first,
                        uint64_t pre, uint64_t t, uint8_t* buf, uint32_t lane, uint64_t base,
                        uint64_t* __restrict__ oid, uint64_t* __restrict__ oval, uint64_t cap,
                        uint32_t& count, uint32_t& entry, uint32_t& x, bool& bad, bool& over) {
    const uint64_t t0 = t * T;
    count = 0;
    entry = 0;
    x = 0;
    uint32_t prev_exit = 0;
    for (uint32_t s = 0; s < T / kXSub; s++) {
        const uint64_t a0 = t0 + (uint64_t)s * kXSub;
        if (a0 >= R) break;
        // records that START before the range end are this range's (a range decode: R < W)
        const uint32_t xhi = kXLo + (R - a0 < kXSub ? (uint32_t)(R - a0) : kXSub);
        const uint64_t ib = a0 - kXLo;  // frame position of image byte 0 (wraps for a0 = 0)
        wave_lds_order();
#pragma unroll
        for (uint32_t i = 0; i < (kXImg + 1023) / 1024; i++) {
            const uint32_t off = i * 1024 + lane * 16;
            if (off < kXImg) {
                const int64_t pos = (int64_t)a0 - (int64_t)kXLo + (int64_t)off;
                const uint4 v = pos >= 0 ? ld16g(wire, (uint64_t)pos, W) : ld16_pre(wire, pos, W, pre);
                *reinterpret_cast<uint4*>(buf + off) = v;
            }
        }
        wave_lds_order();
        // segment starts: lane 0 the chunk before a0, lane j >= 1 chunk j; ends: the next lane's
        // start, lane 63 the merge point of the chunk at a0 + 4096
        uint32_t xa;
        if (lane == 0) xa = (a0 == 0 && first) ? kXLo : merge16(buf, 0, ib, W);
        else xa = merge16(buf, kXLo + lane * 64, ib, W);
        uint32_t xb = wave_next(xa);
        if (lane == 63) xb = merge16(buf, kXHi, ib, W);
        bool b = xa == FAILX || xb == FAILX || xa > xb || (lane == 0 && xa > kXLo);
        // walk: count the records that start in [kXLo, xhi); note the first start >= kXLo (lane 0)
        // and the first position >= xhi (the exit)
        uint32_t n = 0, fst = FAILX, ex = FAILX;
        if (!b) {
            uint32_t pos = xa;
            int guard = 0;
            while (pos < xb && guard < 24) {
                if (pos >= kXLo && fst == FAILX) fst = pos;
                if (pos >= xhi) {
                    if (ex == FAILX) ex = pos;
                } else {
                    uint32_t e0, e1, e2, e3;
                    lds16(buf, pos, e0, e1, e2, e3);
                    const uint32_t L = rec_check16(e0, e1, W - (ib + pos));
                    if (!L) break;
                    if (pos >= kXLo) n++;
                    pos += L;
                    guard++;
                    continue;
                }
                // past the sub-tile: step by the length byte only (the next sub-tile checks it)
                const uint32_t L = buf[pos];
                if (L - 12u > 4u) break;
                pos += L;
                guard++;
            }
            b = pos != xb;
            if (pos >= kXLo && fst == FAILX) fst = pos;  // segment end (e.g. the frame end)
            if (pos >= xhi && ex == FAILX) ex = pos;
        }
        if (__any(b)) {
            bad = true;
            return;
        }
        const uint32_t f0 = (uint32_t)__builtin_amdgcn_readlane((int)fst, 0);
        const uint32_t exw = wave_min_u32(ex);
        if (s == 0) entry = f0 - kXLo;
        else if (f0 != prev_exit) {  // the sub-tiles' chains must meet
            bad = true;
            return;
        }
        const uint32_t inc = wave_incl_scan(n);
        if (EMIT) {
            uint64_t row = base + count + (inc - n);
            uint32_t pos = xa;
            while (pos < xb && pos < xhi) {
                uint32_t e0, e1, e2, e3;
                lds16(buf, pos, e0, e1, e2, e3);
                const uint32_t L = e0 & 0xffu;
                if (pos >= kXLo) {
                    uint64_t id, val;
                    rec_decode16(e0, e1, e2, e3, L, id, val);
                    if (row < cap) {
                        oid[row] = id;
                        oval[row] = val;
                    } else {
                        over = true;
                    }
                    row++;
                }
                pos += L;
            }
        }
        count += wave_last(inc);
        // the chain leaves the sub-tile at exw (image offset); the frame end if it ends inside
        const uint32_t endw = W - ib < (uint64_t)kXImg ? (uint32_t)(W - ib) : FAILX;
        const uint32_t xo = exw != FAILX ? exw : endw;
        if (xo == FAILX) {
            bad = true;
            return;
        }
        prev_exit = xo - kXSub;  // the next sub-tile's entry, as an image offset
        if (xhi < kXHi && exw != FAILX) {  // the range ends inside this sub-tile
            x = s * kXSub + (xo - kXLo);
            break;
        }
        x = s * kXSub + (xo - kXLo);
    }
}


}  // namespace f64rec16
