// nxg_fmx_common.h -- device code shared by the fast mixed decoder (nxg_decode_mixed.hip) and the
// fast archive-batch decoder (nxg_archive_fast.hip): 4 KiB tile images in LDS and the
// branch-light value decoder with its text (UTF-8) checks. Included by one .hip file each; not ABI.
#pragma once
#include "nxg_internal.h"
#include "nxg_msg.h"

namespace fmx {
#ifndef NXG_COL_NT
#define NXG_COL_NT 1  // column stores of the emit passes nontemporal (rows are not read again here)
#endif
template <typename T>
NXG_DEV void col_st(T* p, T v) {
    if (NXG_COL_NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
constexpr uint32_t TILE = 4096;
constexpr uint32_t CH = 64;
constexpr uint32_t IMG = TILE + 256;    // image: the tile + 256 B
constexpr uint32_t MAXM = TILE / 4;     // messages (items) per tile in the emit pass's list
constexpr uint32_t MAXC = 256;          // array elements per round of 64 messages (lane-parallel)
constexpr int TPB = 256;
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t FAIL = 0xfffffffeu;
}  // namespace fmx

namespace {
using namespace fmx;
using namespace nxgmsg;

NXG_DEV uint4 ld16(const uint8_t* __restrict__ wire, uint64_t off, uint64_t W) {
    if (off + 16 <= W) return *reinterpret_cast<const uint4*>(wire + off);
    uint32_t q[4] = {0, 0, 0, 0};
    for (int k = 0; k < 16; k++)
        if (off + k < W) q[k >> 2] |= (uint32_t)wire[off + k] << (8 * (k & 3));
    return make_uint4(q[0], q[1], q[2], q[3]);
}

// the tile's image: 4 KiB from 64 lanes x 4, the 256-byte tail from lanes 0..15 (zeros past W),
// loaded into registers (tile_load, one tile ahead) and then written to LDS (tile_store)
struct TileRegs {
    uint4 v[5];
};
NXG_DEV void tile_load(TileRegs& g, const uint8_t* __restrict__ wire, uint64_t t0, uint64_t W,
                       uint32_t lane) {
    if (t0 + IMG <= W) {
        const uint4* p = reinterpret_cast<const uint4*>(wire + t0);
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) g.v[i] = p[i * 64 + lane];
        if (lane < 16) g.v[4] = p[256 + lane];
    } else {
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) g.v[i] = ld16(wire, t0 + i * 1024 + lane * 16, W);
        if (lane < 16) g.v[4] = ld16(wire, t0 + 4096 + lane * 16, W);
    }
}
NXG_DEV void tile_store(uint8_t* img, const TileRegs& g, uint32_t lane) {
    wave_lds_order();  // the previous tile's reads are issued
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) *reinterpret_cast<uint4*>(img + i * 1024 + lane * 16) = g.v[i];
    if (lane < 16) *reinterpret_cast<uint4*>(img + 4096 + lane * 16) = g.v[4];
    wave_lds_order();
}

// contiguous tile ranges per wave: tiles [run_begin(r), run_begin(r + 1)) of R
NXG_DEV uint64_t run_begin(uint64_t nt, uint32_t R, uint32_t r) { return nt * r / R; }

// image bytes r..r+15 as two little-endian words (reads up to 20 bytes from r & ~3)
struct Win16 {
    uint64_t lo, hi;
};
NXG_DEV Win16 win16(lds_bytes img, uint32_t r) {
    lds_words w = (lds_words)(img + (r & ~3u));
    const uint32_t sh = r & 3u;
    const uint32_t a0 = w[0], a1 = w[1], a2 = w[2], a3 = w[3], a4 = w[4];
    return Win16{(uint64_t)alignbyte(a1, a0, sh) | ((uint64_t)alignbyte(a2, a1, sh) << 32),
                 (uint64_t)alignbyte(a3, a2, sh) | ((uint64_t)alignbyte(a4, a3, sh) << 32)};
}

// ---- the emit pass's value decoder ---------------------------------------------------------------
// Value::decode (netidx-value/src/lib.rs:470-506) for the values this path takes, restated as
// nxg_msg.h dleaf / dcontainer do. Every field is computed from the 12 bytes after the tag (three
// words already in registers) with 32-bit tile offsets, and selected by tag, so that a wave whose
// lanes hold different tags runs one instruction stream; only a varint longer than 4 bytes and a
// DateTime outside +-2^42 s or with a leap second branch. Text is checked for UTF-8 by the caller
// (ascii_ok per lane, utf8_wave for the rest). Any decode error clears ok: the frame then goes to
// the general decoder, which reports it.

// the 7-bit groups of the (up to) 8 bytes of y, least significant first
NXG_DEV uint64_t compress7(uint64_t y) {
    const uint64_t z1 = (y & 0x007f007f007f007full) | ((y >> 1) & 0x3f803f803f803f80ull);
    const uint64_t z2 = (z1 & 0x00003fff00003fffull) | ((z1 >> 2) & 0x0fffc0000fffc000ull);
    return (z2 & 0x0fffffffull) | ((z2 >> 4) & 0x00fffffff0000000ull);
}
NXG_DEV uint32_t compress7_32(uint32_t y) {
    return (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
}

// LEB128 (pack.rs:504-520) at window byte 0: its length (0: no terminator in 10 bytes); bits
// past 64 dropped as decode_varint does
NXG_DEV uint32_t wvar(uint64_t lo, uint64_t hi, uint64_t& v) {
    const uint64_t stop = ~lo & 0x8080808080808080ull;
    if (stop) {
        const uint32_t nb = ((uint32_t)__builtin_ctzll(stop) >> 3) + 1;
        v = compress7(nb == 8 ? lo : (lo & ((1ull << (8 * nb)) - 1)));
        return nb;
    }
    const uint64_t b8 = hi & 0xffu, b9 = (hi >> 8) & 0xffu;
    const uint64_t base = compress7(lo);
    if (b8 < 0x80u) {
        v = base | (b8 << 56);
        return 9;
    }
    v = base | ((b8 & 0x7fu) << 56) | ((b9 & 1u) << 63);
    return b9 < 0x80u ? 10u : 0u;
}
// the same over the words w0, w1, w2 (bytes 0..11): one to four bytes without a branch
NXG_DEV uint32_t var3(uint32_t w0, uint32_t w1, uint32_t w2, uint64_t& v) {
    const uint32_t st = ~w0 & 0x80808080u;
    if (__builtin_expect(st != 0u, 1)) {
        const uint32_t nb = ((uint32_t)__builtin_ctz(st) >> 3) + 1;
        v = compress7_32(w0 & (0xffffffffu >> (32u - 8u * nb)));
        return nb;
    }
    return wvar((uint64_t)w0 | ((uint64_t)w1 << 32), w2, v);
}

// image bytes r .. r+4n-1 as n little-endian words (reads n+1 aligned words from r & ~3)
template <int N>
NXG_DEV void win_words(lds_bytes img, uint32_t r, uint32_t* q) {
    lds_words w = (lds_words)(img + (r & ~3u));
    const uint32_t sh = r & 3u;
    uint32_t a[N + 1];
#pragma unroll
    for (int k = 0; k <= N; k++) a[k] = w[k];
#pragma unroll
    for (int k = 0; k < N; k++) q[k] = alignbyte(a[k + 1], a[k], sh);
}

struct FV {
    uint64_t fixed;
    uint32_t tag, aux;
    uint32_t end;         // tile offset after the value
    uint32_t kids;        // Array: element count
    uint32_t soff, slen;  // text to check for UTF-8 (slen 0: none)
    bool ok;
};

// The value with tag t whose payload starts at tile offset u; P0..P2 = its first 12 bytes; lim =
// the message end (tile offset, >= u). Arrays only when `arr` (a row).
// value classes as tag bit sets (bit tests, so that the compiler forms no switch on the tag)
constexpr uint32_t B(uint32_t t) { return 1u << t; }
constexpr uint32_t kVarTags = B(1) | B(3) | B(5) | B(7);    // V32 Z32 V64 Z64
constexpr uint32_t kVar32 = B(1) | B(3), kZig = B(3) | B(7);
constexpr uint32_t kTxtTags = B(12) | B(13) | B(18) | B(22);  // String Bytes Error(String)
constexpr uint32_t kSgnTags = B(2) | B(24) | B(26);         // I32 I8 I16
NXG_DEV FV val_decode(uint32_t t, uint32_t P0, uint32_t P1, uint32_t P2, uint32_t u, uint32_t lim,
                      bool arr, uint64_t t0) {
    const uint32_t bit = t < 32u ? 1u << t : 0u;
    // Error(Value) whose inner value is a String: the String after its tag (12)
    const bool e22 = bit & B(22);
    const bool bad = t >= 28u || (bit & B(21)) || ((bit & B(19)) && !arr) ||
                     (e22 && (P0 & 0xffu) != 12u);
    P0 = e22 ? alignbyte(P1, P0, 1) : P0;
    P1 = e22 ? alignbyte(P2, P1, 1) : P1;
    P2 = e22 ? P2 >> 8 : P2;
    u += e22 ? 1u : 0u;
    const uint32_t room = lim > u ? lim - u : 0u;
    uint64_t v;
    const uint32_t nb = var3(P0, P1, P2, v);
    const bool vok = nb != 0 && nb <= room;
    const uint32_t p = u + nb;  // after a length / count varint
    const uint32_t rest = lim > p ? lim - p : 0u;
    const uint32_t v32 = (uint32_t)v;
    // fixed-size payloads: n big-endian bytes (0: Bool / Null; 12: DateTime, Duration)
    const uint32_t f1 = fixed_size1(t);
    const uint32_t n = f1 - 1u;
    const uint32_t b0 = bswap32(P0), b1 = bswap32(P1);
    const bool n8 = f1 >= 9u;                       // 8 or 12 bytes
    const uint32_t sh = (32u - 8u * n) & 31u;       // 1, 2, 4 bytes: b0 >> 24, 16, 0
    const bool sgn = bit & kSgnTags;
    const uint32_t lo32 = f1 >= 2u ? (sgn ? (uint32_t)((int32_t)b0 >> sh) : b0 >> sh)
                                   : ((bit & B(14)) ? 1u : 0u);
    const uint32_t fhi = n8 ? b0 : (sgn ? (uint32_t)((int32_t)lo32 >> 31) : 0u);
    const uint32_t flo = n8 ? b1 : lo32;
    // DateTime::from_timestamp: |secs| < 2^42 with ns < 10^9 is always valid (no branch)
    uint32_t ns = bswap32(P2);
    const uint64_t secs = ((uint64_t)b0 << 32) | b1;
    bool fok = room >= n;
    const bool easy = ns < 1000000000u && secs + ((1ull << 42) - 1) < (1ull << 43) - 1;
    if (__builtin_expect((bit & B(10)) && !easy, 0)) fok = fok && datetime_valid((int64_t)secs, ns);
    // Duration::new normalisation (dleaf case 11); ns < 2^32 < 5 * 10^9
    const bool dur = bit & B(11);
    const uint32_t add = dur ? (uint32_t)(ns >= 1000000000u) + (ns >= 2000000000u) +
                                   (ns >= 3000000000u) + (ns >= 4000000000u)
                             : 0u;
    const uint64_t s2 = secs + add;
    fok = fok && s2 >= secs;
    ns -= add * 1000000000u;
    // varint scalars: V32 (truncated), Z32, V64, Z64
    const uint32_t z32 = (v32 >> 1) ^ (0u - (v32 & 1u));
    const uint64_t z64 = (v >> 1) ^ (0ull - (v & 1ull));
    const bool isvar = bit & kVarTags, iszig = bit & kZig, is32 = bit & kVar32;
    const uint64_t v32x = iszig ? (uint64_t)(int64_t)(int32_t)z32 : (uint64_t)v32;
    const uint64_t vfix = is32 ? v32x : (iszig ? z64 : v);
    const bool istxt = bit & kTxtTags, isarr = bit & B(19), isdec = bit & B(20);
    const bool isfix = f1 != 0u;
    // Abstract: len-wrapped (dleaf case 27); the wrap may claim past the message
    const uint64_t take = v >= 1 ? v - vl64(v) : 0ull;
    const uint32_t l2 = take < (uint64_t)rest ? p + (uint32_t)take : lim;
    // ValArray header (array.rs:595-612): count guard as dcontainer
    const bool aok = vok && v <= kMaxVec / 16 && v * 16 <= ((uint64_t)rest << 8);
    const bool tok = vok && v <= (uint64_t)(room - nb);
    const bool bok = vok && v >= 1 && l2 >= p + 16u;
    const bool ok = isfix ? fok : (isvar ? vok : (istxt ? tok : (isarr ? aok : (isdec ? room >= 16u : bok))));
    FV o;
    o.tag = (bit & B(17)) ? 16u : (e22 ? 18u : t);
    o.ok = ok && !bad;
    const uint32_t endv = isvar || isarr ? p : (istxt ? p + v32 : (isdec ? u + 16u : l2));
    o.end = isfix ? u + n : endv;
    const uint64_t off = t0 + (isdec ? u : p);  // text, Decimal, Abstract: where in the frame
    const uint64_t fval = dur ? s2 : (((uint64_t)fhi << 32) | flo);
    o.fixed = isfix ? fval : (isvar ? vfix : (isarr ? 0ull : off));
    const uint32_t avar = istxt || isarr ? v32 : (isdec ? 16u : (isvar ? 0u : l2 - p));
    o.aux = isfix ? (n == 12u ? ns : 0u) : avar;
    o.kids = isarr ? v32 : 0u;
    o.soff = p;
    o.slen = o.ok && istxt && !(bit & B(13)) ? v32 : 0u;
    return o;
}

// val_decode for a round's row values when each lane's tag is in one of the common classes -- a
// fixed-size scalar (F), DateTime / Duration (D), String / Bytes / Error(String) (S), Array (A):
// each class's fields are computed only when the round holds that class (wave-uniform tests), so a
// round pays for the classes present instead of every field of every tag. The same results as
// val_decode(t, P0, P1, P2, u, lim, true, t0) for those tags (the same rules, restated per class:
// dleaf / dcontainer in nxg_msg.h, netidx-value/src/lib.rs:470-506). Returns false (uniform) when
// some lane holds another tag: the caller then runs val_decode.
NXG_DEV bool row_value_cls(uint32_t t, uint32_t P0, uint32_t P1, uint32_t P2, uint32_t u,
                           uint32_t lim, uint64_t t0, bool has, FV& o) {
    const uint32_t f1 = fixed_size1(t);
    const bool isD = t == 10u || t == 11u;
    const bool isF = f1 != 0u && !isD;
    const bool isS = t == 12u || t == 13u || t == 18u;
    const bool isA = t == 19u;
    if (__any(has && !(isF || isD || isS || isA))) return false;
    const uint32_t room = lim > u ? lim - u : 0u;
    const uint32_t b0 = bswap32(P0), b1 = bswap32(P1);
    const uint32_t bit = 1u << (t & 31u);
    {  // F (every lane: the cheapest class, and the default)
        const uint32_t n = f1 - 1u;
        const bool n8 = f1 == 9u;
        const uint32_t sh = (32u - 8u * n) & 31u;
        const bool sgn = bit & kSgnTags;
        const uint32_t lo32 = f1 >= 2u ? (sgn ? (uint32_t)((int32_t)b0 >> sh) : b0 >> sh)
                                       : ((bit & B(14)) ? 1u : 0u);
        const uint32_t fhi = n8 ? b0 : (sgn ? (uint32_t)((int32_t)lo32 >> 31) : 0u);
        o.fixed = ((uint64_t)fhi << 32) | (n8 ? b1 : lo32);
        o.tag = t == 17u ? 16u : t;
        o.aux = 0;
        o.end = u + n;
        o.kids = 0;
        o.soff = 0;
        o.slen = 0;
        o.ok = room >= n;
    }
    if (__any(isD)) {  // DateTime (from_timestamp validity), Duration (Duration::new normalisation)
        uint32_t ns = bswap32(P2);
        const uint64_t secs = ((uint64_t)b0 << 32) | b1;
        bool fok = room >= 12u;
        const bool easy = ns < 1000000000u && secs + ((1ull << 42) - 1) < (1ull << 43) - 1;
        if (__builtin_expect(t == 10u && !easy, 0)) fok = fok && datetime_valid((int64_t)secs, ns);
        const bool dur = t == 11u;
        const uint32_t add = dur ? (uint32_t)(ns >= 1000000000u) + (ns >= 2000000000u) +
                                       (ns >= 3000000000u) + (ns >= 4000000000u)
                                 : 0u;
        const uint64_t s2 = secs + add;
        fok = fok && s2 >= secs;
        ns -= add * 1000000000u;
        if (isD) {
            o.fixed = dur ? s2 : secs;
            o.aux = ns;
            o.end = u + 12u;
            o.ok = fok;
        }
    }
    if (__any(isS || isA)) {  // a length / count varint
        uint64_t v;
        const uint32_t nb = var3(P0, P1, P2, v);
        const bool vok = nb != 0 && nb <= room;
        const uint32_t p = u + nb;
        const uint32_t rest = lim > p ? lim - p : 0u;
        const uint32_t v32 = (uint32_t)v;
        if (isS) {
            const bool tok = vok && v <= (uint64_t)(room - nb);
            o.fixed = t0 + p;
            o.aux = v32;
            o.end = p + v32;
            o.soff = p;
            o.slen = tok && t != 13u ? v32 : 0u;
            o.ok = tok;
        } else if (isA) {
            o.fixed = 0;
            o.aux = v32;
            o.kids = v32;
            o.end = p;
            o.soff = p;
            o.ok = vok && v <= kMaxVec / 16 && v * 16 <= ((uint64_t)rest << 8);
        }
    }
    return true;
}

// index of the first byte >= 0x80 among bytes 0..15 of the words q[0..3] (16: none)
NXG_DEV uint32_t first_high16(const uint32_t* q) {
    const uint64_t lo = (((uint64_t)q[1] << 32) | q[0]) & 0x8080808080808080ull;
    const uint64_t hi = (((uint64_t)q[3] << 32) | q[2]) & 0x8080808080808080ull;
    return lo ? (uint32_t)__builtin_ctzll(lo) >> 3 : (hi ? 8u + ((uint32_t)__builtin_ctzll(hi) >> 3) : 16u);
}
// bytes [s, s + n) of the image are all ASCII: 32 bytes from one batch of LDS reads, longer text
// (up to 127 bytes) 32 more per step
NXG_DEV bool ascii_ok(lds_bytes img, uint32_t s, uint32_t n) {
    bool na = false;
#pragma unroll 1
    for (uint32_t k = 0; k < n; k += 32) {
        uint32_t q[8];
        win_words<8>(img, s + k, q);
        const uint32_t f0 = first_high16(q), f1 = first_high16(q + 4);  // 16: none
        na |= (f0 < 16u ? f0 : (f1 < 16u ? 16u + f1 : 0xffffu)) < n - k;
    }
    return !na;
}

// inclusive max-scan over the wave (DPP, identity 0)
NXG_DEV uint32_t wave_max_scan(uint32_t x) {
    x = max(x, dpp0<0x111, 0xf>(x));
    x = max(x, dpp0<0x112, 0xf>(x));
    x = max(x, dpp0<0x114, 0xf>(x));
    x = max(x, dpp0<0x118, 0xf>(x));
    x = max(x, dpp0<0x142, 0xa>(x));
    x = max(x, dpp0<0x143, 0xc>(x));
    return x;
}

// std::str::from_utf8 (pack.rs:462) of bytes [s, s + n) of the image (s >= 3), checked by the
// whole wave one byte per lane: a continuation byte exactly where a lead within the three bytes
// before asks for one, no C0 / C1 / F5..FF, no overlong 3- or 4-byte form, surrogate or code
// point past U+10FFFF (the byte after E0 / ED / F0 / F4), and every sequence ends inside the text.
// All 64 lanes must be active.
NXG_DEV bool utf8_wave(lds_bytes img, uint32_t s, uint32_t n, uint32_t lane) {
    bool bad = false;
#pragma unroll 1
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + lane;
        if (i < n) {
            const uint32_t r = s + i - 3;
            lds_words w = (lds_words)(img + (r & ~3u));
            const uint32_t x = alignbyte(w[1], w[0], r & 3u);  // bytes i-3 .. i
            const uint32_t c = x >> 24;
            const uint32_t c1 = i >= 1 ? (x >> 16) & 0xffu : 0u;
            const uint32_t c2 = i >= 2 ? (x >> 8) & 0xffu : 0u;
            const uint32_t c3 = i >= 3 ? x & 0xffu : 0u;
            const bool cont = (c & 0xc0u) == 0x80u;
            const bool need = c1 >= 0xc0u || c2 >= 0xe0u || c3 >= 0xf0u;
            const uint32_t L = c < 0xc0u ? 0u : (c < 0xe0u ? 2u : (c < 0xf0u ? 3u : 4u));
            bad |= cont != need;
            bad |= c == 0xc0u || c == 0xc1u || c >= 0xf5u;
            bad |= (c1 == 0xe0u && c < 0xa0u) || (c1 == 0xedu && c > 0x9fu) ||
                   (c1 == 0xf0u && c < 0x90u) || (c1 == 0xf4u && c > 0x8fu);
            bad |= i + L > n;
        }
    }
    return !__any(bad);
}

// the text of the lanes with `na` (not all ASCII), one after another by the whole wave
NXG_DEV bool utf8_lanes(lds_bytes img, bool na, uint32_t soff, uint32_t slen, uint32_t lane) {
    uint64_t m = __ballot(na);
    bool good = true;
#pragma unroll 1
    while (m && good) {
        const int j = (int)__builtin_ctzll(m);
        m &= m - 1;
        good = utf8_wave(img, (uint32_t)__builtin_amdgcn_readlane((int)soff, j),
                         (uint32_t)__builtin_amdgcn_readlane((int)slen, j), lane);
    }
    return good;
}

// The same, all the texts at once: their bytes laid end to end, one per lane (64 per step), each
// lane finding its text through `mark` (LDS, 256 bytes: the text starting at each position). More
// than 256 bytes: utf8_lanes. The checks are utf8_wave's.
NXG_DEV bool utf8_packed(lds_bytes img, uint8_t* mark, bool na, uint32_t soff, uint32_t slen,
                         uint32_t lane) {
    const uint32_t len = na ? slen : 0u;
    const uint32_t inc = wave_incl_scan<uint32_t>(len);
    const uint32_t pre = inc - len;
    const uint32_t T = wave_last<uint32_t>(inc);
    if (T == 0) return true;
    if (T > 256u) return utf8_lanes(img, na, soff, slen, lane);
    reinterpret_cast<uint32_t*>(mark)[lane] = 0u;
    wave_lds_order();
    if (len) mark[pre] = (uint8_t)(lane + 1);
    wave_lds_order();
    bool bad = false;
    uint32_t carry = 0;
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < T; b0 += 64) {
        const uint32_t L = b0 + lane;
        const uint32_t j1 = max(wave_max_scan(L < T ? (uint32_t)mark[L] : 0u), carry);
        carry = wave_last<uint32_t>(j1);
        const int j = (int)j1 - 1;  // >= 0: text 0 starts at byte 0
        const uint32_t s = (uint32_t)__shfl((int)soff, j, 64);
        const uint32_t n = (uint32_t)__shfl((int)len, j, 64);
        const uint32_t i = L - (uint32_t)__shfl((int)pre, j, 64);
        if (L < T) {
            const uint32_t r = s + i - 3;
            lds_words w = (lds_words)(img + (r & ~3u));
            const uint32_t x = alignbyte(w[1], w[0], r & 3u);  // bytes i-3 .. i
            const uint32_t c = x >> 24;
            const uint32_t c1 = i >= 1 ? (x >> 16) & 0xffu : 0u;
            const uint32_t c2 = i >= 2 ? (x >> 8) & 0xffu : 0u;
            const uint32_t c3 = i >= 3 ? x & 0xffu : 0u;
            const bool cont = (c & 0xc0u) == 0x80u;
            const bool need = c1 >= 0xc0u || c2 >= 0xe0u || c3 >= 0xf0u;
            const uint32_t Lq = c < 0xc0u ? 0u : (c < 0xe0u ? 2u : (c < 0xf0u ? 3u : 4u));
            bad |= cont != need;
            bad |= c == 0xc0u || c == 0xc1u || c >= 0xf5u;
            bad |= (c1 == 0xe0u && c < 0xa0u) || (c1 == 0xedu && c > 0x9fu) ||
                   (c1 == 0xf0u && c < 0x90u) || (c1 == 0xf4u && c > 0x8fu);
            bad |= i + Lq > n;
        }
    }
    wave_lds_order();
    return !__any(bad);
}

// The deferred text checks of a tile: entries soff | slen << 16 in `list`, 64 per pass (ASCII per
// lane, the rest by utf8_packed). Uniform; false on invalid UTF-8.
// Text that leaves the tile's image (lanes with `want`: n bytes at frame offset off): the ASCII
// check by the whole wave from global memory, 4 bytes per lane, one text after the other; a text
// holding a byte >= 0x80 is then checked exactly (std::str::from_utf8 rules, utf8_ok) by its own
// lane. All 64 lanes active. Returns the lane's verdict (true when it has no such text).
NXG_DEV bool far_text_ok(const uint8_t* wire, bool want, uint64_t off, uint32_t n, uint32_t lane) {
    bool ok = true;
#pragma unroll 1
    for (uint64_t m = __ballot(want); m; m &= m - 1) {
        const uint32_t j = (uint32_t)__builtin_ctzll(m);
        const uint64_t sj =
            (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)off, (int)j) |
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(off >> 32), (int)j) << 32);
        const uint32_t nj = (uint32_t)__builtin_amdgcn_readlane((int)n, (int)j);
        bool hi = false;
#pragma unroll 1
        for (uint32_t k = 0; k < nj; k += 256) {
            const uint32_t o = k + 4u * lane;
            if (o < nj) {
                const uint32_t rem = nj - o;
#pragma unroll
                for (uint32_t q = 0; q < 4; q++)
                    if (q < rem) hi |= wire[sj + o + q] >= 0x80u;
            }
        }
        if (__any(hi) && lane == j) ok = utf8_ok(GlbSrc{(gbl_bytes)wire}, sj, nj);
    }
    return ok;
}

NXG_DEV bool text_flush(lds_bytes img, const uint32_t* list, uint32_t ntxt, uint8_t* mark,
                        uint32_t lane, DevStatus* st) {
    bool good = true;
#pragma unroll 1
    for (uint32_t b = 0; b < ntxt && good; b += 64) {
        const uint32_t i = b + lane;
        const uint32_t e = i < ntxt ? list[i] : 0u;
        const uint32_t so = e & 0xffffu, sl = e >> 16;
        // texts longer than 32 bytes: the ASCII check by the whole wave, 4 bytes per lane, one
        // text after the other (a lane alone would take a round of 32 bytes each while the
        // others wait)
        bool na_long = false;
#pragma unroll 1
        for (uint64_t lm = __ballot(sl > 32u); lm; lm &= lm - 1) {
            const uint32_t j = (uint32_t)__builtin_ctzll(lm);
            const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)so, (int)j);
            const uint32_t nj = (uint32_t)__builtin_amdgcn_readlane((int)sl, (int)j);
            bool hi = false;
#pragma unroll 1
            for (uint32_t k = 0; k < nj; k += 256) {
                const uint32_t off = k + 4u * lane;
                if (off < nj) {
                    uint32_t q[1];
                    win_words<1>(img, sj + off, q);
                    const uint32_t rem = nj - off;
                    const uint32_t keep = rem >= 4u ? 0xffffffffu : (1u << (8u * rem)) - 1u;
                    hi |= (q[0] & keep & 0x80808080u) != 0u;
                }
            }
            if (__any(hi) && lane == j) na_long = true;
        }
        const bool na = sl && (sl > 32u ? na_long : !ascii_ok(img, so, sl));
#if NXG_FMX_PROF
        {
            const uint64_t nm = __ballot(na);
            const uint32_t T = wave_sum<uint32_t>(na ? sl : 0u);
            if (lane == 0) {
                atomicAdd(&st->diag[4], 1ull);
                atomicAdd(&st->diag[5], (unsigned long long)__popcll(nm) | ((unsigned long long)T << 32));
            }
        }
#endif
        good = utf8_packed(img, mark, na, so, sl, lane);
    }
    return good;
}

// A fixed-size element other than DateTime / Duration (n = 0, 1, 2, 4 or 8 payload bytes): the
// fixed-size part of val_decode alone. q: 16 bytes from the tag; e0 / elim: tile offsets of the
// element and of its message end.
NXG_DEV FV fixed_elem(const uint32_t* q, uint32_t e0, uint32_t elim) {
    const uint32_t t = q[0] & 0xffu;
    const uint32_t bit = 1u << (t & 31u);
    const uint32_t f1 = fixed_size1(t), n = f1 - 1u;
    const uint32_t b0 = bswap32(alignbyte(q[1], q[0], 1)), b1 = bswap32(alignbyte(q[2], q[1], 1));
    const bool n8 = f1 == 9u;
    const uint32_t sh = (32u - 8u * n) & 31u;
    const bool sgn = bit & kSgnTags;
    const uint32_t lo32 = f1 >= 2u ? (sgn ? (uint32_t)((int32_t)b0 >> sh) : b0 >> sh)
                                   : ((bit & B(14)) ? 1u : 0u);
    FV o;
    o.tag = (bit & B(17)) ? 16u : t;
    o.fixed = n8 ? (((uint64_t)b0 << 32) | b1)
                 : (((uint64_t)(sgn ? (uint32_t)((int32_t)lo32 >> 31) : 0u) << 32) | lo32);
    o.aux = 0;
    o.end = e0 + f1;
    o.kids = 0;
    o.soff = 0;
    o.slen = 0;
    o.ok = elim >= e0 + f1;
    return o;
}
// fixed-size element tags fixed_elem takes (not DateTime 10, Duration 11)
NXG_DEV bool simple_fixed(uint32_t t) { return fixed_size1(t) != 0u && t != 10u && t != 11u; }

// A round's Array elements (non-containers): this lane's kd elements from tile offset oend (its
// array's first element, inside the message ending at lim), element slots cnext + kpre ..; rk =
// the round's total. Stride path: an array whose first element has a fixed size is taken to be
// all elements of that size; element j of the round is found from its array (a max-scan over
// `mark`) and checked by its own tag. Any array that does not fit (a variable-size element) sends
// the round to the exact walk. The pending text checks in el[0, ntxt) are flushed when the exact
// walk needs el. Returns true (uniform) on a decode error.
NXG_DEV bool round_elements(uint8_t* img, uint8_t* mark, uint32_t* el, uint32_t kd, uint32_t kpre,
                            uint32_t rk, uint32_t oend, uint32_t lim, uint64_t cnext,
                            const ColsDesc& cols, uint64_t t0, uint32_t lane, uint32_t& ntxt,
                            DevStatus* st) {
    const lds_bytes limg = (lds_bytes)img;
    bool bad = false, ok = true;
    bool strided = false;
    if (rk <= MAXC) {
        const uint32_t ep = oend;
        const uint32_t f1a = kd && ep < lim ? fixed_size1(img[ep]) : 0u;
        if (!__any(kd && f1a == 0u)) {
            reinterpret_cast<uint32_t*>(mark)[lane] = 0u;
            wave_lds_order();
            if (kd) mark[kpre] = (uint8_t)(lane + 1);
            wave_lds_order();
            strided = true;
            uint32_t carry = 0;
#pragma unroll 1
            for (uint32_t j0 = 0; j0 < rk; j0 += 64) {
                const uint32_t j = j0 + lane;
                const bool he = j < rk;
                const uint32_t a1 = max(wave_max_scan(he ? (uint32_t)mark[j] : 0u), carry);
                carry = wave_last<uint32_t>(a1);
                const int ai = (int)a1 - 1;  // mark[0] is set: the first array's kpre is 0
                // (ds_bpermute reads 0 from inactive lanes: all 64 take part)
                const uint32_t fa = (uint32_t)__shfl((int)f1a, ai, 64);
                const uint32_t epa = (uint32_t)__shfl((int)ep, ai, 64);
                const uint32_t kpa = (uint32_t)__shfl((int)kpre, ai, 64);
                const uint32_t lma = (uint32_t)__shfl((int)lim, ai, 64);
                const uint32_t e0 = he ? epa + (j - kpa) * fa : 8u;
                const uint32_t elim = he ? lma : 16u;
                uint32_t q[4];
                win_words<4>(limg, e0, q);
                const uint32_t et = q[0] & 0xffu;
                if (!__all(!he || (e0 < elim && fixed_size1(et) == fa))) {
                    strided = false;
                    break;
                }
                FV e;
                if (__all(!he || simple_fixed(et))) {  // scalars only: no text, no branches
                    e = fixed_elem(q, e0, elim);
                    bad = __any(he && !e.ok);
                } else {  // DateTime / Duration elements
                    e = val_decode(et, alignbyte(q[1], q[0], 1), alignbyte(q[2], q[1], 1),
                                   alignbyte(q[3], q[2], 1), e0 + 1, elim, false, t0);
                    bad = __any(he && !e.ok);
                }
                if (bad) break;
                const uint64_t slot = cnext + j;
                if (he && slot < cols.cap_children) {
                    col_st(&cols.ctag[slot], (uint8_t)e.tag);
                    col_st(&cols.cfixed[slot], (uint64_t)e.fixed);
                    col_st(&cols.caux[slot], (uint32_t)e.aux);
                }
            }
            wave_lds_order();
            if (bad) return true;
        }
    }
    if (!strided && ntxt) {  // the exact walk below uses el
        bad = !text_flush(limg, el, ntxt, mark, lane, st);
        ntxt = 0;
        wave_lds_order();
        if (bad) return true;
    }
    if (strided) {
    } else if (rk <= MAXC) {
        // element starts: a run of elements of the first one's fixed size is confirmed 8 at
        // a time from tags loaded together; other elements are sized by val_decode
        uint32_t ep = oend;
#pragma unroll 1
        for (uint32_t c = 0; c < kd;) {
            if (ep >= lim) {
                ok = false;
                break;
            }
            const uint32_t et = img[ep];
            const uint32_t f1 = fixed_size1(et);  // 1 + payload bytes (0: variable size)
            if (f1) {
                uint32_t tg[8];
#pragma unroll
                for (uint32_t r = 1; r < 8; r++) {
                    const uint32_t x = ep + r * f1;
                    tg[r] = c + r < kd && x < lim ? img[x] : 0xffu;
                }
                uint32_t r = 1;
#pragma unroll
                for (uint32_t k = 1; k < 8; k++) r += (r == k && fixed_size1(tg[k]) == f1) ? 1u : 0u;
#pragma unroll 1
                for (uint32_t k = 0; k < r; k++) {
                    const uint32_t x = ep + k * f1;
                    el[kpre + c + k] = x | ((lim - x) << 13);
                }
                ep += r * f1;
                c += r;
            } else {
                el[kpre + c] = ep | ((lim - ep) << 13);
                uint32_t q[3];
                win_words<3>(limg, ep + 1, q);
                const FV e = val_decode(et, q[0], q[1], q[2], ep + 1, lim, false, t0);
                ok = e.ok;
                ep = e.end;
                c++;
                if (!ok) break;
            }
        }
        bad = __any(!ok);
        if (bad) return true;
        wave_lds_order();
#pragma unroll 1
        for (uint32_t j0 = 0; j0 < rk; j0 += 64) {
            const uint32_t j = j0 + lane;
            const bool he = j < rk;
            const uint32_t ev = he ? el[j] : (8u << 13) | 8u;
            const uint32_t e0 = ev & 0x1fffu, elim = e0 + (ev >> 13);
            uint32_t q[4];
            win_words<4>(limg, e0, q);
            FV e;
            if (__all(!he || simple_fixed(q[0] & 0xffu))) {  // scalars only: no text, no branches
                e = fixed_elem(q, e0, elim);
                bad = __any(he && !e.ok);
            } else {
                e = val_decode(q[0] & 0xffu, alignbyte(q[1], q[0], 1), alignbyte(q[2], q[1], 1),
                               alignbyte(q[3], q[2], 1), e0 + 1, elim, false, t0);
                const bool eok = !he || e.ok;
                const bool ena = he && eok && e.slen && !ascii_ok(limg, e.soff, e.slen);
                bad = __any(!eok) || !utf8_packed(limg, mark, ena, e.soff, e.slen, lane);
            }
            if (bad) break;
            const uint64_t slot = cnext + j;
            if (he && slot < cols.cap_children) {
                col_st(&cols.ctag[slot], (uint8_t)e.tag);
                col_st(&cols.cfixed[slot], (uint64_t)e.fixed);
                col_st(&cols.caux[slot], (uint32_t)e.aux);
            }
        }
        wave_lds_order();
    } else {  // more elements than the list holds: each lane decodes its own
        uint32_t ep = oend;
#pragma unroll 1
        for (uint32_t c = 0; ok && c < kd; c++) {
            ok = ep < lim;
            if (!ok) break;
            const uint32_t et = img[ep];
            uint32_t q[3];
            win_words<3>(limg, ep + 1, q);
            const FV e = val_decode(et, q[0], q[1], q[2], ep + 1, lim, false, t0);
            ok = e.ok && (!e.slen || utf8_ok(LdsSrc{limg, t0}, t0 + e.soff, e.slen));
            const uint64_t slot = cnext + kpre + c;
            if (ok && slot < cols.cap_children) {
                col_st(&cols.ctag[slot], (uint8_t)e.tag);
                col_st(&cols.cfixed[slot], (uint64_t)e.fixed);
                col_st(&cols.caux[slot], (uint32_t)e.aux);
            }
            ep = e.end;
        }
        bad = __any(!ok);
    }
    return bad;
}

}  // namespace
