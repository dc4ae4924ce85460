// nxg_decode_mixed.hip -- the fast path of the mixed decode (config 3) for gfx950.
//
// Frames whose messages are all From::Update(id, v) with a one-byte length prefix (L < 128) and
// a value that is a scalar, text, Decimal or an Array of non-container elements -- what a
// publisher of ordinary values sends -- are decoded in two passes over 4 KiB tiles with no
// speculation across tiles beyond one checked guess. Anything else (control messages, longer
// messages, Map / Error(Value) / Abstract values, nested containers, any content error) raises
// fast_fail and the host reruns the frame on the general decoder (nxg_decode_gen.hip), which
// covers every case and reports errors exactly. The values are decoded by the same restatement
// as the general path (nxg_msg.h dleaf / dcontainer), so the columns are identical.
//
// Message boundaries. With one-byte lengths a message at p ends at p + b[p], and a message start
// is a byte in [4, 127] followed by the Update variant (4). Per tile, each lane takes a 64-byte
// chunk: its candidate starts (SWAR over its bytes) and, for its first two candidates, where the
// chain of messages from them leaves the chunk (an LDS walk of a few steps; every position on the
// way must be a candidate). One uniform loop over the 64 chunks then follows the true chain from
// the tile's entry: a chunk whose entry is its first or second candidate takes that candidate's
// exit, anything else is walked (rare). The count pass guesses the tile's entry (its first
// candidates, until one yields a complete chain); a false guess almost always merges into the
// true chain within the tile, so its exit is right and only its counts are wrong: the fix pass
// recounts every tile whose entry is not its predecessor's exit from that exit. The check then
// requires every tile's entry to be its predecessor's exit, the first 0 and the last exit W,
// which by induction from tile 0 makes every tile's chain the true one.
//
//   count   per tile: entry, exit, messages, child slots (array element counts)
//   fix     recount tiles entered off their predecessor's exit
//   scan    prefix sums (nxg_scan_u32) -> each tile's first row and child
//   check   the chain, the capacities, the totals
//   emit    per tile: the message list in LDS (wave scan of the per-chunk counts), then messages
//           k, k+64, ... per lane, decoded by fast_value (branch-light: every field from the 16
//           bytes after the tag, selected by tag), rows written 64 at a time, children at a wave
//           prefix of the element counts
#include <algorithm>

#include "nxg_internal.h"
#include "nxg_msg.h"

namespace fmx {
constexpr uint32_t TILE = 4096;
constexpr uint32_t CH = 64;
constexpr uint32_t IMG = TILE + 256;    // image: the tile + 256 B (messages are < 128 bytes)
constexpr uint32_t MAXM = TILE / 4;     // messages per tile (>= 4 bytes each)
constexpr uint32_t MAXC = 256;          // array elements per round of 64 messages (lane-parallel)
constexpr int TPB = 256;
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t FAIL = 0xfffffffeu;
}  // namespace fmx

namespace {
using namespace fmx;
using namespace nxgmsg;

struct CountLds {  // count / fix passes
    uint8_t img[IMG];
};
struct EmitLds {
    uint8_t img[IMG];
    uint16_t msg[MAXM];  // the tile's message starts
    uint32_t el[MAXC];   // a round's array elements: position | (message end - position) << 13
};

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

// candidate message starts in the lane's chunk: bit i = byte c+i in [4, 127] and byte c+i+1 == 4
NXG_DEV uint64_t cand_mask(const uint8_t* img, uint32_t c) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(img + c);
    uint64_t m = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t a = w[k], b = w[k + 1];
        const uint32_t len = ((a & 0x7f7f7f7fu) + 0x7c7c7c7cu) & ~a & 0x80808080u;
        const uint32_t var = zero_bytes(alignbyte(b, a, 1) ^ 0x04040404u);
        m |= (uint64_t)nib(len & var) << (4 * k);
    }
    return m;
}

// where the chain of messages from tile offset x (a candidate of chunk j) leaves the chunk, or
// FAIL (a position on the way is not a candidate start). `lim`: the tile's end in the frame
// (TILE, or less in the frame's last tile), where the chain stops.
NXG_DEV uint32_t chunk_exit(const uint8_t* img, uint32_t x, uint32_t j, uint64_t m, uint32_t lim) {
    const uint32_t end = min((j + 1) * CH, lim);
#pragma unroll 1
    for (int g = 0; g < 32 && x < end; g++) {
        if (!((m >> (x - j * CH)) & 1ull)) return FAIL;
        x += img[x];
    }
    return x < end ? FAIL : x;
}

// The tile's chain from entry e (tile offset): each lane's chunk entry (NONE: no message starts
// in the chunk) and the exit (first start >= lim), or FAIL. Uniform in the wave.
NXG_DEV uint32_t tile_chain(const uint8_t* img, uint32_t e, uint32_t lim, uint32_t lane,
                            uint64_t m, uint32_t c0, uint32_t x0, uint32_t c1, uint32_t x1,
                            uint32_t& ce) {
    ce = NONE;
    uint32_t x = e;
#pragma unroll 1
    for (uint32_t j = 0; j < TILE / CH && x < lim; j++) {
        if (x >= (j + 1) * CH) continue;  // a message covers the whole chunk
        if (lane == j) ce = x;
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)c0, (int)j);
        const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)c1, (int)j);
        if (x == a0) {
            x = (uint32_t)__builtin_amdgcn_readlane((int)x0, (int)j);
        } else if (x == a1) {
            x = (uint32_t)__builtin_amdgcn_readlane((int)x1, (int)j);
        } else {
            const uint32_t mlo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m, (int)j);
            const uint32_t mhi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(m >> 32), (int)j);
            x = chunk_exit(img, x, j, ((uint64_t)mhi << 32) | mlo, lim);
        }
        if (x == FAIL) return FAIL;
    }
    return x;
}

// per lane: the chunk's candidates and the first two's chunk exits
struct Cands {
    uint64_t m;
    uint32_t c0, x0, c1, x1;
};
NXG_DEV Cands lane_cands(const uint8_t* img, uint32_t lane, uint32_t lim) {
    Cands r;
    r.m = cand_mask(img, lane * CH);
    r.c0 = r.c1 = r.x0 = r.x1 = FAIL;
    uint64_t m = r.m;
    if (m) {
        r.c0 = lane * CH + (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        r.x0 = chunk_exit(img, r.c0, lane, r.m, lim);
    }
    if (m) {
        r.c1 = lane * CH + (uint32_t)__builtin_ctzll(m);
        r.x1 = chunk_exit(img, r.c1, lane, r.m, lim);
    }
    return r;
}

// The tile's chain as a scan (no serial loop). The state at the boundary in front of chunk j
// says where the next message start is: N0 / N1 = chunk j's first / second candidate, F0 / F1 =
// chunk j+1's (chunk j lies inside one message), END = at or past the tile end, FAIL = anywhere
// else. Chunk j maps the state in front of it to the state behind it: from N_a the chain runs to
// x_a, which lies in chunk j+1 or j+2 (messages are < 128 bytes) and must be a first or second
// candidate there; F_a becomes N_a; END and FAIL stay. These maps (6 states x 3 bits) compose
// associatively, so a wave scan of them gives every chunk's entry state at once. A chain that
// enters some chunk at a third candidate comes out FAIL here and goes to tile_chain.
constexpr uint32_t S_N0 = 0, S_N1 = 1, S_F0 = 2, S_F1 = 3, S_FAIL = 4, S_END = 5;
constexpr uint32_t T_ID = (0u << 0) | (1u << 3) | (2u << 6) | (3u << 9) | (4u << 12) | (5u << 15);
NXG_DEV uint32_t tget(uint32_t T, uint32_t st) { return (T >> (3 * st)) & 7u; }
NXG_DEV uint32_t tcompose(uint32_t later, uint32_t earlier) {
    uint32_t c = 0;
#pragma unroll
    for (uint32_t st = 0; st < 6; st++) c |= tget(later, tget(earlier, st)) << (3 * st);
    return c;
}
template <int CTRL, int ROWS>
NXG_DEV uint32_t dpp_fill(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, CTRL, ROWS, 0xf, false);
}
NXG_DEV uint32_t tscan(uint32_t T) {  // inclusive: lane j gets T_j o ... o T_0
    T = tcompose(T, dpp_fill<0x111, 0xf>(T, T_ID));
    T = tcompose(T, dpp_fill<0x112, 0xf>(T, T_ID));
    T = tcompose(T, dpp_fill<0x114, 0xf>(T, T_ID));
    T = tcompose(T, dpp_fill<0x118, 0xf>(T, T_ID));
    T = tcompose(T, dpp_fill<0x142, 0xa>(T, T_ID));
    T = tcompose(T, dpp_fill<0x143, 0xc>(T, T_ID));
    return T;
}

NXG_DEV uint32_t tile_chain_scan(uint32_t e, uint32_t lim, uint32_t lane, uint32_t c0, uint32_t x0,
                                 uint32_t c1, uint32_t x1, uint32_t& ce) {
    ce = NONE;
    // the candidates of chunks j+1 and j+2 (none past the tile)
    const uint32_t c0n = dpp_fill<0x130, 0xf>(c0, FAIL), c1n = dpp_fill<0x130, 0xf>(c1, FAIL);
    const uint32_t c0nn = dpp_fill<0x130, 0xf>(c0n, FAIL), c1nn = dpp_fill<0x130, 0xf>(c1n, FAIL);
    auto out = [&](uint32_t x) -> uint32_t {
        if (x == FAIL) return S_FAIL;
        if (x >= lim) return S_END;
        const uint32_t d = (x >> 6) - lane;
        if (d == 1) return x == c0n ? S_N0 : (x == c1n ? S_N1 : S_FAIL);
        if (d == 2) return x == c0nn ? S_F0 : (x == c1nn ? S_F1 : S_FAIL);
        return S_FAIL;
    };
    const uint32_t T = out(x0) | (out(x1) << 3) | (S_N0 << 6) | (S_N1 << 9) | (S_FAIL << 12) |
                       (S_END << 15);
    // the state in front of chunk 0
    uint32_t s0;
    if (e >= lim) {
        return e;  // no message starts in this tile
    } else if (e < CH) {
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)c0, 0);
        const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)c1, 0);
        s0 = e == a0 ? S_N0 : (e == a1 ? S_N1 : S_FAIL);
    } else if (e < 2 * CH) {
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)c0, 1);
        const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)c1, 1);
        s0 = e == a0 ? S_F0 : (e == a1 ? S_F1 : S_FAIL);
    } else {
        s0 = S_FAIL;
    }
    if (s0 == S_FAIL) return FAIL;
    const uint32_t sout = tget(tscan(T), s0);          // state behind chunk j
    const uint32_t sin = dpp_fill<0x138, 0xf>(sout, s0);  // in front of chunk j (wave_shr:1)
    if (wave_last<uint32_t>(sout) != S_END) return FAIL;
    if (sin == S_N0) ce = c0;
    else if (sin == S_N1) ce = c1;
    // the exit: the last start's chunk, whose state behind is the first END
    const bool last = (sin == S_N0 || sin == S_N1) && sout == S_END;
    const uint64_t lm = __ballot(last);
    if (!lm) return FAIL;
    const uint32_t xl = sin == S_N0 ? x0 : x1;
    return (uint32_t)__builtin_amdgcn_readlane((int)xl, (int)__builtin_ctzll(lm));
}

// Header of the message at tile offset p: child slots (Array element count), or FAIL when the
// message is not for the fast path. The value tag sits after the variant and the id varint.
NXG_DEV uint32_t msg_kids(const uint8_t* img, uint32_t p) {
    const uint64_t w = win16((lds_bytes)img, p + 2).lo;  // id varint, tag, next byte
    const uint64_t stop = ~w & 0x8080808080808080ull;
    const uint32_t k = stop ? (uint32_t)__builtin_ctzll(stop) >> 3 : 8u;
    if (k >= 5) return FAIL;  // ids wider than 35 bits: the general decoder
    const uint32_t t = (uint32_t)(w >> (8 * k + 8)) & 0xffu;
    const uint32_t c = (uint32_t)(w >> (8 * k + 16)) & 0xffu;
    if (t == 19) return c < 0x80u ? c : FAIL;
    if (t == 21 || t >= 28u) return FAIL;
    if (t == 22 && c != 12u) return FAIL;  // Error(Value) of a non-String
    return 0;
}

// the messages of the lane's chunk from its entry: count, child slots, and their starts as bits
// of the chunk (bit i: chunk byte i)
NXG_DEV bool chunk_msgs(const uint8_t* img, uint32_t ce, uint32_t lane, uint32_t lim, uint32_t& n,
                        uint32_t& kids, uint64_t& bits) {
    n = 0;
    kids = 0;
    bits = 0;
    if (ce == NONE) return true;
    uint32_t x = ce;
    const uint32_t c = lane * CH, end = min(c + CH, lim);
#pragma unroll 1
    while (x < end) {
        const uint32_t k = msg_kids(img, x);
        if (k == FAIL) return false;
        bits |= 1ull << (x - c);
        n++;
        kids += k;
        x += img[x];
    }
    return true;
}

// tile descriptor (count pass -> resolve -> emit)
struct TileDesc {
    uint32_t entry, exit;  // tile offsets
    uint32_t rows, kids;
};

// The tile's descriptor for the chain from entry e: exit, messages, child slots (FAIL entry and
// exit when the chain breaks, or does not end exactly at the frame end in the last tile).
// `bits`: the lane's message starts (chunk_msgs).
NXG_DEV TileDesc count_from(const uint8_t* img, const Cands& cd, uint32_t e, uint32_t lim,
                            bool last, uint32_t lane, uint64_t& bits) {
    uint32_t ce;
    uint32_t x = tile_chain_scan(e, lim, lane, cd.c0, cd.x0, cd.c1, cd.x1, ce);
    if (x == FAIL) x = tile_chain(img, e, lim, lane, cd.m, cd.c0, cd.x0, cd.c1, cd.x1, ce);
    bool bad = x == FAIL || (last && x != lim);
    uint32_t n = 0, k = 0;
    bits = 0;
    if (!bad) bad = !chunk_msgs(img, ce, lane, lim, n, k, bits);
    bad = __any(bad);
    if (bad) return TileDesc{FAIL, FAIL, 0, 0};
    return TileDesc{e, x, wave_sum<uint32_t>(n), wave_sum<uint32_t>(k)};
}

// ---- the emit pass's value decoder ---------------------------------------------------------------
// Value::decode (netidx-value/src/lib.rs:470-506) for the values this path takes, restated as
// nxg_msg.h dleaf / dcontainer do, but with every field computed from the 16 bytes after the tag
// and selected by tag, so that a wave whose lanes hold different tags runs one instruction stream
// (only text validation and array elements loop). Any decode error returns false: the frame
// then goes to the general decoder, which reports it.

// the 7-bit groups of the (up to) 8 bytes of y, least significant first
NXG_DEV uint64_t compress7(uint64_t y) {
    const uint64_t z1 = (y & 0x007f007f007f007full) | ((y >> 1) & 0x3f803f803f803f80ull);
    const uint64_t z2 = (z1 & 0x00003fff00003fffull) | ((z1 >> 2) & 0x0fffc0000fffc000ull);
    return (z2 & 0x0fffffffull) | ((z2 >> 4) & 0x00fffffff0000000ull);
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

struct FVal {
    uint32_t tag, aux;
    uint64_t fixed, next, kids;
};

// The value whose tag t was consumed, payload at q (< lim, the message's end); arrays only when
// `arr` (a row), with their element count in kids (the caller sets fixed to the child base).
NXG_DEV bool fast_value(lds_bytes img, uint64_t t0, uint32_t t, uint64_t q, uint64_t lim, bool arr,
                        FVal& o) {
    if (t >= 28u || t == 21u || (t == 19u && !arr)) return false;
    Win16 wn = win16(img, (uint32_t)(q - t0));
    const bool e22 = t == 22u;
    if (e22) {  // Error(Value) whose inner value is a String: the String after its tag (12)
        if ((wn.lo & 0xffu) != 12u) return false;
        wn.lo = (wn.lo >> 8) | (wn.hi << 56);
        wn.hi >>= 8;
        q += 1;
    }
    const uint64_t room = lim > q ? lim - q : 0;
    uint64_t v;
    const uint32_t nb = wvar(wn.lo, wn.hi, v);
    const bool vok = nb != 0 && nb <= room;
    const uint32_t f1 = fixed_size1(t);
    o.tag = t == 17u ? 16u : (e22 ? 18u : t);
    o.aux = 0;
    o.kids = 0;
    bool ok;
    if (f1) {  // fixed-size payload: n big-endian bytes (0: Bool / Null; 12: DateTime, Duration)
        const uint32_t n = f1 - 1;
        const uint64_t be8 = __builtin_bswap64(wn.lo);
        const uint32_t sh = 64u - 8u * min(n, 8u);
        const uint64_t fx = n ? (be8 >> (sh & 63u)) : 0ull;
        const uint32_t sb = t == 2u ? 32u : (t == 24u ? 8u : (t == 26u ? 16u : 0u));  // signed
        o.fixed = t == 14u ? 1ull : (sb ? (uint64_t)((int64_t)(fx << (64u - sb)) >> (64u - sb)) : fx);
        o.next = q + n;
        ok = room >= n;
        if (n == 12u) {
            uint32_t ns = bswap32((uint32_t)wn.hi);
            uint64_t secs = be8;
            if (t == 10u) {
                ok &= datetime_valid((int64_t)secs, ns);
            } else if (ns >= 1000000000u) {  // Duration::new normalisation (dleaf case 11)
                const uint64_t add = ns / 1000000000u;
                ok &= secs + add >= secs;
                secs += add;
                ns %= 1000000000u;
            }
            o.fixed = secs;
            o.aux = ns;
        }
    } else if (t == 1u || t == 3u || t == 5u || t == 7u) {
        const uint32_t n32 = (uint32_t)v;
        const int32_t z32 = (int32_t)(n32 >> 1) ^ (int32_t)(0u - (n32 & 1u));
        o.fixed = t == 1u ? (uint64_t)n32
                : t == 3u ? (uint64_t)(int64_t)z32
                : t == 5u ? v : ((v >> 1) ^ (0ull - (v & 1ull)));
        o.next = q + nb;
        ok = vok;
    } else if (t == 19u) {  // ValArray header (array.rs:595-612): count guard as dcontainer
        const uint64_t p = q + nb;
        ok = vok && v <= kMaxVec / 16 && v * 16 <= ((lim - p) << 8);
        o.aux = (uint32_t)v;
        o.kids = v;
        o.next = p;
        o.fixed = 0;
    } else if (t == 20u) {  // Decimal: 16 bytes, not interpreted
        ok = room >= 16;
        o.fixed = q;
        o.aux = 16;
        o.next = q + 16;
    } else if (t == 27u) {  // Abstract: len-wrapped (dleaf case 27)
        const uint64_t p = q + nb;
        ok = vok && v >= 1;
        const uint64_t take = ok ? v - vl64(v) : 0;
        const uint64_t l2 = take < lim - p ? p + take : lim;
        ok &= l2 - p >= 16;
        o.fixed = p;
        o.aux = (uint32_t)(l2 - p);
        o.next = l2;
    } else {  // String / Bytes / Error(String): varint length, then the bytes (UTF-8 but Bytes)
        const uint64_t off = q + nb;
        ok = vok && v <= room - nb;
        o.fixed = off;
        o.aux = (uint32_t)v;
        o.next = off + v;
        if (ok && t != 13u) ok = utf8_ok(LdsSrc{img, t0}, off, v);
    }
    return ok;
}

}  // namespace

// The count pass for one tile (image in LDS). The entry of tile 0 is 0; any other tile guesses
// its entry: the first candidates of its first two chunks, in order, until one gives a complete
// chain. A false guess whose chain merges into the true one gives the true exit but wrong counts:
// the fix pass recounts such tiles from their predecessor's exit.
NXG_DEV TileDesc count_tile(const uint8_t* img, uint64_t t, uint64_t nt, uint64_t W,
                            uint32_t lane, uint64_t& bits) {
    const uint64_t t0 = t * TILE;
    const uint32_t lim = (uint32_t)min<uint64_t>(TILE, W - t0);
    const bool last = t + 1 == nt;
    const Cands cd = lane_cands(img, lane, lim);
    TileDesc d{FAIL, FAIL, 0, 0};
    bits = 0;
    if (t == 0) return count_from(img, cd, 0, lim, last, lane, bits);
    uint64_t mm = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cd.m, 0) |
                  ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(cd.m >> 32), 0) << 32);
    uint64_t m1 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cd.m, 1) |
                  ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(cd.m >> 32), 1) << 32);
#pragma unroll 1
    for (int tries = 0; tries < 4 && d.entry == FAIL && (mm | m1); tries++) {
        uint32_t g;
        if (mm) {
            g = (uint32_t)__builtin_ctzll(mm);
            mm &= mm - 1;
        } else {
            g = CH + (uint32_t)__builtin_ctzll(m1);
            m1 &= m1 - 1;
        }
        d = count_from(img, cd, g, lim, last, lane, bits);
    }
    return d;
}

// count pass: one wave per tile
__global__ __launch_bounds__(TPB) void nxg_fmx_count_kernel(const uint8_t* __restrict__ wire,
                                                            uint64_t W, uint64_t nt,
                                                            TileDesc* __restrict__ td,
                                                            uint64_t* __restrict__ starts,
                                                            DevStatus* zst) {
    zero_status(zst);
    __shared__ __attribute__((aligned(16))) CountLds lds[TPB / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t t = (uint64_t)blockIdx.x * (TPB / 64) + w;
    if (t >= nt) return;
    uint8_t* img = lds[w].img;
    TileRegs g;
    tile_load(g, wire, t * TILE, W, lane);
    tile_store(img, g, lane);
    uint64_t bits;
    const TileDesc d = count_tile(img, t, nt, W, lane, bits);
    starts[t * 64 + lane] = bits;
    if (lane == 0) td[t] = d;
}

// fix pass: a tile whose entry is not its predecessor's exit is recounted from that exit. One
// lane per tile finds them (64 tiles per wave), the wave recounts each; the others' descriptors
// are copied. Counts go to rows[] / kids[] for the scans.
__global__ __launch_bounds__(TPB) void nxg_fmx_fix_kernel(const uint8_t* __restrict__ wire,
                                                          uint64_t W, uint64_t nt,
                                                          const TileDesc* __restrict__ td,
                                                          TileDesc* __restrict__ td2,
                                                          uint32_t* __restrict__ rows,
                                                          uint32_t* __restrict__ kids,
                                                          uint64_t* __restrict__ starts) {
    __shared__ __attribute__((aligned(16))) CountLds lds[TPB / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t base = ((uint64_t)blockIdx.x * (TPB / 64) + w) * 64;
    if (base >= nt) return;
    const uint64_t tl = base + lane;
    bool mis = false;
    if (tl < nt) {
        const TileDesc d = td[tl];
        if (tl > 0) {
            // (a failed predecessor fails the frame in the check pass)
            const uint32_t px = td[tl - 1].exit;
            mis = px != FAIL && px - TILE != d.entry;
        }
        if (!mis) {
            td2[tl] = d;
            rows[tl] = d.rows;
            kids[tl] = d.kids;
        }
    }
    uint64_t m = __ballot(mis);
    uint8_t* img = lds[w].img;
#pragma unroll 1
    while (m) {
        const uint64_t t = base + (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        const uint32_t px = td[t - 1].exit;
        const uint64_t t0 = t * TILE;
        const uint32_t lim = (uint32_t)min<uint64_t>(TILE, W - t0);
        TileRegs g;
        tile_load(g, wire, t0, W, lane);
        tile_store(img, g, lane);
        const Cands cd = lane_cands(img, lane, lim);
        uint64_t bits;
        const TileDesc d = count_from(img, cd, px - TILE, lim, t + 1 == nt, lane, bits);
        starts[t * 64 + lane] = bits;
        if (lane == 0) {
            td2[t] = d;
            rows[t] = d.rows;
            kids[t] = d.kids;
        }
    }
}

// resolve: every tile's entry is its predecessor's exit (the first: 0); totals to the status
__global__ __launch_bounds__(TPB) void nxg_fmx_check_kernel(uint64_t W, uint64_t nt,
                                                            const TileDesc* __restrict__ td,
                                                            const uint64_t* __restrict__ rbase,
                                                            const uint64_t* __restrict__ cbase,
                                                            uint64_t cap_rows, uint64_t cap_children,
                                                            DevStatus* __restrict__ st) {
    const uint64_t t = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    bool bad = false;
    if (t < nt) {
        const TileDesc d = td[t];
        if (d.entry == FAIL) bad = true;
        else if (t == 0) bad = d.entry != 0;
        else bad = td[t - 1].exit != d.entry + TILE;
        if (t == nt - 1) {
            const uint64_t nr = rbase[t] + d.rows, nc = cbase[t] + d.kids;
            // columns too small: the general decoder reports the capacity error
            if (nr > cap_rows || nc > cap_children) bad = true;
            if (!bad) {
                st->n_rows = nr;
                st->n_children = nc;
                st->path = 4;  // the fast mixed decoder (mixed layout)
            }
        }
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(&st->fast_fail, 1u);
}

// emit: one wave per tile. The message starts come from the count / fix passes (bits per
// chunk), so the emit pass does not walk the chain again.
__global__ __launch_bounds__(TPB) void nxg_fmx_emit_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, const TileDesc* __restrict__ td,
    const uint64_t* __restrict__ rbase, const uint64_t* __restrict__ cbase,
    const uint64_t* __restrict__ starts, ColsDesc cols, DevStatus* __restrict__ st) {
    __shared__ __attribute__((aligned(16))) EmitLds lds[TPB / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t t = (uint64_t)blockIdx.x * (TPB / 64) + w;
    if (t >= nt) return;
    uint8_t* img = lds[w].img;
    uint16_t* msg = lds[w].msg;
    const lds_bytes limg = (lds_bytes)img;
    const uint64_t t0 = t * TILE;
    TileRegs g;
    tile_load(g, wire, t0, W, lane);
    uint64_t bits = starts[t * 64 + lane];
    const uint32_t nm = td[t].rows;
    const uint64_t rb = rbase[t];
    uint64_t cnext = cbase[t];  // first child slot of this round's messages
    if (ld_agent32(&st->fast_fail)) return;
    tile_store(img, g, lane);
    // the message list in wire order
    const uint32_t n0 = (uint32_t)__popcll(bits);
    uint32_t at = wave_incl_scan<uint32_t>(n0) - n0;
    bool bad = wave_last<uint32_t>(at + n0) != nm;
#pragma unroll 1
    while (bits) {
        msg[at++] = (uint16_t)(lane * CH + (uint32_t)__builtin_ctzll(bits));
        bits &= bits - 1;
    }
    wave_lds_order();
#pragma unroll 1
    for (uint32_t k = 0; k < nm && !bad; k += 64) {
        const uint32_t i = k + lane;
        const bool has = i < nm;
        const uint32_t p = has ? msg[i] : 0u;
        // header: length (one byte), Update variant, id varint, value tag
        const uint64_t pa = t0 + p;
        const uint64_t lim = pa + img[p];
        const Win16 h = win16(limg, p + 2);
        uint64_t id;
        const uint32_t nb = wvar(h.lo, h.hi, id);
        const uint64_t q = pa + 2 + nb;
        bool ok = !has || (lim <= W && nb != 0 && q < lim);
        FVal o{0, 0, 0, 0, 0};
        if (has && ok) ok = fast_value(limg, t0, img[q - t0], q + 1, lim, true, o);
        const uint32_t kd = has && ok ? (uint32_t)o.kids : 0u;
        const uint32_t kpre = wave_incl_scan<uint32_t>(kd) - kd;
        const uint64_t cb = cnext + kpre;
        if (has && ok) {
            const uint64_t row = rb + i;
            cols.id[row] = id;
            cols.tag[row] = (uint8_t)o.tag;
            cols.fixed[row] = o.tag == 19u ? cb : o.fixed;
            cols.aux[row] = o.aux;
        }
        // array elements (non-containers): their starts (a walk by size), then one lane each
        const uint32_t rk = wave_sum<uint32_t>(kd);
        uint32_t* el = lds[w].el;
        uint64_t ep = o.next;
        if (rk <= MAXC) {
#pragma unroll 1
            for (uint32_t c = 0; ok && c < kd; c++) {
                ok = ep < lim;
                if (!ok) break;
                el[kpre + c] = (uint32_t)(ep - t0) | ((uint32_t)(lim - ep) << 13);
                const uint32_t et = img[ep - t0];
                const uint32_t f1 = fixed_size1(et);  // 1 + payload bytes (0: variable size)
                if (f1) {
                    ep += f1;
                } else {
                    FVal e{0, 0, 0, 0, 0};
                    ok = fast_value(limg, t0, et, ep + 1, lim, false, e);
                    ep = e.next;
                }
            }
            wave_lds_order();
#pragma unroll 1
            for (uint32_t j0 = 0; j0 < rk && !__any(!ok); j0 += 64) {
                const uint32_t j = j0 + lane;
                if (j < rk) {
                    const uint32_t ev = el[j];
                    const uint64_t e0 = t0 + (ev & 0x1fffu);
                    FVal e{0, 0, 0, 0, 0};
                    ok = fast_value(limg, t0, img[ev & 0x1fffu], e0 + 1, e0 + (ev >> 13), false, e);
                    const uint64_t slot = cnext + j;
                    if (ok && slot < cols.cap_children) {
                        cols.ctag[slot] = (uint8_t)e.tag;
                        cols.cfixed[slot] = e.fixed;
                        cols.caux[slot] = e.aux;
                    }
                }
            }
            wave_lds_order();
        } else {  // more elements than the list holds: each lane decodes its own
#pragma unroll 1
            for (uint32_t c = 0; ok && c < kd; c++) {
                FVal e{0, 0, 0, 0, 0};
                ok = ep < lim && fast_value(limg, t0, img[ep - t0], ep + 1, lim, false, e);
                const uint64_t slot = cb + c;
                if (ok && slot < cols.cap_children) {
                    cols.ctag[slot] = (uint8_t)e.tag;
                    cols.cfixed[slot] = e.fixed;
                    cols.caux[slot] = e.aux;
                }
                ep = e.next;
            }
        }
        bad = __any(!ok);
        cnext += wave_sum<uint32_t>(kd);
    }
    if (bad && lane == 0) atomicOr(&st->fast_fail, 1u);
}

// ---- launch (host) --------------------------------------------------------------------------------
uint64_t nxg_fmx_tiles(uint64_t W) { return (W + TILE - 1) / TILE; }

uint64_t nxg_fmx_scratch_bytes(uint64_t W) {
    const uint64_t nt = nxg_fmx_tiles(W);
    // 2 descs 32 B, message starts 512 B, rows + kids 8 B, rbase + cbase 16 B per tile, block
    // sums, alignment
    return nt * 568 + 2 * 8 * (nt / 4096 + 2) + 8 * 16;
}

// persistent grids: every workgroup co-resident (count: [0], emit: [1])
void nxg_fmx_wgs(int ncu, int* wgs) {
    int a = 0, b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, nxg_fmx_count_kernel, TPB, 0) !=
            hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, nxg_fmx_emit_kernel, TPB, 0) != hipSuccess) {
        a = b = 1;
    }
    wgs[0] = std::max(1, a) * ncu;
    wgs[1] = std::max(1, b) * ncu;
}

hipError_t nxg_launch_dec_fmx(const uint8_t* wire, uint64_t W, const ColsDesc& cols,
                              uint8_t* scratch, const int* wgs, DevStatus* st, hipStream_t s) {
    const uint64_t nt = nxg_fmx_tiles(W);
    if (nt == 0) return hipSuccess;
    uint8_t* p = scratch;
    auto take = [&](uint64_t bytes) {
        uint8_t* r = p;
        p += (bytes + 15) & ~15ull;
        return r;
    };
    TileDesc* td = reinterpret_cast<TileDesc*>(take(16 * nt));
    TileDesc* td2 = reinterpret_cast<TileDesc*>(take(16 * nt));
    uint64_t* starts = reinterpret_cast<uint64_t*>(take(512 * nt));
    uint32_t* rows = reinterpret_cast<uint32_t*>(take(4 * nt));
    uint32_t* kids = reinterpret_cast<uint32_t*>(take(4 * nt));
    uint64_t* rbase = reinterpret_cast<uint64_t*>(take(8 * nt));
    uint64_t* cbase = reinterpret_cast<uint64_t*>(take(8 * nt));
    uint64_t* bs0 = reinterpret_cast<uint64_t*>(take(8 * (nt / 4096 + 2)));
    uint64_t* bs1 = reinterpret_cast<uint64_t*>(take(8 * (nt / 4096 + 2)));
    constexpr uint64_t WV = TPB / 64;  // waves per workgroup
    // one tile per wave measured faster than persistent waves with the next tile prefetched
    // (count 184 vs 237 us, emit 534 vs 653 us at 10^7 records): the passes are bound by the
    // latency of their own LDS walks, which more resident waves hide better
    (void)wgs;
    const uint32_t gc = (uint32_t)((nt + WV - 1) / WV), ge = gc;
    hipLaunchKernelGGL(nxg_fmx_count_kernel, dim3(gc), dim3(TPB), 0, s, wire, W, nt, td, starts,
                       nxg_take_zero_slot());
    hipLaunchKernelGGL(nxg_fmx_fix_kernel, dim3((uint32_t)((nt + 64 * WV - 1) / (64 * WV))),
                       dim3(TPB), 0, s, wire, W, nt, td, td2, rows, kids, starts);
    hipError_t e;
    if ((e = nxg_scan_u32(rows, nt, rbase, bs0, s)) != hipSuccess) return e;
    if ((e = nxg_scan_u32(kids, nt, cbase, bs1, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(nxg_fmx_check_kernel, dim3((uint32_t)((nt + TPB - 1) / TPB)), dim3(TPB), 0,
                       s, W, nt, td2, rbase, cbase, cols.cap_rows, cols.cap_children, st);
    hipLaunchKernelGGL(nxg_fmx_emit_kernel, dim3(ge), dim3(TPB), 0, s, wire, W, nt, td2, rbase,
                       cbase, starts, cols, st);
    return hipGetLastError();
}
