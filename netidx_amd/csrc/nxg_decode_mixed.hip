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
//   resolve one launch: recount tiles entered off their predecessor's exit, a block scan of the
//           (messages, child slots) pairs, and the last block to arrive scans the block sums and
//           checks the capacities (no workgroup waits on another)
//   emit    per tile: the chain check (entry = predecessor's exit), the message list in LDS (wave
//           scan of the per-chunk counts), then messages k, k+64, ... per lane, decoded by
//           val_decode (every field from the bytes after the tag, selected by tag bit sets), rows
//           written 64 at a time; text checked once per tile (ASCII per lane, the rest by one
//           packed wave pass); array elements found by stride speculation (each element's tag
//           confirms the size) and decoded one per lane, the exact walk as the fallback
#include <algorithm>

#include "nxg_internal.h"
#include "nxg_msg.h"

#ifndef NXG_FMX_SKIP
#define NXG_FMX_SKIP 0  // timing experiments only: 1 elements, 2 text, 4 row values, 8 row stores
#endif
// timing experiments only: per-section wave clocks of the emit pass summed into DevStatus.diag
#if NXG_FMX_PROF
#define PMARK(k)                                          \
    do {                                                  \
        const uint64_t _t = __builtin_amdgcn_s_memtime(); \
        _acc[k] += _t - _pt;                              \
        _pt = _t;                                         \
    } while (0)
#else
#define PMARK(k) \
    do {         \
    } while (0)
#endif

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
    uint8_t mark[256];   // utf8_packed
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
// candidate there; F_a becomes N_a; END and FAIL stay. These maps (a byte per state) compose
// associatively, so a wave scan of them gives every chunk's entry state at once. A chain that
// enters some chunk at a third candidate comes out FAIL here and goes to tile_chain.
constexpr uint32_t S_N0 = 0, S_N1 = 1, S_F0 = 2, S_F1 = 3, S_FAIL = 4, S_END = 5;
// A map is 8 bytes (states 0..7, byte s = the image of s) in two words; composing two maps is a
// byte select of the later map by the earlier one (v_perm_b32: selector bytes 0..3 pick bytes
// of its second operand, 4..7 of its first).
struct SMap {
    uint32_t lo, hi;
};
constexpr uint32_t ID_LO = 0x03020100u, ID_HI = 0x07060504u;
NXG_DEV SMap scompose(SMap later, SMap earlier) {
    return SMap{__builtin_amdgcn_perm(later.hi, later.lo, earlier.lo),
                __builtin_amdgcn_perm(later.hi, later.lo, earlier.hi)};
}
NXG_DEV uint32_t sget(SMap m, uint32_t st) {
    return ((st < 4u ? m.lo : m.hi) >> (8u * (st & 3u))) & 0xffu;
}
template <int CTRL, int ROWS>
NXG_DEV uint32_t dpp_fill(uint32_t v, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS>
NXG_DEV SMap dpp_map(SMap m) {
    return SMap{dpp_fill<CTRL, ROWS>(m.lo, ID_LO), dpp_fill<CTRL, ROWS>(m.hi, ID_HI)};
}
NXG_DEV SMap sscan(SMap T) {  // inclusive: lane j gets T_j o ... o T_0
    T = scompose(T, dpp_map<0x111, 0xf>(T));
    T = scompose(T, dpp_map<0x112, 0xf>(T));
    T = scompose(T, dpp_map<0x114, 0xf>(T));
    T = scompose(T, dpp_map<0x118, 0xf>(T));
    T = scompose(T, dpp_map<0x142, 0xa>(T));
    T = scompose(T, dpp_map<0x143, 0xc>(T));
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
    // F0 -> N0, F1 -> N1, FAIL and END (and the unused 6, 7) stay
    const SMap T{out(x0) | (out(x1) << 8) | (S_N0 << 16) | (S_N1 << 24),
                 S_FAIL | (S_END << 8) | (6u << 16) | (7u << 24)};
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
    const uint32_t sout = sget(sscan(T), s0);          // state behind chunk j
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
NXG_DEV bool text_flush(lds_bytes img, const uint32_t* list, uint32_t ntxt, uint8_t* mark,
                        uint32_t lane, DevStatus* st) {
    bool good = true;
#pragma unroll 1
    for (uint32_t b = 0; b < ntxt && good; b += 64) {
        const uint32_t i = b + lane;
        const uint32_t e = i < ntxt ? list[i] : 0u;
        const uint32_t so = e & 0xffffu, sl = e >> 16;
        const bool na = sl && !ascii_ok(img, so, sl);
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

// resolve: everything between the count and the emit passes in one launch (no waiting on other
// workgroups). A lane per tile: a tile whose entry is not its predecessor's exit is recounted
// from that exit by its wave, tile by tile; then a block scan of (rows | child slots << 32) gives
// each tile its offset in the block (tloc), and the last block to arrive (a counter in the call's
// status slot, DevStatus.diag[7], zeroed with the slot) scans the block sums (bpre), checks the
// capacities and writes the totals. The chain (every entry its predecessor's exit) is checked by
// the emit pass. Frames are shorter than 2^32 bytes here, so both halves stay in 32 bits.
__global__ __launch_bounds__(TPB) void nxg_fmx_resolve_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, const TileDesc* __restrict__ td,
    TileDesc* __restrict__ td2, uint64_t* __restrict__ starts, uint64_t* __restrict__ tloc,
    uint64_t* __restrict__ bsum, uint64_t* __restrict__ bpre, uint64_t cap_rows,
    uint64_t cap_children, DevStatus* __restrict__ st) {
    __shared__ __attribute__((aligned(16))) CountLds lds[TPB / 64];
    __shared__ uint64_t scan_tmp[TPB / 64];
    __shared__ uint32_t is_last;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t tl = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    TileDesc d{FAIL, FAIL, 0, 0};
    bool mis = false;
    if (tl < nt) {
        d = td[tl];
        if (tl > 0) {
            // (a failed predecessor fails the frame in the emit pass's chain check)
            const uint32_t px = td[tl - 1].exit;
            mis = px != FAIL && px - TILE != d.entry;
        }
    }
    uint64_t m = __ballot(mis);
#if NXG_FMX_PROF
    if (lane == 0 && m) {
        atomicAdd(&st->diag[5], (unsigned long long)__popcll(m));
        atomicMax(&st->diag[4], (unsigned long long)__popcll(m));
    }
#endif
    uint8_t* img = lds[w].img;
#pragma unroll 1
    while (m) {
        const uint32_t j = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        const uint64_t t = tl - lane + j;
        const uint32_t px = td[t - 1].exit;
        const uint64_t t0 = t * TILE;
        const uint32_t lim = (uint32_t)min<uint64_t>(TILE, W - t0);
        TileRegs g;
        tile_load(g, wire, t0, W, lane);
        tile_store(img, g, lane);
        const Cands cd = lane_cands(img, lane, lim);
        uint64_t bits;
        const TileDesc r = count_from(img, cd, px - TILE, lim, t + 1 == nt, lane, bits);
        starts[t * 64 + lane] = bits;
        if (lane == j) d = r;
    }
    if (tl < nt) td2[tl] = d;
    const uint64_t v = tl < nt ? (uint64_t)d.rows | ((uint64_t)d.kids << 32) : 0ull;
    uint64_t tot;
    const uint64_t ex = block_excl_scan<uint64_t, TPB>(v, scan_tmp, &tot);
    if (tl < nt) tloc[tl] = ex;
    // the block sum goes out with an agent-scope store and is drained before the arrival count
    // (an agent-scope fence would write back the XCD's L2, full of the count pass's output);
    // the last block reads the sums with agent-scope loads
    if (threadIdx.x == 0) {
        st_agent(&bsum[blockIdx.x], tot);
        drain_stores();
        is_last = atomicAdd(&st->diag[7], 1ull) == (unsigned long long)gridDim.x - 1;
    }
    __syncthreads();
    if (!is_last) return;
    const uint32_t nb = gridDim.x;
    uint64_t run = 0;
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < nb; b0 += TPB) {
        const uint32_t b = b0 + threadIdx.x;
        const uint64_t x = b < nb ? ld_agent(&bsum[b]) : 0ull;
        uint64_t t2;
        const uint64_t e2 = block_excl_scan<uint64_t, TPB>(x, scan_tmp, &t2);
        if (b < nb) bpre[b] = run + e2;
        run += t2;
    }
    if (threadIdx.x == 0) {
        const uint64_t nr = run & 0xffffffffull, nc = run >> 32;
        // columns too small: the general decoder reports the capacity error
        if (nr > cap_rows || nc > cap_children) {
            atomicOr(&st->fast_fail, 1u);
        } else {
            st->n_rows = nr;
            st->n_children = nc;
            st->path = 4;  // the fast mixed decoder (mixed layout)
        }
    }
}

// emit: one wave per tile. The message starts come from the count / fix passes (bits per
// chunk), so the emit pass does not walk the chain again. Per round of 64 messages each lane
// decodes one: the header from 20 bytes at its start (length, id varint, tag and the 12 bytes
// after the tag), the value by val_decode; then the text of the round (ASCII per lane, the rest
// by the wave), the rows (64 consecutive per store), and the array elements: their starts by a
// walk per lane (by size), then one element per lane.
__global__ __launch_bounds__(TPB) void nxg_fmx_emit_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, const TileDesc* __restrict__ td,
    const uint64_t* __restrict__ tloc, const uint64_t* __restrict__ bpre,
    const uint64_t* __restrict__ starts, ColsDesc cols, DevStatus* __restrict__ st) {
    __shared__ __attribute__((aligned(16))) EmitLds lds[TPB / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t t = (uint64_t)blockIdx.x * (TPB / 64) + w;
    if (t >= nt) return;
#if NXG_FMX_PROF
    uint64_t _pt = __builtin_amdgcn_s_memtime();
    uint64_t _acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    uint8_t* img = lds[w].img;
    uint16_t* msg = lds[w].msg;
    uint32_t* el = lds[w].el;
    const lds_bytes limg = (lds_bytes)img;
    const uint64_t t0 = t * TILE;
    // message ends past this tile offset lie past the frame
    const uint32_t wend = (uint32_t)min<uint64_t>(W - t0, IMG);
    TileRegs g;
    tile_load(g, wire, t0, W, lane);
    uint64_t bits = starts[t * 64 + lane];
    const TileDesc d = td[t];
    // the chain: this tile is entered at its predecessor's exit (tile 0 at 0); the count pass
    // made the last tile end exactly at W
    const uint32_t px = t ? td[t - 1].exit : TILE;
    const uint64_t base = bpre[t / TPB] + tloc[t];
    const uint32_t nm = d.rows;
    const uint64_t rb = base & 0xffffffffull;
    uint64_t cnext = base >> 32;  // first child slot of this round's messages
    if (ld_agent32(&st->fast_fail)) return;
    tile_store(img, g, lane);
    // the message list in wire order
    const uint32_t n0 = (uint32_t)__popcll(bits);
    uint32_t at = wave_incl_scan<uint32_t>(n0) - n0;
    bool bad = d.entry == FAIL || px == FAIL || px - TILE != d.entry ||
               wave_last<uint32_t>(at + n0) != nm;
#pragma unroll 1
    while (bits) {
        msg[at++] = (uint16_t)(lane * CH + (uint32_t)__builtin_ctzll(bits));
        bits &= bits - 1;
    }
    wave_lds_order();
    PMARK(0);
    uint32_t ntxt = 0;  // deferred text checks in el[0, ntxt)
#pragma unroll 1
    for (uint32_t k = 0; k < nm && !bad; k += 64) {
        const uint32_t i = k + lane;
        const bool has = i < nm;
        const uint32_t p = has ? msg[i] : 0u;
        // header: length, Update variant (both checked by the count pass), id varint (at most
        // 5 bytes: the count pass), value tag, then the 12 bytes after the tag
        uint32_t h[5];
        win_words<5>(limg, p, h);
        const uint32_t lim = p + (h[0] & 0xffu);
        const uint32_t a = alignbyte(h[1], h[0], 2), b = alignbyte(h[2], h[1], 2);  // bytes 2..9
        const uint32_t sa = ~a & 0x80808080u;
        const uint32_t nb = sa ? ((uint32_t)__builtin_ctz(sa) >> 3) + 1 : 5u;
        const uint64_t id = (uint64_t)compress7_32(nb >= 4u ? a : (a & ((1u << (8u * nb)) - 1u))) |
                            (nb == 5u ? (uint64_t)(b & 0x7fu) << 28 : 0ull);
        const uint32_t tg = (uint32_t)(((((uint64_t)b << 32) | a) >> (8u * nb)) & 0xffu);
        const uint32_t u = 3u + nb;  // the payload, relative to p: 4..8
        const bool up = u >= 8u;
        const uint32_t g0 = up ? h[2] : h[1], g1 = up ? h[3] : h[2], g2 = up ? h[4] : h[3],
                       g3 = up ? 0u : h[4];
        const uint32_t su = u & 3u;
        FV o = val_decode(tg, alignbyte(g1, g0, su), alignbyte(g2, g1, su),
                          alignbyte(g3, g2, su), p + u, lim, true, t0);
        if (NXG_FMX_SKIP & 4) o = FV{g0, tg, g1, lim, 0, 0, 0, true};
        bool ok = !has || ((sa != 0u || !(b & 0x80u)) && u <= (lim - p) && lim <= wend && o.ok);
        PMARK(1);
        // text: the lanes with non-ASCII bytes are checked by the whole wave
        // text: checked once per tile (text_flush) from a list in `el`
        bad = __any(!ok);
        if (!bad && !(NXG_FMX_SKIP & 2)) {
            const bool tx = has && o.slen;
            const uint64_t tm = __ballot(tx);
            const uint32_t tn = (uint32_t)__popcll(tm);
            if (ntxt + tn > MAXC) {
                bad = !text_flush(limg, el, ntxt, lds[w].mark, lane, st);
                ntxt = 0;
                wave_lds_order();
            }
            if (tx) el[ntxt + __builtin_amdgcn_mbcnt_hi((uint32_t)(tm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)tm, 0u))] = o.soff | (o.slen << 16);
            ntxt += tn;
        }
        PMARK(2);
        if (bad) break;
        const uint32_t kd = has ? o.kids : 0u;
        const uint32_t kinc = wave_incl_scan<uint32_t>(kd);
        const uint32_t kpre = kinc - kd;
        const uint32_t rk = wave_last<uint32_t>(kinc);
        if (has && !(NXG_FMX_SKIP & 8)) {
            const uint64_t row = rb + i;
            cols.id[row] = id;
            cols.tag[row] = (uint8_t)o.tag;
            cols.fixed[row] = o.tag == 19u ? cnext + kpre : o.fixed;
            cols.aux[row] = o.aux;
        }
        PMARK(3);
        if (rk == 0 || (NXG_FMX_SKIP & 1)) {
            cnext += rk;
            continue;
        }
        // array elements (non-containers)
        // Array elements (non-containers). Stride path: an array whose first element has a fixed
        // size is taken to be all elements of that size; element j of the round is found from
        // its array (a max-scan over `mark`) and checked by its own tag. Any array that does not
        // fit (a variable-size element) sends the round to the exact walk below.
        bool strided = false;
        if (rk <= MAXC) {
            const uint32_t ep = o.end;
            const uint32_t f1a = kd && ep < lim ? fixed_size1(img[ep]) : 0u;
#if NXG_FMX_PROF
#endif
            if (!__any(kd && f1a == 0u)) {
                uint8_t* mark = lds[w].mark;
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
                        cols.ctag[slot] = (uint8_t)e.tag;
                        cols.cfixed[slot] = e.fixed;
                        cols.caux[slot] = e.aux;
                    }
                }
                wave_lds_order();
                if (bad) break;
            }
        }
        PMARK(4);
#if NXG_FMX_PROF
        _acc[7] += strided;
#endif
        if (!strided && ntxt) {  // the exact walk below uses el
            bad = !text_flush(limg, el, ntxt, lds[w].mark, lane, st);
            ntxt = 0;
            wave_lds_order();
            if (bad) break;
        }
        if (strided) {
        } else if (rk <= MAXC) {
            // element starts: a run of elements of the first one's fixed size is confirmed 8 at
            // a time from tags loaded together; other elements are sized by val_decode
            uint32_t ep = o.end;
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
            if (bad) break;
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
                    bad = __any(!eok) || !utf8_packed(limg, lds[w].mark, ena, e.soff, e.slen, lane);
                }
                if (bad) break;
                const uint64_t slot = cnext + j;
                if (he && slot < cols.cap_children) {
                    cols.ctag[slot] = (uint8_t)e.tag;
                    cols.cfixed[slot] = e.fixed;
                    cols.caux[slot] = e.aux;
                }
            }
            wave_lds_order();
        } else {  // more elements than the list holds: each lane decodes its own
            uint32_t ep = o.end;
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
                    cols.ctag[slot] = (uint8_t)e.tag;
                    cols.cfixed[slot] = e.fixed;
                    cols.caux[slot] = e.aux;
                }
                ep = e.end;
            }
            bad = __any(!ok);
        }
        PMARK(5);
        cnext += rk;
    }
#if NXG_FMX_PROF
    _acc[3] += (uint64_t)ntxt << 40;
#endif
    if (!bad && ntxt) bad = !text_flush(limg, el, ntxt, lds[w].mark, lane, st);
#if NXG_FMX_PROF
    _acc[6] = 1;
    _acc[4] = 0;
    _acc[5] = 0;
    if (lane == 0)
        for (int k = 0; k < 7; k++) atomicAdd(&st->diag[k], (unsigned long long)_acc[k]);
#endif
    if (bad && lane == 0) atomicOr(&st->fast_fail, 1u);
}

// ---- launch (host) --------------------------------------------------------------------------------
uint64_t nxg_fmx_tiles(uint64_t W) { return (W + TILE - 1) / TILE; }

uint64_t nxg_fmx_scratch_bytes(uint64_t W) {
    const uint64_t nt = nxg_fmx_tiles(W);
    // 2 descs 32 B, message starts 512 B, tloc 8 B per tile; bsum + bpre 16 B per 256 tiles;
    // alignment
    return nt * 552 + 16 * (nt / TPB + 1) + 6 * 16;
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
    uint64_t* tloc = reinterpret_cast<uint64_t*>(take(8 * nt));
    const uint64_t nb = (nt + TPB - 1) / TPB;
    uint64_t* bsum = reinterpret_cast<uint64_t*>(take(8 * nb));
    uint64_t* bpre = reinterpret_cast<uint64_t*>(take(8 * nb));
    constexpr uint64_t WV = TPB / 64;  // waves per workgroup
    // one tile per wave measured faster than persistent waves with the next tile prefetched
    // (count 184 vs 237 us, emit 534 vs 653 us at 10^7 records): the passes are bound by the
    // latency of their own LDS walks, which more resident waves hide better
    (void)wgs;
    const uint32_t gc = (uint32_t)((nt + WV - 1) / WV);
    hipLaunchKernelGGL(nxg_fmx_count_kernel, dim3(gc), dim3(TPB), 0, s, wire, W, nt, td, starts,
                       nxg_take_zero_slot());
    hipLaunchKernelGGL(nxg_fmx_resolve_kernel, dim3((uint32_t)nb), dim3(TPB), 0, s, wire, W, nt,
                       td, td2, starts, tloc, bsum, bpre, cols.cap_rows, cols.cap_children, st);
    hipLaunchKernelGGL(nxg_fmx_emit_kernel, dim3(gc), dim3(TPB), 0, s, wire, W, nt, td2, tloc,
                       bpre, starts, cols, st);
    return hipGetLastError();
}
