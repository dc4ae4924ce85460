// nxg_decode_mixed.hip -- the fast path of the mixed decode (config 3) for gfx950.
//
// Frames whose messages are From::Update(id, v) with a value that is a scalar, text, Decimal or
// an Array of non-container elements -- what a publisher of ordinary values sends -- and
// From::Heartbeat (02 05, kept as a control span, connection.rs:434) are decoded in two passes
// over 4 KiB tiles with no speculation across tiles beyond one checked guess. Length prefixes of
// one byte (messages < 128 bytes) and two bytes (< 16384: text values only, the text checked from
// global memory where it leaves the tile's image) are taken. Anything else (other control
// messages, Map / Error(Value) / Abstract values, nested containers, any content error) raises
// fast_fail and the host reruns the frame on the general decoder (nxg_decode_gen.hip), which
// covers every case and reports errors exactly. The values are decoded by the same restatement
// as the general path (nxg_msg.h dleaf / dcontainer), so the columns are identical.
//
// Message boundaries. A message at p ends at p + L (L the varint at p; canonical prefixes only),
// and a message start is a byte in [4, 127] followed by the Update variant (4), 02 05 (a
// Heartbeat), or a two-byte prefix (a byte >= 0x80, then one in [1, 127]) followed by 4. Per tile, each lane takes a 64-byte
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
#include <type_traits>

#include "nxg_fmx_common.h"

#ifndef NXG_FMX_CAND
#define NXG_FMX_CAND 7  // candidate rules (A/B timing only): 1 one-byte prefix, 2 Heartbeat, 4 two-byte
#endif
#ifndef NXG_FMX_CLS
#define NXG_FMX_CLS 1  // the emit's row values by class (row_value_cls), val_decode for the rest
#endif
#ifndef NXG_FF_CHECK
#define NXG_FF_CHECK 1  // emit waves skip a frame already declined
#endif
#ifndef NXG_FMX_LEAN
#define NXG_FMX_LEAN 1  // the emit's lean rounds for tiles of one-byte-prefix Updates (A/B: 0)
#endif
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



namespace {
using namespace fmx;
using namespace nxgmsg;

struct CountLds {  // count / fix passes
    uint8_t img[IMG];
};
#ifndef NXG_FMX_DEFER
#define NXG_FMX_DEFER 0  // 1: the emit gathers Array elements over rounds (defer_flush). Measured slower
// (config 3 at 10^7: 0.290-0.303 ms with the walk inlined, 0.54 ms out of line, against 0.253-0.268
// ms per round): the batch state spills the emit at 96 VGPRs (scratch 8 -> 52 bytes per lane)
#endif
constexpr uint32_t DMAXA = 64;  // deferred arrays per batch (a round's arrays fit one)
struct EmitLds {
    uint8_t img[IMG];
    uint16_t msg[MAXM];  // the tile's message starts
    uint32_t el[MAXC];   // a round's array elements: position | (message end - position) << 13
    uint8_t mark[256];   // utf8_packed
#if NXG_FMX_DEFER
    uint8_t emark[MAXC];    // deferred elements: array index + 1 at each array's first element
    // deferred arrays: first element | (message end - first element) << 13 | element size << 20
    // | batch index of the first element << 24
    uint32_t adesc[DMAXA];
#endif
};
// a workgroup's EmitLds in 32 KB: 5 workgroups per CU (NXG_FMX_EOCC)
static_assert(sizeof(EmitLds) * (TPB / 64) <= 32768, "emit LDS");

// candidate message starts in the lane's chunk: bit i = byte c+i starts an Update with a one-byte
// prefix (a byte in [4, 127], then 4) or a Heartbeat (02 05): the return value; or an Update with
// a two-byte prefix (a byte >= 0x80, a byte in [1, 127], then 4): `two`. The two-byte pattern is
// common inside ordinary messages (a two-byte id followed by value tag 4), so those candidates
// only ever continue a chain (chunk walks); the chunk's first two candidates, the tile's entry
// guesses and the chain scan use the one-byte ones (a chain through a long message is walked).
// The lanes' chunks are 64 bytes (16 banks) apart, so lane j reads its words in the order
// k + j / 2 (mod 16): at each step the 32 lanes of a half-wave read 32 different banks
// (ds_read_b32: bank = dword address mod 32), where the plain order put 16 lanes on one bank.
// FULL = false (a lean count): one-byte-prefix Update candidates only -- what most tiles of most
// frames hold; a tile with anything else then has no lean chain and is recounted by the resolve
// pass from every candidate kind.
template <bool FULL = true>
NXG_DEV uint64_t cand_mask(const uint8_t* img, uint32_t c, uint64_t& two) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(img + c);
    const uint32_t rot = (c >> 7) & 15u;  // (c / 64) / 2
    uint64_t m = 0;
    two = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t kk = ((uint32_t)k + rot) & 15u;
        const uint32_t a = w[kk], b = w[kk + 1];
        const uint32_t a1 = alignbyte(b, a, 1), a2 = alignbyte(b, a, 2);
        const uint32_t len = ((a & 0x7f7f7f7fu) + 0x7c7c7c7cu) & ~a & 0x80808080u;
        const uint32_t var = zero_bytes(a1 ^ 0x04040404u);
        if (FULL) {
            const uint32_t hb = zero_bytes(a ^ 0x02020202u) & zero_bytes(a1 ^ 0x05050505u);
            const uint32_t tw =
                a & ~a1 & ~zero_bytes(a1) & zero_bytes(a2 ^ 0x04040404u) & 0x80808080u;
            m |= (uint64_t)nib(((NXG_FMX_CAND & 1) ? (len & var) : 0u) |
                               ((NXG_FMX_CAND & 2) ? hb : 0u))
                 << (4 * kk);
            two |= (uint64_t)nib((NXG_FMX_CAND & 4) ? tw : 0u) << (4 * kk);
        } else {
            (void)a2;
            m |= (uint64_t)nib(len & var) << (4 * kk);
        }
    }
    return m;
}

#ifndef NXG_FMX_CM
#define NXG_FMX_CM 2  // candidate scan: 1 dword pairs in per-lane word order, 2 ds_read_b128 pieces
#endif
// 4 bits of x (flags at bits 7, 15, 23, 31 only) gathered into bits 28..31: the partial products
// of x * 0x00204081 land at distinct positions below 32, so nothing carries
NXG_DEV uint32_t nib4(uint32_t x) { return (x * 0x00204081u) >> 28; }
// cand_mask, reading the lane's chunk as four 16-byte pieces (ds_read_b128). Lane j takes piece
// (i + (j / 4) % 4) % 4 at step i: the 16 lanes of each ds_read_b128 lane group then cover the 64
// banks once (MI355X_MICROARCH.md LDS table), where the plain order is 4-way. The nibbles are
// placed in that rotated order (constant shifts) and the 64-bit mask rotated back once. The word
// after the chunk (the next chunk's first) comes from the next lane (DPP); lane 63 reads it.
template <bool FULL = true>
NXG_DEV uint64_t cand_mask_b128(const uint8_t* img, uint32_t lane, uint64_t& two) {
    const uint32_t c = lane * CH;
    const uint32_t r = (lane >> 2) & 3u;
    uint32_t P[4][4];
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
        const uint4 v = *reinterpret_cast<const uint4*>(img + c + 16u * ((i + r) & 3u));
        P[i][0] = v.x, P[i][1] = v.y, P[i][2] = v.z, P[i][3] = v.w;
    }
    // the chunk's first word is in the piece read at step (4 - r) % 4
    const uint32_t i0 = (4u - r) & 3u;
    const uint32_t w0 = i0 == 0 ? P[0][0] : (i0 == 1 ? P[1][0] : (i0 == 2 ? P[2][0] : P[3][0]));
    uint32_t w16 = wave_next(w0);
    if (lane == 63) w16 = *reinterpret_cast<const uint32_t*>(img + c + 64);
    uint32_t lo = 0, hi = 0, tlo = 0, thi = 0;
#pragma unroll
    for (uint32_t i = 0; i < 4; i++) {
        // the word after this piece: the next piece's first, or w16 after the chunk's last piece
        const uint32_t nx = i == 3u - r ? w16 : P[(i + 1) & 3][0];
#pragma unroll
        for (uint32_t e = 0; e < 4; e++) {
            const uint32_t a = P[i][e], b = e < 3 ? P[i][e + 1] : nx;
            const uint32_t a1 = alignbyte(b, a, 1);
            const uint32_t len = ((a & 0x7f7f7f7fu) + 0x7c7c7c7cu) & ~a & 0x80808080u;
            const uint32_t var = zero_bytes(a1 ^ 0x04040404u);
            uint32_t f = (NXG_FMX_CAND & 1) ? (len & var) : 0u, t = 0;
            if (FULL) {
                const uint32_t a2 = alignbyte(b, a, 2);
                if (NXG_FMX_CAND & 2) f |= zero_bytes(a ^ 0x02020202u) & zero_bytes(a1 ^ 0x05050505u);
                if (NXG_FMX_CAND & 4)
                    t = a & ~a1 & ~zero_bytes(a1) & zero_bytes(a2 ^ 0x04040404u) & 0x80808080u;
            }
            const uint32_t sh = 4u * (4u * i + e);  // a constant
            if (sh < 32) {
                lo |= nib4(f) << sh;
                if (FULL) tlo |= nib4(t) << sh;
            } else {
                hi |= nib4(f) << (sh - 32);
                if (FULL) thi |= nib4(t) << (sh - 32);
            }
        }
    }
    // rotate left by 16 r bits: r & 2 swaps the halves, r & 1 rotates by 16 (v_alignbit)
    auto rot = [&](uint32_t x, uint32_t y) -> uint64_t {
        if (r & 2u) {
            const uint32_t z = x;
            x = y;
            y = z;
        }
        if (r & 1u) {
            const uint32_t nl = __builtin_amdgcn_alignbit(x, y, 16), nh = __builtin_amdgcn_alignbit(y, x, 16);
            x = nl;
            y = nh;
        }
        return ((uint64_t)y << 32) | x;
    };
    two = FULL ? rot(tlo, thi) : 0ull;
    return rot(lo, hi);
}

// the length of the message at tile offset x (its canonical one- or two-byte prefix)
NXG_DEV uint32_t msg_len(const uint8_t* img, uint32_t x) {
    const uint32_t b0 = img[x];
    return b0 < 0x80u ? b0 : (b0 & 0x7fu) | ((uint32_t)img[x + 1] << 7);
}

// where the chain of messages from tile offset x (a candidate of chunk j) leaves the chunk, or
// FAIL (a position on the way is not a candidate start). `lim`: the tile's end in the frame
// (TILE, or less in the frame's last tile), where the chain stops.
NXG_DEV uint32_t chunk_exit(const uint8_t* img, uint32_t x, uint32_t j, uint64_t m, uint32_t lim) {
    const uint32_t end = min((j + 1) * CH, lim);
#pragma unroll 1
    for (int g = 0; g < 32 && x < end; g++) {
        if (!((m >> (x - j * CH)) & 1ull)) return FAIL;
        x += msg_len(img, x);
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

// per lane: the chunk's candidates (every kind), and the first two one-byte / Heartbeat
// candidates with their chunk exits
struct Cands {
    uint64_t m;
    uint32_t c0, x0, c1, x1;
};
template <bool FULL = true>
NXG_DEV Cands lane_cands(const uint8_t* img, uint32_t lane, uint32_t lim) {
    Cands r;
    uint64_t two;
    uint64_t m = NXG_FMX_CM == 2 ? cand_mask_b128<FULL>(img, lane, two)
                                 : cand_mask<FULL>(img, lane * CH, two);
    r.m = m | two;
    r.c0 = r.c1 = r.x0 = r.x1 = FAIL;
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

constexpr uint32_t GIVEUP = 0xfffffffdu;  // tile_chain_scan: too many resumes (tile_chain decides)
NXG_DEV SMap sconst(uint32_t st) { return SMap{st * 0x01010101u, st * 0x01010101u}; }

// The tile's chain from entry e (as tile_chain, without its serial loop over the chunks): from a
// resume point -- the entry, or where a message leaves the model (it lands more than two chunks
// on, or at a chunk's third candidate: long text) -- the chain is followed through that chunk
// exactly, then the state maps of the chunks after it are scanned; the first chunk whose chain
// leaves the model is the next resume point. A tile of short messages takes one scan, each long
// message one more. Returns the exit, FAIL (the chain breaks), or GIVEUP (more than 64 resumes).
NXG_DEV uint32_t tile_chain_scan(const uint8_t* img, uint32_t e, uint32_t lim, uint32_t lane,
                                 const Cands& cd, uint32_t& ce) {
    ce = NONE;
    const uint32_t c0 = cd.c0, x0 = cd.x0, c1 = cd.c1, x1 = cd.x1;
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
    if (e >= lim) return e;  // no message starts in this tile
    uint32_t sout = S_FAIL;            // the state behind the lane's chunk
    uint32_t cin = NONE, cout = FAIL;  // where the chain enters / leaves the lane's chunk
    uint32_t k = e >> 6, xs = e;       // the resume point: chunk k, entered at xs (uniform)
    bool done = false;
#pragma unroll 1
    for (int it = 0; it < 64 && !done; it++) {
        // the chain from xs through chunk k
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)c0, (int)k);
        const uint32_t a1 = (uint32_t)__builtin_amdgcn_readlane((int)c1, (int)k);
        uint32_t xe;
        if (xs == a0) {
            xe = (uint32_t)__builtin_amdgcn_readlane((int)x0, (int)k);
        } else if (xs == a1) {
            xe = (uint32_t)__builtin_amdgcn_readlane((int)x1, (int)k);
        } else {
            const uint32_t mlo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cd.m, (int)k);
            const uint32_t mhi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(cd.m >> 32), (int)k);
            xe = chunk_exit(img, xs, k, ((uint64_t)mhi << 32) | mlo, lim);
        }
        if (xe == FAIL) return FAIL;
        const uint32_t sk = (uint32_t)__builtin_amdgcn_readlane((int)out(xe), (int)k);
        if (lane == k) {
            cin = xs;
            cout = xe;
            sout = sk;
        }
        if (sk == S_END) {
            if (lane > k) sout = S_END;
            break;
        }
        if (sk == S_FAIL) {  // a long message (or a third candidate): resume where it lands
            k = xe >> 6;
            xs = xe;
            continue;
        }
        // the chunks after k: a scan of their maps from the state sk behind chunk k
        const SMap Tk = lane <= k ? sconst(sk) : T;
        const uint32_t so = sget(sscan(Tk), S_FAIL);
        const uint32_t si = dpp_fill<0x138, 0xf>(so, sk);  // the state in front of the chunk
        if (lane > k) {
            sout = so;
            cin = si == S_N0 ? c0 : (si == S_N1 ? c1 : NONE);
            cout = si == S_N0 ? x0 : (si == S_N1 ? x1 : FAIL);
        }
        // the first chunk after k whose chain leaves the model: the next resume point
        const uint64_t off = __ballot(lane > k && (si == S_N0 || si == S_N1) && so == S_FAIL);
        if (!off) {
            done = true;
            break;
        }
        const uint32_t l = (uint32_t)__builtin_ctzll(off);
        const uint32_t xl = (uint32_t)__builtin_amdgcn_readlane((int)cout, (int)l);
        if (xl == FAIL) return FAIL;
        if (lane > l) {
            sout = S_FAIL;
            cin = NONE;
            cout = FAIL;
        }
        k = xl >> 6;
        xs = xl;
    }
    if (!done && wave_last<uint32_t>(sout) != S_END) return GIVEUP;
    if (wave_last<uint32_t>(sout) != S_END) return FAIL;
    ce = cin;
    // the exit: the last start's chunk, whose state behind is the first END
    const uint64_t lm = __ballot(cin != NONE && sout == S_END);
    if (!lm) return FAIL;
    return (uint32_t)__builtin_amdgcn_readlane((int)cout, (int)__builtin_ctzll(lm));
}

// Header of the message at tile offset p: child slots (Array element count), HB for a
// Heartbeat, or FAIL when the message is not for the fast path. The value tag sits after the
// variant and the id varint; a message with a two-byte prefix must hold text.
constexpr uint32_t HB = 0xfffffffdu;
NXG_DEV uint32_t msg_kids(const uint8_t* img, uint32_t p) {
    const uint32_t b0 = img[p];
    if (b0 == 2u) return img[p + 1] == 5u ? HB : FAIL;  // Heartbeat (02 05)
    const uint32_t nbp = b0 < 0x80u ? 1u : 2u;
    const uint64_t w = win16((lds_bytes)img, p + nbp + 1).lo;  // id varint, tag, next byte
    const uint64_t stop = ~w & 0x8080808080808080ull;
    const uint32_t k = stop ? (uint32_t)__builtin_ctzll(stop) >> 3 : 8u;
    if (k >= 5) return FAIL;  // ids wider than 35 bits: the general decoder
    const uint32_t t = (uint32_t)(w >> (8 * k + 8)) & 0xffu;
    const uint32_t c = (uint32_t)(w >> (8 * k + 16)) & 0xffu;
    if (nbp == 2u) return (t == 12u || t == 13u || t == 18u || (t == 22u && c == 12u)) ? 0u : FAIL;
    if (t == 19) return c < 0x80u ? c : FAIL;
    if (t == 21 || t >= 28u) return FAIL;
    if (t == 22 && c != 12u) return FAIL;  // Error(Value) of a non-String
    return 0;
}

// the messages of the lane's chunk from its entry: Updates, Heartbeats, child slots, and their
// starts as bits of the chunk (bit i: chunk byte i)
NXG_DEV bool chunk_msgs(const uint8_t* img, uint32_t ce, uint32_t lane, uint32_t lim, uint32_t& n,
                        uint32_t& nhb, uint32_t& kids, uint64_t& bits, bool& two) {
    n = 0;
    nhb = 0;
    kids = 0;
    bits = 0;
    two = false;
    if (ce == NONE) return true;
    uint32_t x = ce;
    const uint32_t c = lane * CH, end = min(c + CH, lim);
#pragma unroll 1
    while (x < end) {
        const uint32_t k = msg_kids(img, x);
        if (k == FAIL) return false;
        bits |= 1ull << (x - c);
        two |= img[x] >= 0x80u;
        if (k == HB) {
            nhb++;
        } else {
            n++;
            kids += k;
        }
        x += msg_len(img, x);
    }
    return true;
}

#ifndef NXG_FMX_LEANMSGS
#define NXG_FMX_LEANMSGS 1
#endif
// chunk_msgs for a chain of the lean count: every position on it is a lean candidate (a one-byte
// prefix in [4, 127], then the Update variant), so no Heartbeat and no two-byte prefix; each
// message's length, id varint, tag and next byte come from one 12-byte window (two ds_read2_b32)
// instead of a byte read, a 20-byte window and another byte read. The same checks as msg_kids.
NXG_DEV bool chunk_msgs_lean(const uint8_t* img, uint32_t ce, uint32_t lane, uint32_t lim,
                             uint32_t& n, uint32_t& kids, uint64_t& bits) {
    n = 0;
    kids = 0;
    bits = 0;
    if (ce == NONE) return true;
    uint32_t x = ce;
    const uint32_t c = lane * CH, end = min(c + CH, lim);
#pragma unroll 1
    while (x < end) {
        uint32_t q[3];
        win_words<3>((lds_bytes)img, x, q);  // bytes x .. x + 11
        const uint32_t L = q[0] & 0xffu;
        // bytes x + 2 .. x + 9: the id varint (at most 5 bytes here), the tag, the byte after
        const uint64_t w = (uint64_t)__builtin_amdgcn_alignbyte(q[1], q[0], 2) |
                           ((uint64_t)__builtin_amdgcn_alignbyte(q[2], q[1], 2) << 32);
        const uint64_t stop = ~w & 0x8080808080808080ull;
        const uint32_t k = stop ? (uint32_t)__builtin_ctzll(stop) >> 3 : 8u;
        if (k >= 5) return false;  // ids wider than 35 bits: the general decoder
        const uint32_t t = (uint32_t)(w >> (8 * k + 8)) & 0xffu;
        const uint32_t cb = (uint32_t)(w >> (8 * k + 16)) & 0xffu;
        uint32_t kk = 0;
        if (t == 19u) {
            if (cb >= 0x80u) return false;
            kk = cb;
        } else if (t == 21u || t >= 28u || (t == 22u && cb != 12u)) {
            return false;
        }
        bits |= 1ull << (x - c);
        n++;
        kids += kk;
        x += L;
    }
    return true;
}

// The decoded range: `wire` is its first byte, W the bytes from there to the frame's end, R <= W
// the range's length (messages that START before R are the range's; the rest is read as
// look-ahead), base = the range's offset in the frame (text / control offsets are frame
// offsets), first = the range starts the frame (tile 0 is entered at 0; else its entry is
// guessed like any tile's). A whole frame: {W, W, 0, true}.
struct FRange {
    uint64_t W, R, base;
    bool first;
    // the end of tile t's messages (tile offset): the tile end, or the range's
    NXG_DEV uint32_t lim(uint64_t t) const {
        return (uint32_t)min<uint64_t>(TILE, R - t * TILE);
    }
    // the range's last tile, when the range ends the frame: its chain must end exactly there
    NXG_DEV bool last(uint64_t t, uint64_t nt) const { return t + 1 == nt && R == W; }
};

// tile descriptor (count pass -> resolve -> emit)
struct TileDesc {
    uint32_t entry, exit;  // tile offsets
    uint32_t rows;         // Updates | Heartbeats << 16
    uint32_t kids;         // child slots | kTwoByte (a message with a two-byte prefix)
};
constexpr uint32_t kTwoByte = 1u << 31;
// a tile of one-byte-prefix Updates only: the emit pass's lean variant
NXG_DEV bool lean_tile(const TileDesc& d) { return (d.rows >> 16) == 0 && !(d.kids & kTwoByte); }

// The tile's descriptor for the chain from entry e: exit, messages, child slots (FAIL entry and
// exit when the chain breaks, or does not end exactly at the frame end in the last tile).
// `bits`: the lane's message starts (chunk_msgs).
template <bool FULL = true>
NXG_DEV TileDesc count_from(const uint8_t* img, const Cands& cd, uint32_t e, uint32_t lim,
                            bool last, uint32_t lane, uint64_t& bits) {
    uint32_t ce;
    uint32_t x = tile_chain_scan(img, e, lim, lane, cd, ce);
    if (x == GIVEUP) x = tile_chain(img, e, lim, lane, cd.m, cd.c0, cd.x0, cd.c1, cd.x1, ce);
    bool bad = x == FAIL || (last && x != lim);
    uint32_t n = 0, h = 0, k = 0;
    bool two = false;
    bits = 0;
    if (!bad) {
        if (!FULL && NXG_FMX_LEANMSGS) bad = !chunk_msgs_lean(img, ce, lane, lim, n, k, bits);
        else bad = !chunk_msgs(img, ce, lane, lim, n, h, k, bits, two);
    }
    bad = __any(bad);
    if (bad) return TileDesc{FAIL, FAIL, 0, 0};
    const uint32_t nh = wave_sum<uint32_t>(n | (h << 16));
    // more messages than the emit pass's list holds (Heartbeats are 2 bytes): the general decoder
    if ((nh & 0xffffu) + (nh >> 16) > MAXM) return TileDesc{FAIL, FAIL, 0, 0};
    return TileDesc{e, x, nh, wave_sum<uint32_t>(k) | (__any(two) ? kTwoByte : 0u)};
}


}  // namespace

// The count pass for one tile (image in LDS). The entry of tile 0 is 0; any other tile guesses
// its entry: the first candidates of its first two chunks, in order, until one gives a complete
// chain. A false guess whose chain merges into the true one gives the true exit but wrong counts:
// the fix pass recounts such tiles from their predecessor's exit.
template <bool FULL>
NXG_DEV TileDesc count_tile(const uint8_t* img, uint64_t t, uint64_t nt, const FRange& rg,
                            uint32_t lane, uint64_t& bits) {
    const uint32_t lim = rg.lim(t);
    const bool last = rg.last(t, nt);
    const Cands cd = lane_cands<FULL>(img, lane, lim);
    TileDesc d{FAIL, FAIL, 0, 0};
    bits = 0;
    if (t == 0 && rg.first) return count_from<FULL>(img, cd, 0, lim, last, lane, bits);
    // the guesses: the first one-byte / Heartbeat candidates of chunks 0 and 1 (c0, c1)
    const uint32_t g00 = (uint32_t)__builtin_amdgcn_readlane((int)cd.c0, 0);
    const uint32_t g01 = (uint32_t)__builtin_amdgcn_readlane((int)cd.c1, 0);
    const uint32_t g10 = (uint32_t)__builtin_amdgcn_readlane((int)cd.c0, 1);
    const uint32_t g11 = (uint32_t)__builtin_amdgcn_readlane((int)cd.c1, 1);
    uint64_t mm = (g00 != FAIL ? 1ull << g00 : 0ull) | (g01 != FAIL ? 1ull << g01 : 0ull);
    uint64_t m1 = (g10 != FAIL ? 1ull << (g10 - CH) : 0ull) | (g11 != FAIL ? 1ull << (g11 - CH) : 0ull);
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
        d = count_from<FULL>(img, cd, g, lim, last, lane, bits);
    }
    if (d.entry == FAIL) {
        // chunks 0 and 1 hold no candidate (the tile starts inside a long text): the first
        // candidate of a later chunk, so that the tile needs no recount in the resolve pass
        const uint64_t cm = __ballot(cd.c0 != FAIL) & ~3ull;
        if (cm) {
            const uint32_t g = (uint32_t)__builtin_amdgcn_readlane((int)cd.c0, (int)__builtin_ctzll(cm));
            d = count_from<FULL>(img, cd, g, lim, last, lane, bits);
        }
    }
    if (FULL && d.entry != FAIL) {
        // a message with a two-byte prefix (long text) that ends where the guessed chain starts
        // is the tile's entry (the guesses use one-byte candidates only): the chain from there,
        // so that the tile needs no recount
        const uint32_t g = d.entry;
        uint32_t x2 = FAIL;
        if (lane <= (g >> 6)) {
#pragma unroll 1
            for (uint64_t m = cd.m; m; m &= m - 1) {
                const uint32_t p = lane * CH + (uint32_t)__builtin_ctzll(m);
                if (p >= g) break;
                if (img[p] >= 0x80u && p + msg_len(img, p) == g) {
                    x2 = p;
                    break;
                }
            }
        }
        x2 = wave_min_u32(x2);
        if (x2 != FAIL) {
            uint64_t b2;
            const TileDesc d2 = count_from(img, cd, x2, lim, last, lane, b2);
            if (d2.entry != FAIL) {
                d = d2;
                bits = b2;
            }
        }
    }
    return d;
}

// count pass: one wave per tile. MODE 0: the lean count (one-byte-prefix Update candidates);
// 1: every candidate kind; 2: the fix pass after either -- the tiles whose count found no chain (a
// lean count on a Heartbeat, a two-byte prefix, a long message) or whose guessed entry is not
// their predecessor's counted exit (a false guess that merged into the chain) are recounted, from
// that exit when it is known, all at once instead of one after another in the resolve pass's
// waves; each counted in DevStatus.diag[5] (`sz` is the call's status slot there, the zero slot
// otherwise). A predecessor being recounted at the same moment may be read before or after its
// rewrite: every descriptor written is a complete count from some entry, and the resolve pass
// checks the chain and recounts in order whatever still disagrees.
template <int MODE>
__global__ __launch_bounds__(TPB) void nxg_fmx_count_kernel(const uint8_t* __restrict__ wire,
                                                            FRange rg, uint64_t nt,
                                                            TileDesc* __restrict__ td,
                                                            uint64_t* __restrict__ starts,
                                                            DevStatus* sz) {
    constexpr bool FULL = MODE != 0;
    if (MODE != 2) zero_status(sz);
    __shared__ __attribute__((aligned(16))) CountLds lds[TPB / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t t = (uint64_t)blockIdx.x * (TPB / 64) + w;
    if (t >= nt) return;
    // (MODE 2) the predecessor's counted exit, when it enters this tile: the tile's entry
    uint32_t pe = FAIL;
    if (MODE == 2) {
        const uint32_t e = __builtin_amdgcn_readfirstlane(td[t].entry);
        if (t > 0) {
            const uint32_t px = __builtin_amdgcn_readfirstlane(td[t - 1].exit);
            if (px != FAIL && px - TILE < TILE) pe = px - TILE;
        }
        if (e != FAIL && (pe == FAIL || pe == e)) return;
        if (lane == 0) atomicAdd(&sz->diag[5], 1ull);
    }
    uint8_t* img = lds[w].img;
    TileRegs g;
    tile_load(g, wire, t * TILE, rg.W, lane);
    tile_store(img, g, lane);
    uint64_t bits;
    TileDesc d;
    if (MODE == 2 && pe != FAIL) {
        const Cands cd = lane_cands<true>(img, lane, rg.lim(t));
        d = count_from(img, cd, pe, rg.lim(t), rg.last(t, nt), lane, bits);
    } else {
        d = count_tile<FULL>(img, t, nt, rg, lane, bits);
    }
    starts[t * 64 + lane] = bits;
    if (lane == 0) td[t] = d;
}

// The fix pass with a lane per tile (NXG_FMX_FIXW): a wave checks 64 tiles -- entry against the
// predecessor's counted exit, as MODE 2 does per wave -- and recounts the ones that disagree one
// after another, so a frame that needs few recounts (42 at config 3's 10^7 records) launches 64x
// fewer waves than tiles. The same recount as MODE 2 (from the predecessor's exit when known,
// else every candidate kind); the resolve pass checks whatever still disagrees.
#ifndef NXG_FMX_FIXW
#define NXG_FMX_FIXW 1  // (A/B at 10^7: plain 0.2564-0.2578 vs 0.2577-0.2604 ms, the frame with control equal)
#endif
#ifndef NXG_FMX_FIXC
#define NXG_FMX_FIXC 0  // 1: the fix wave follows a recount's new exit into the tiles after it (measured
// slower: plain 0.261-0.262 vs 0.251-0.255, control 0.343-0.346 vs 0.337-0.338 ms; the recounts
// were 42 / 55 either way, no cascades)
#endif
__global__ __launch_bounds__(TPB) void nxg_fmx_fix_kernel(const uint8_t* __restrict__ wire, FRange rg,
                                                          uint64_t nt, TileDesc* __restrict__ td,
                                                          uint64_t* __restrict__ starts,
                                                          DevStatus* sz) {
    __shared__ __attribute__((aligned(16))) CountLds lds[TPB / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t t0 = ((uint64_t)blockIdx.x * (TPB / 64) + w) * 64;
    if (t0 >= nt) return;
    const uint64_t tl = t0 + lane;
    uint32_t pe = FAIL;
    bool redo = false;
    if (tl < nt) {
        const uint32_t e = td[tl].entry;
        if (tl > 0) {
            const uint32_t px = td[tl - 1].exit;
            if (px != FAIL && px - TILE < TILE) pe = px - TILE;
        }
        redo = !(e != FAIL && (pe == FAIL || pe == e));
    }
    uint8_t* img = lds[w].img;
#if NXG_FMX_FIXC
    // in tile order from the first tile to redo: a tile after a recounted one is recounted too
    // when its entry is not the new exit (the cascade the resolve pass would otherwise walk)
    const uint64_t m = __ballot(redo);
    uint32_t ex = tl < nt ? td[tl].exit : FAIL, en = tl < nt ? td[tl].entry : FAIL;
    bool chain = false;  // (uniform) the previous tile was recounted here
#pragma unroll 1
    for (uint32_t j = m ? (uint32_t)__builtin_ctzll(m) : 64u; j < 64u && t0 + j < nt; j++) {
        const uint64_t t = t0 + j;
        uint32_t pj = (uint32_t)__builtin_amdgcn_readlane((int)pe, (int)j);
        if (chain) {
            const uint32_t px = (uint32_t)__builtin_amdgcn_readlane((int)ex, (int)(j - 1));
            const uint32_t ej = (uint32_t)__builtin_amdgcn_readlane((int)en, (int)j);
            if (px != FAIL && px - TILE < TILE) {
                if (px - TILE == ej && !((m >> j) & 1ull)) {
                    chain = false;
                    continue;
                }
                pj = px - TILE;
            } else if (!((m >> j) & 1ull)) {
                chain = false;
                continue;
            }
        } else if (!((m >> j) & 1ull)) {
            continue;
        }
        chain = true;
#else
#pragma unroll 1
    for (uint64_t m = __ballot(redo); m; m &= m - 1) {
        const uint32_t j = (uint32_t)__builtin_ctzll(m);
        const uint64_t t = t0 + j;
        const uint32_t pj = (uint32_t)__builtin_amdgcn_readlane((int)pe, (int)j);
#endif
        if (lane == 0) atomicAdd(&sz->diag[5], 1ull);
        TileRegs g;
        tile_load(g, wire, t * TILE, rg.W, lane);
        tile_store(img, g, lane);
        uint64_t bits;
        TileDesc d;
        if (pj != FAIL) {
            const Cands cd = lane_cands<true>(img, lane, rg.lim(t));
            d = count_from(img, cd, pj, rg.lim(t), rg.last(t, nt), lane, bits);
        } else {
            d = count_tile<true>(img, t, nt, rg, lane, bits);
        }
        starts[t * 64 + lane] = bits;
        if (lane == 0) td[t] = d;
#if NXG_FMX_FIXC
        if (lane == j) {
            ex = d.exit;
            en = d.entry;
        }
#endif
    }
}

// The exit at which the chain leaves tile t - 1 (t >= 1), by the whole wave (uniform), from the
// count pass's descriptors: the last tile before t whose entry is its predecessor's exit keeps
// its exit; each tile after it passes the chain on -- a tile one long message covers entirely
// unchanged, a tile entered at its counted entry by its counted exit, and a tile entered
// elsewhere (a false guess, or the end of a long message) by a recount from its true entry, as
// the wave that owns it does. FAIL: the chain breaks on the way. Lets a wave's first tile see past
// the previous wave's recounts.
NXG_DEV uint32_t exit_before(const uint8_t* __restrict__ wire, const FRange& rg, uint64_t nt,
                             const TileDesc* td, uint64_t t, uint8_t* img, uint32_t lane) {
    const uint64_t W = rg.W;
    uint64_t k = t - 1;
#pragma unroll 1
    for (uint32_t back = 0; k > 0 && back < 64; back++, k--) {
        const uint32_t bx = td[k - 1].exit;
        if (bx != FAIL && bx - TILE == td[k].entry) break;
    }
    uint32_t x = td[k].exit;
#pragma unroll 1
    for (k = k + 1; k < t && x != FAIL; k++) {
        const uint32_t e = x - TILE;  // tile k's true entry
        if (e >= TILE) {
            x = e;  // covered: no message starts in tile k
            continue;
        }
        const TileDesc a = td[k];
        if (e == a.entry) {
            x = a.exit;
            continue;
        }
        const uint64_t t0 = k * TILE;
        const uint32_t lim = rg.lim(k);
        TileRegs g;
        tile_load(g, wire, t0, W, lane);
        tile_store(img, g, lane);
        const Cands cd = lane_cands(img, lane, lim);
        uint64_t bits;
        x = count_from(img, cd, e, lim, rg.last(k, nt), lane, bits).exit;
    }
    return x;
}

// resolve: everything between the count and the emit passes in one launch (no waiting on other
// workgroups). A lane per tile: a tile whose entry is not its predecessor's exit is recounted
// from that exit by its wave, tile by tile; then a block scan of (rows | child slots << 32) gives
// each tile its offset in the block (tloc), and the last block to arrive (a counter in the call's
// status slot, DevStatus.diag[7], zeroed with the slot) scans the block sums (bpre), checks the
// capacities and writes the totals. The chain (every entry its predecessor's exit) is checked by
// the emit pass. Frames are shorter than 2^32 bytes here, so both halves stay in 32 bits.
__global__ __launch_bounds__(TPB) void nxg_fmx_resolve_kernel(
    const uint8_t* __restrict__ wire, FRange rg, uint64_t nt, const TileDesc* __restrict__ td,
    TileDesc* __restrict__ td2, uint64_t* __restrict__ starts, uint64_t* __restrict__ tloc,
    uint64_t* __restrict__ bsum, uint64_t* __restrict__ bpre, uint64_t* __restrict__ wexit,
    uint64_t cap_rows,
    uint64_t cap_children, uint64_t cap_ctl, bool ctl_ok, DevStatus* __restrict__ st) {
    __shared__ __attribute__((aligned(16))) CountLds lds[TPB / 64];
    __shared__ uint64_t scan_tmp[TPB / 64];
    __shared__ uint32_t is_last;
    __shared__ uint32_t sh_tile;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // blocks by ticket (DevStatus.diag[6]): a wave waits only on waves that are running
    const uint32_t bid = next_tile(&st->diag[6], &sh_tile);
    const uint64_t tl = (uint64_t)bid * TPB + threadIdx.x;
    TileDesc d{FAIL, FAIL, 0, 0};
    bool mis = false;
    uint8_t* img = lds[w].img;
    // the exit the chain leaves the wave's previous tile at (FAIL: unknown), by the whole wave
    const uint64_t tw = tl - lane;  // the wave's first tile
    const uint64_t W = rg.W;
    uint32_t px0 = tw > 0 && tw < nt ? exit_before(wire, rg, nt, td, tw, img, lane) : FAIL;
    if (tw > 0 && tw < nt && px0 == FAIL) {
        // no tile of the count pass to start from within 64 (frames of long messages): the
        // previous wave's exit after its recounts, which it publishes below. Only lower-numbered
        // waves are waited on (dispatched earlier, so resident or done); on the watchdog the
        // emit pass's chain check fails the frame.
        const uint64_t t_start = rt_now();
        uint64_t v = ld_agent(&wexit[tw / 64 - 1]);
        uint32_t polls = 0;
#pragma unroll 1
        while (!(v >> 63) && !spin_expired(t_start, ++polls)) {
            __builtin_amdgcn_s_sleep(2);
            v = ld_agent(&wexit[tw / 64 - 1]);
        }
        px0 = (v >> 63) ? (uint32_t)v : FAIL;
        if (lane == 0) atomicAdd(&st->diag[4], 1ull);  // waves that waited (diagnostics)
    }
    if (tl < nt) {
        d = td[tl];
        if (tl > 0) {
            // (a failed predecessor fails the frame in the emit pass's chain check)
            const uint32_t px = lane == 0 ? px0 : td[tl - 1].exit;
            mis = px != FAIL && px - TILE != d.entry;
        }
    }
    const uint64_t m = __ballot(mis);
#if NXG_FMX_PROF
    if (lane == 0 && m) {
        atomicAdd(&st->diag[5], (unsigned long long)__popcll(m));
        atomicMax(&st->diag[4], (unsigned long long)__popcll(m));
    }
#endif
    if (m) {
        // in tile order from the first mismatch: a tile is recounted when its entry is not its
        // predecessor's exit as it stands after the predecessor's own recount (a long message
        // that covers whole tiles moves the exits of the tiles after it)
        const uint32_t j0 = (uint32_t)__builtin_ctzll(m);
#pragma unroll 1
        for (uint32_t j = j0; j < 64 && tw + j < nt; j++) {
            const uint64_t t = tw + j;
            const uint32_t px = j == 0 ? px0
                                       : (uint32_t)__builtin_amdgcn_readlane((int)d.exit, (int)(j - 1));
            const uint32_t ej = (uint32_t)__builtin_amdgcn_readlane((int)d.entry, (int)j);
            if (px == FAIL || px - TILE == ej) continue;
            const uint64_t t0 = t * TILE;
            const uint32_t lim = rg.lim(t);
            TileRegs g;
            tile_load(g, wire, t0, W, lane);
            tile_store(img, g, lane);
            const Cands cd = lane_cands(img, lane, lim);
            uint64_t bits;
            const TileDesc r = count_from(img, cd, px - TILE, lim, rg.last(t, nt), lane, bits);
            starts[t * 64 + lane] = bits;
            if (lane == j) d = r;
            if (lane == 0) atomicAdd(&st->diag[5], 1ull);  // recounted tiles (diagnostics)
        }
    }
    if (tl < nt) td2[tl] = d;
    {  // tiles holding a Heartbeat or a two-byte prefix (DevStatus.diag[0]: the host's choice of
       // count pass for the connection's next frame)
        const uint64_t nl = __ballot(tl < nt && !lean_tile(d));
        if (lane == 0 && nl) atomicAdd(&st->diag[0], (unsigned long long)__popcll(nl));
    }
    {  // the exit the chain leaves the wave's last tile at (FAIL: broken), for the next wave
        const uint32_t lx = (uint32_t)__builtin_amdgcn_readlane((int)d.exit, 63);
        if (lane == 0 && tw < nt) st_agent(&wexit[tw / 64], (1ull << 63) | lx);
    }
    // two scans: (Updates | child slots << 32) and Heartbeats
    const uint64_t v =
        tl < nt ? (uint64_t)(d.rows & 0xffffu) | ((uint64_t)(d.kids & ~kTwoByte) << 32) : 0ull;
    const uint64_t vh = tl < nt ? (uint64_t)(d.rows >> 16) : 0ull;
    uint64_t tot, toth;
    const uint64_t ex = block_excl_scan<uint64_t, TPB>(v, scan_tmp, &tot);
    const uint64_t exh = block_excl_scan<uint64_t, TPB>(vh, scan_tmp, &toth);
    if (tl < nt) {
        tloc[2 * tl] = ex;
        tloc[2 * tl + 1] = exh;
    }
    // the block sums go out with agent-scope stores and are drained before the arrival count
    // (an agent-scope fence would write back the XCD's L2, full of the count pass's output);
    // the last block reads the sums with agent-scope loads
    if (threadIdx.x == 0) {
        st_agent(&bsum[2 * bid], tot);
        st_agent(&bsum[2 * bid + 1], toth);
        drain_stores();
        is_last = atomicAdd(&st->diag[7], 1ull) == (unsigned long long)gridDim.x - 1;
    }
    __syncthreads();
    if (!is_last) return;
    const uint32_t nb = gridDim.x;
    uint64_t run = 0, runh = 0;
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < nb; b0 += TPB) {
        const uint32_t b = b0 + threadIdx.x;
        const uint64_t x = b < nb ? ld_agent(&bsum[2 * b]) : 0ull;
        const uint64_t xh = b < nb ? ld_agent(&bsum[2 * b + 1]) : 0ull;
        uint64_t t2, t2h;
        const uint64_t e2 = block_excl_scan<uint64_t, TPB>(x, scan_tmp, &t2);
        const uint64_t e2h = block_excl_scan<uint64_t, TPB>(xh, scan_tmp, &t2h);
        if (b < nb) {
            bpre[2 * b] = run + e2;
            bpre[2 * b + 1] = runh + e2h;
        }
        run += t2;
        runh += t2h;
    }
    if (threadIdx.x == 0) {
        const uint64_t nr = run & 0xffffffffull, nc = run >> 32;
        // columns too small: the general decoder reports the capacity error (a range decode
        // reports it itself: capacity set)
        if (nr > cap_rows || nc > cap_children || runh > cap_ctl || (runh && !ctl_ok)) {
            if (nr > cap_rows || nc > cap_children || runh > cap_ctl) st->capacity = 1u;
            atomicOr(&st->fast_fail, 1u);
        } else {
            st->n_rows = nr;
            st->n_children = nc;
            st->n_ctl = runh;
            st->n_heartbeat = runh;
            st->path = 4;  // the fast mixed decoder (mixed layout)
        }
    }
}

#if NXG_FMX_DEFER
// defer_flush's fallback, out of line (rare; its registers kept out of the emit's): lane a walks
// array a by val_decode, with the UTF-8 check per element. Returns this lane's ok.
#ifndef NXG_FMX_DWALK_NI
#define NXG_FMX_DWALK_NI 1
#endif
#if NXG_FMX_DWALK_NI
__device__ __noinline__
#else
NXG_DEV
#endif
bool defer_walk(EmitLds& L, uint32_t ne, uint32_t na, uint64_t cpend,
                                        const ColsDesc& cols, uint64_t t0f, uint32_t lane) {
    const lds_bytes limg = (lds_bytes)L.img;
    bool ok = true;
    if (lane < na) {
        const uint32_t dsc = L.adesc[lane], k0 = dsc >> 24;
        const uint32_t k1 = lane + 1u < na ? L.adesc[lane + 1u] >> 24 : ne;
        uint32_t ep = dsc & 0x1fffu;
        const uint32_t lim = ep + ((dsc >> 13) & 127u);
#pragma unroll 1
        for (uint32_t c = k0; ok && c < k1; c++) {
            ok = ep < lim;
            if (!ok) break;
            const uint32_t et = L.img[ep];
            uint32_t q[3];
            win_words<3>(limg, ep + 1, q);
            const FV e = val_decode(et, q[0], q[1], q[2], ep + 1, lim, false, t0f);
            ok = e.ok && (!e.slen || utf8_ok(LdsSrc{limg, t0f}, t0f + e.soff, e.slen));
            const uint64_t slot = cpend + c;
            if (ok && slot < cols.cap_children) {
                col_st(&cols.ctag[slot], (uint8_t)e.tag);
                col_st(&cols.cfixed[slot], (uint64_t)e.fixed);
                col_st(&cols.caux[slot], (uint32_t)e.aux);
            }
            ep = e.end;
        }
    }
    return ok;
}

// The deferred Array elements of a tile: ne elements of na arrays gathered over rounds (each
// array's first element of a fixed size), batch element j in slot cpend + j, one element per
// lane: its array from a max-scan over emark, its position from the array's stride, checked by
// its own tag (as round_elements' stride path, over up to 256 elements of several rounds instead
// of one round's). An array whose elements differ in size sends the batch to a walk per lane
// (lane a: array a, val_decode and the UTF-8 check per element). emark is left zero. Returns
// true (uniform) on a decode error.
NXG_DEV bool defer_flush(EmitLds& L, uint32_t ne, uint32_t na, uint64_t cpend,
                         const ColsDesc& cols, uint64_t t0f, uint32_t lane) {
    const lds_bytes limg = (lds_bytes)L.img;
    bool bad = false, strided = true;
    uint32_t carry = 0;
    wave_lds_order();
#pragma unroll 1
    for (uint32_t j0 = 0; j0 < ne; j0 += 64) {
        const uint32_t j = j0 + lane;
        const bool he = j < ne;
        // emark[0] is set (the batch's first array starts it): a1 >= 1 on every lane
        const uint32_t a1 = max(wave_max_scan(he ? (uint32_t)L.emark[j] : 0u), carry);
        carry = wave_last<uint32_t>(a1);
        const uint32_t dsc = L.adesc[a1 - 1u];
        const uint32_t fa = (dsc >> 20) & 15u, k0 = dsc >> 24, ep = dsc & 0x1fffu;
        const uint32_t e0 = he ? ep + (j - k0) * fa : 8u;
        const uint32_t elim = he ? ep + ((dsc >> 13) & 127u) : 16u;
        uint32_t q[4];
        win_words<4>(limg, e0, q);
        const uint32_t et = q[0] & 0xffu;
        if (!__all(!he || (e0 < elim && fixed_size1(et) == fa))) {
            strided = false;
            break;
        }
        FV e;
        if (__all(!he || simple_fixed(et))) e = fixed_elem(q, e0, elim);  // scalars only
        else  // DateTime / Duration elements
            e = val_decode(et, alignbyte(q[1], q[0], 1), alignbyte(q[2], q[1], 1),
                           alignbyte(q[3], q[2], 1), e0 + 1, elim, false, t0f);
        bad = __any(he && !e.ok);
        if (bad) break;
        const uint64_t slot = cpend + j;
        if (he && slot < cols.cap_children) {
            col_st(&cols.ctag[slot], (uint8_t)e.tag);
            col_st(&cols.cfixed[slot], (uint64_t)e.fixed);
            col_st(&cols.caux[slot], (uint32_t)e.aux);
        }
    }
    if (!strided) bad = __any(!defer_walk(L, ne, na, cpend, cols, t0f, lane));
    wave_lds_order();
    if (lane < na) L.emark[L.adesc[lane] >> 24] = 0;
    wave_lds_order();
    return bad;
}
#endif

// emit: one wave per tile. The message starts come from the count / fix passes (bits per
// chunk), so the emit pass does not walk the chain again. Per round of 64 messages each lane
// decodes one: the header from 20 bytes at its start (length, id varint, tag and the 12 bytes
// after the tag), the value by val_decode; then the text of the round (ASCII per lane, the rest
// by the wave), the rows (64 consecutive per store), and the array elements: their starts by a
// walk per lane (by size), then one element per lane.
#ifndef NXG_FMX_EOCC
#define NXG_FMX_EOCC 5  // waves per SIMD asked of the emit's register allocation (LDS allows 5; A/B 0.258 vs 0.273 ms)
#endif
__global__ __launch_bounds__(TPB, NXG_FMX_EOCC) void nxg_fmx_emit_kernel(
    const uint8_t* __restrict__ wire, FRange rg, uint64_t nt, const TileDesc* __restrict__ td,
    const uint64_t* __restrict__ tloc, const uint64_t* __restrict__ bpre,
    const uint64_t* __restrict__ starts, ColsDesc cols, bool ctl_on, DevStatus* __restrict__ st) {
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
    const uint64_t W = rg.W;
    const uint64_t t0 = t * TILE;
    const uint64_t t0f = rg.base + t0;  // the tile's offset in the frame (text, control spans)
    // message ends past this tile offset lie past the frame
    const uint32_t wend = (uint32_t)min<uint64_t>(W - t0, IMG);
    TileRegs g;
    tile_load(g, wire, t0, W, lane);
    uint64_t bits = starts[t * 64 + lane];
    const TileDesc d = td[t];
    // the chain: this tile is entered at its predecessor's exit (tile 0 at 0); the count pass
    // made the last tile end exactly at W
    // (a range that does not start the frame: tile 0 is entered at its counted entry, which the
    // caller links with the previous range's exit)
    const uint32_t px = t ? td[t - 1].exit : (rg.first ? TILE : TILE + d.entry);
    if (lane == 0 && t == 0) st->diag[2] = (uint64_t)d.entry + 1;  // the range's entry (+1)
    if (lane == 0 && t + 1 == nt) st->diag[3] = t0 + d.exit + 1;  // its exit (+1)
    const uint64_t base = bpre[2 * (t / TPB)] + tloc[2 * t];
    uint64_t hnext = bpre[2 * (t / TPB) + 1] + tloc[2 * t + 1];  // next ctl slot (Heartbeats)
    const uint32_t nm = (d.rows & 0xffffu) + (d.rows >> 16);    // Updates + Heartbeats
    uint64_t rnext = base & 0xffffffffull;  // next row
    uint64_t cnext = base >> 32;  // first child slot of this round's messages
    // message ends past this tile offset lie past the frame (long text is checked from global
    // memory where it leaves the image)
    const uint32_t fend = (uint32_t)min<uint64_t>(W - t0, 0xffffffffull);
    // a frame already declined by the resolve pass (a plain read: one scalar load per CU, not an
    // agent-scope load per wave on one address)
    if (NXG_FF_CHECK && st->fast_fail) return;
    tile_store(img, g, lane);
#if NXG_FMX_DEFER
    reinterpret_cast<uint32_t*>(lds[w].emark)[lane] = 0u;
    static_assert(MAXC == 256, "emark: a word per lane");
#endif
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
    // the rounds, in a lean variant for tiles of one-byte-prefix Updates only (no Heartbeat, no
    // two-byte prefix, no text past the image: most tiles), chosen per tile
    auto rounds = [&](auto lean_c) {
        constexpr bool LEAN = decltype(lean_c)::value;
        uint32_t ntxt = 0;  // deferred text checks in el[0, ntxt)
        uint32_t pe = 0, pa = 0;  // deferred elements and arrays (NXG_FMX_DEFER)
        uint64_t cpend = 0;       // the first deferred element's slot
    #pragma unroll 1
        for (uint32_t k = 0; k < nm && !bad; k += 64) {
            const uint32_t i = k + lane;
            const bool has = i < nm;
            const uint32_t p0 = has ? msg[i] : 0u;
            // a Heartbeat (02 05, checked by the count pass): a control span before the next row
            const uint32_t c0 = img[p0];
            const bool ishb = !LEAN && has && c0 == 2u;
            const bool upd = has && !ishb;
            const uint64_t hm = LEAN ? 0ull : __ballot(ishb);
            const uint32_t hbefore = LEAN ? 0u : __builtin_amdgcn_mbcnt_hi((uint32_t)(hm >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)hm, 0u));
            const uint64_t row = rnext + (lane - hbefore);  // Updates before this lane in the round
            if (ishb && ctl_on) {
                const uint64_t c = hnext + hbefore;
                cols.ctl_row[c] = row;
                cols.ctl_off[c] = t0f + p0;
                cols.ctl_len[c] = 2u;
                cols.ctl_variant[c] = 5u;
            }
            // header: length (one or two bytes), Update variant (both checked by the count pass), id
            // varint (at most 5 bytes: the count pass), value tag, then the 12 bytes after the tag;
            // read from p, the last length byte
            const uint32_t nbp = LEAN || c0 < 0x80u ? 1u : 2u;
            const uint32_t p = p0 + nbp - 1u;
            uint32_t h[5];
            win_words<5>(limg, p, h);
            const uint32_t lim = p0 + (nbp == 1u ? c0 : (c0 & 0x7fu) | ((h[0] & 0xffu) << 7));
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
            const uint32_t V0 = alignbyte(g1, g0, su), V1 = alignbyte(g2, g1, su),
                           V2 = alignbyte(g3, g2, su);
            FV o;
            if (!NXG_FMX_CLS || !row_value_cls(upd ? tg : 1u, V0, V1, V2, p + u,
                                               upd ? lim : p + u + 12u, t0f, upd, o))
                o = val_decode(upd ? tg : 1u, V0, V1, V2, p + u, upd ? lim : p + u + 12u, true, t0f);
            if (NXG_FMX_SKIP & 4) o = FV{g0, tg, g1, lim, 0, 0, 0, true};
            // past the image: text only (the count pass), checked here from global memory
            const bool far = !LEAN && upd && lim > wend;
            bool ok = !upd || ((sa != 0u || !(b & 0x80u)) && u <= (lim - p) && lim <= fend && o.ok);
            if (!LEAN) {  // (text past the image: the whole wave, one text after the other)
                const bool fw = far && ok && o.slen;
                const bool fo = far_text_ok(wire, fw, t0 + o.soff, o.slen, lane);
                if (fw) ok = fo;
            }
            PMARK(1);
            // text: checked once per tile (text_flush) from a list in `el`
            bad = __any(!ok);
            if (!bad && !(NXG_FMX_SKIP & 2)) {
                const bool tx = upd && !far && o.slen;
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
            const uint32_t kd = upd ? o.kids : 0u;
            const uint32_t kinc = wave_incl_scan<uint32_t>(kd);
            const uint32_t kpre = kinc - kd;
            const uint32_t rk = wave_last<uint32_t>(kinc);
            {
                const uint32_t nh = (uint32_t)__popcll(hm);
                rnext += min(nm - k, 64u) - nh;
                hnext += nh;
            }
            if (upd && !(NXG_FMX_SKIP & 8)) {
                col_st(&cols.id[row], (uint64_t)id);
                col_st(&cols.tag[row], (uint8_t)o.tag);
                col_st(&cols.fixed[row], (uint64_t)(o.tag == 19u ? cnext + kpre : o.fixed));
                col_st(&cols.aux[row], (uint32_t)o.aux);
            }
            PMARK(3);
#if NXG_FMX_DEFER
            if (NXG_FMX_SKIP & 1) {
                cnext += rk;
                continue;
            }
            {
                // a round whose every array starts with a fixed-size element joins the batch (a
                // round without arrays too); the batch is flushed before a round that does not fit
                // or join it and after the tile's last round (one call site: defer_flush inlined
                // once)
                const uint32_t f1a = kd && o.end < lim ? fixed_size1(img[o.end]) : 0u;
                const uint64_t am = __ballot(kd != 0u);
                const uint32_t narr = (uint32_t)__popcll(am);
                const bool join = !__any(kd && (f1a == 0u || lim - o.end > 127u || o.end > 0x1fffu)) && rk <= MAXC;
                const bool last = k + 64u >= nm;
                bool app = false;
    #pragma unroll 1
                for (;;) {
                    if (pe && (app ? last : (!join || pe + rk > MAXC || pa + narr > DMAXA))) {
                        bad = defer_flush(lds[w], pe, pa, cpend, cols, t0f, lane);
                        pe = pa = 0;
                        if (bad) break;
                    }
                    if (app || !join) break;
                    if (pe == 0) cpend = cnext;
                    if (kd) {
                        const uint32_t ai = pa + __builtin_amdgcn_mbcnt_hi(
                                                     (uint32_t)(am >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
                        lds[w].adesc[ai] = o.end | ((lim - o.end) << 13) | (f1a << 20) |
                                           ((pe + kpre) << 24);
                        lds[w].emark[pe + kpre] = (uint8_t)(ai + 1u);
                    }
                    pe += rk;
                    pa += narr;
                    app = true;
                }
                if (bad) break;
                if (join) {
                    cnext += rk;
                    PMARK(5);
                    continue;
                }
            }
#else
            if (rk == 0 || (NXG_FMX_SKIP & 1)) {
                cnext += rk;
                continue;
            }
#endif
            bad = round_elements(img, lds[w].mark, el, kd, kpre, rk, o.end, lim, cnext, cols, t0f, lane,
                                 ntxt, st);
            if (bad) break;
            PMARK(5);
            cnext += rk;
        }
    #if NXG_FMX_PROF
        _acc[3] += (uint64_t)ntxt << 40;
    #endif
        if (!bad && ntxt) bad = !text_flush(limg, el, ntxt, lds[w].mark, lane, st);
    };
    if (NXG_FMX_LEAN && lean_tile(d)) rounds(std::integral_constant<bool, true>{});
    else rounds(std::integral_constant<bool, false>{});
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
    // 2 descs 32 B, message starts 512 B, tloc 16 B per tile; bsum + bpre 32 B per 256 tiles;
    // one exit word per 64 tiles; alignment
    return nt * 560 + 32 * (nt / TPB + 1) + 8 * (nt / 64 + 1) + 7 * 16;
}

// persistent grids: every workgroup co-resident (count: [0], emit: [1])
void nxg_fmx_wgs(int ncu, int* wgs) {
    int a = 0, b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, nxg_fmx_count_kernel<1>, TPB, 0) !=
            hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, nxg_fmx_emit_kernel, TPB, 0) != hipSuccess) {
        a = b = 1;
    }
    wgs[0] = std::max(1, a) * ncu;
    wgs[1] = std::max(1, b) * ncu;
}

// The messages that start in [begin, end) of a frame of W bytes (a whole frame: 0, W); rows,
// children and control spans numbered from 0, text and control offsets in frame bytes; the
// range's entry / exit (+1, relative to begin) in DevStatus.diag[2] / diag[3].
hipError_t nxg_launch_dec_fmx_range(const uint8_t* wire, uint64_t W, uint64_t begin, uint64_t end,
                                    const ColsDesc& cols, uint8_t* scratch, const int* wgs,
                                    DevStatus* st, hipStream_t s, bool lean_count) {
    if (begin > end || end > W) return hipErrorInvalidValue;
    const FRange rg{W - begin, end - begin, begin, begin == 0};
    wire += begin;
    const uint64_t nt = nxg_fmx_tiles(rg.R);
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
    uint64_t* tloc = reinterpret_cast<uint64_t*>(take(16 * nt));
    const uint64_t nb = (nt + TPB - 1) / TPB;
    uint64_t* bsum = reinterpret_cast<uint64_t*>(take(16 * nb));
    uint64_t* bpre = reinterpret_cast<uint64_t*>(take(16 * nb));
    const uint64_t nwv = (nt + 63) / 64;
    uint64_t* wexit = reinterpret_cast<uint64_t*>(take(8 * nwv));
    hipError_t e = hipMemsetAsync(wexit, 0, 8 * nwv, s);
    if (e != hipSuccess) return e;
    constexpr uint64_t WV = TPB / 64;  // waves per workgroup
    // one tile per wave measured faster than persistent waves with the next tile prefetched
    // (count 184 vs 237 us, emit 534 vs 653 us at 10^7 records): the passes are bound by the
    // latency of their own LDS walks, which more resident waves hide better
    (void)wgs;
    const uint32_t gc = (uint32_t)((nt + WV - 1) / WV);
    if (lean_count) {
        hipLaunchKernelGGL(nxg_fmx_count_kernel<0>, dim3(gc), dim3(TPB), 0, s, wire, rg, nt, td,
                           starts, nxg_take_zero_slot());
        if (NXG_FMX_FIXW)
            hipLaunchKernelGGL(nxg_fmx_fix_kernel, dim3((uint32_t)((nt + 64 * WV - 1) / (64 * WV))),
                               dim3(TPB), 0, s, wire, rg, nt, td, starts, st);
        else
            hipLaunchKernelGGL(nxg_fmx_count_kernel<2>, dim3(gc), dim3(TPB), 0, s, wire, rg, nt,
                               td, starts, st);
    } else {
        hipLaunchKernelGGL(nxg_fmx_count_kernel<1>, dim3(gc), dim3(TPB), 0, s, wire, rg, nt, td,
                           starts, nxg_take_zero_slot());
        if (NXG_FMX_FIXW)
            hipLaunchKernelGGL(nxg_fmx_fix_kernel, dim3((uint32_t)((nt + 64 * WV - 1) / (64 * WV))),
                               dim3(TPB), 0, s, wire, rg, nt, td, starts, st);
        else
            hipLaunchKernelGGL(nxg_fmx_count_kernel<2>, dim3(gc), dim3(TPB), 0, s, wire, rg, nt,
                               td, starts, st);
    }
    const bool ctl_on = cols.ctl_row && cols.ctl_off && cols.ctl_len && cols.ctl_variant;
    hipLaunchKernelGGL(nxg_fmx_resolve_kernel, dim3((uint32_t)nb), dim3(TPB), 0, s, wire, rg, nt,
                       td, td2, starts, tloc, bsum, bpre, wexit, cols.cap_rows, cols.cap_children,
                       cols.cap_ctl, ctl_on, st);
    hipLaunchKernelGGL(nxg_fmx_emit_kernel, dim3(gc), dim3(TPB), 0, s, wire, rg, nt, td2, tloc,
                       bpre, starts, cols, ctl_on, st);
    return hipGetLastError();
}

hipError_t nxg_launch_dec_fmx(const uint8_t* wire, uint64_t W, const ColsDesc& cols,
                              uint8_t* scratch, const int* wgs, DevStatus* st, hipStream_t s,
                              bool lean_count) {
    return nxg_launch_dec_fmx_range(wire, W, 0, W, cols, scratch, wgs, st, s, lean_count);
}
