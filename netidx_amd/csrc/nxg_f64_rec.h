// nxg_f64_rec.h -- canonical f64 Update records on the wire, and the tile machinery shared by
// the f64 decode kernels (nxg_decode_f64.hip).
//
// Every From::Update(Id, F64) message is canonical on the wire:
//     varint(L) 04 varint(id) 09 f64be      L = lw(10 + vl(id)) = 11 + nb,  nb = vl(id) in 1..4
// (len_wrapped_encode pack.rs:527-535, derive lib.rs:289-381, Value::encode lib.rs:404-407).
//
// Finding record boundaries without a sequential walk ("merge points")
// ---------------------------------------------------------------------
// Each lane owns a 64-byte chunk [c, c+64). Records are at most 15 bytes, so the first record
// that starts at or after c lies in [c, c+15). Every position p in that window whose 16 bytes
// form a valid record starts a "walk" (p, p+L(p), ...). The walks are advanced in position
// order until they all coincide; that common position is the chunk's merge point X(c). The
// true record chain passes through one of the window's positions, so it also passes through
// X(c). The merge point depends only on the bytes, so the lane that owns chunk c-64 computes
// the same value when it finishes its own chunk.
//
// Lane j decodes exactly the records that start in [X_j, X_{j+1}). Its walk from X_j must land
// exactly on X_{j+1}, and every record on the way must be a valid f64 Update. If any of these
// checks fails, or the walks do not merge within 64 bytes, the frame is not (provably)
// homogeneous-f64. The kernel then raises DevStatus.fast_fail, and the host reruns the frame on
// the general kernel. The fast path never silently mis-decodes.
#pragma once
#include "nxg_device.h"

using namespace f64dec;

namespace {

constexpr uint32_t FAIL = 0xffffffffu;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // first-class vector: no memcpy

// 16 bytes at tile-relative byte `rel` (any alignment) as four little-endian dwords.
NXG_DEV void load16(const uint8_t* buf, uint32_t rel, uint32_t& e0, uint32_t& e1, uint32_t& e2,
                    uint32_t& e3) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(buf + (rel & ~3u));
    const uint32_t s = rel & 3u;
    const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
    e0 = alignbyte(d1, d0, s);
    e1 = alignbyte(d2, d1, s);
    e2 = alignbyte(d3, d2, s);
    e3 = alignbyte(d4, d3, s);
}

// Valid canonical f64 Update record in the first bytes e0,e1? Returns its length L or 0.
// `rem` = bytes from the record start to the end of the frame.
NXG_DEV uint32_t rec_check(uint32_t e0, uint32_t e1, uint64_t rem) {
    const uint32_t L = e0 & 0xffu;
    if (L - 12u > 3u) return 0;                  // 1-byte varint L in 12..15
    if (((e0 >> 8) & 0xffu) != 4u) return 0;     // From::Update
    if (rem < L) return 0;
    const uint32_t nb = L - 11u;                 // id varint bytes
    const uint32_t x = alignbyte(e1, e0, 2);     // bytes 2..5
    const uint32_t m = nb == 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u);
    const uint32_t want = 0x80808080u & ((1u << (8 * (nb - 1))) - 1u);
    if (((x & 0x80808080u) & m) != want) return 0;  // exactly nb varint bytes
    const uint64_t q = ((uint64_t)e1 << 32) | e0;
    if (((q >> (8 * (2 + nb))) & 0xffu) != 9u) return 0;  // Value::F64
    return L;
}

// rec_check without branches (the same checks): `rem` = bytes from the record start to the end
// of the frame, saturated to 32 bits.
NXG_DEV uint32_t rec_check32(uint32_t e0, uint32_t e1, uint32_t rem) {
    const uint32_t L = e0 & 0xffu;
    const bool head = (e0 & 0xfffcu) == 0x040cu;        // L in 12..15, then From::Update
    const uint32_t sh = 8u * ((L & 3u) + 1u);           // 8 * nb (nb = L - 11 when head)
    const uint32_t m = 0xffffffffu >> (32u - sh);       // the nb id bytes
    const uint32_t x = alignbyte(e1, e0, 2);            // bytes 2..5
    const bool var = (x & 0x80808080u & m) == (0x80808080u & (m >> 8));  // exactly nb bytes
    const uint32_t tag = __builtin_amdgcn_ubfe(alignbyte(e1, e0, 3), sh - 8u, 8u);  // byte 2+nb
    return (head && var && tag == 9u && rem >= L) ? L : 0u;
}

NXG_DEV void rec_decode(uint32_t e0, uint32_t e1, uint32_t e2, uint32_t e3, uint32_t L,
                        uint64_t& id, uint64_t& val) {
    const uint32_t nb = L - 11u;
    const uint32_t m = nb == 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u);
    const uint32_t xb = alignbyte(e1, e0, 2) & m;
    id = (xb & 0x7fu) | ((xb >> 1) & (0x7fu << 7)) | ((xb >> 2) & (0x7fu << 14)) |
         ((xb >> 3) & (0x7fu << 21));
    const uint32_t lo = alignbyte(e2, e1, nb - 1);  // value bytes 0..3 (wire order)
    const uint32_t hi = alignbyte(e3, e2, nb - 1);  // value bytes 4..7
    val = ((uint64_t)bswap32(lo) << 32) | bswap32(hi);  // big-endian f64 (pack.rs:592-598)
}


// Merge point of all record walks starting in [r, r+15) (tile-relative). r is 4-aligned;
// d0..d4 are the 20 bytes at r (the candidate mask comes from them; the candidates' records and
// the walks are read from the LDS image `buf`).
NXG_DEV uint32_t merge_point_d(const uint8_t* buf, uint32_t r, uint64_t t0, uint64_t W,
                               uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t d4) {
    const uint64_t abs_r = t0 + r;
    if (abs_r >= W) return (uint32_t)(W - t0);  // chunk past the end: the END position
    const uint64_t remr = W - abs_r;
    // candidate starts: byte in 12..15 followed by 0x04
    const uint32_t a = nib(zero_bytes((d0 & 0xfcfcfcfcu) ^ 0x0c0c0c0cu)) |
                       (nib(zero_bytes((d1 & 0xfcfcfcfcu) ^ 0x0c0c0c0cu)) << 4) |
                       (nib(zero_bytes((d2 & 0xfcfcfcfcu) ^ 0x0c0c0c0cu)) << 8) |
                       (nib(zero_bytes((d3 & 0xfcfcfcfcu) ^ 0x0c0c0c0cu)) << 12);
    const uint32_t b = nib(zero_bytes(d0 ^ 0x04040404u)) | (nib(zero_bytes(d1 ^ 0x04040404u)) << 4) |
                       (nib(zero_bytes(d2 ^ 0x04040404u)) << 8) |
                       (nib(zero_bytes(d3 ^ 0x04040404u)) << 12) |
                       (nib(zero_bytes(d4 ^ 0x04040404u)) << 16);
    uint32_t cand = a & (b >> 1) & 0x7fffu;
    uint64_t S = 0;
    if (remr < 15) S |= 1ull << remr;  // the frame end is a valid (terminal) position
    while (cand) {
        const uint32_t p = __builtin_ctz(cand);
        cand &= cand - 1;
        uint32_t e0, e1, e2, e3;
        load16(buf, r + p, e0, e1, e2, e3);
        if (rec_check(e0, e1, remr - p)) S |= 1ull << p;
    }
    // advance the lowest walk until one remains; walks that hit an invalid record die
    for (int it = 0; it < WIN && __popcll(S) > 1; it++) {
        const uint32_t p = __builtin_ctzll(S);
        S &= S - 1;
        uint32_t e0, e1, e2, e3;
        load16(buf, r + p, e0, e1, e2, e3);
        const uint32_t L = rec_check(e0, e1, remr - p);
        const uint32_t np = p + L;
        if (np >= (uint32_t)WIN) return FAIL;
        bool ok = (np == remr);
        if (!ok) {
            load16(buf, r + np, e0, e1, e2, e3);
            ok = rec_check(e0, e1, remr - np) != 0;
        }
        if (ok) S |= 1ull << np;
    }
    if (__popcll(S) != 1) return FAIL;
    return r + (uint32_t)__builtin_ctzll(S);
}
NXG_DEV uint32_t merge_point(const uint8_t* buf, uint32_t r, uint64_t t0, uint64_t W) {
    if (t0 + r >= W) return (uint32_t)(W - t0);
    const u32x4 q = *reinterpret_cast<const u32x4*>(buf + r);  // r is 64-byte aligned
    const uint32_t d4 = *reinterpret_cast<const uint32_t*>(buf + r + 16);
    return merge_point_d(buf, r, t0, W, q.x, q.y, q.z, q.w, d4);
}

NXG_DEV uint4 ld16_guard(const uint8_t* __restrict__ wire, uint64_t off, uint64_t W) {
    if (off + 16 <= W) return *reinterpret_cast<const uint4*>(wire + off);
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; k++)
        if (off + k < W) v[k >> 2] |= (uint32_t)wire[off + k] << (8 * (k & 3));
    return make_uint4(v[0], v[1], v[2], v[3]);
}
// ---- per-tile helpers shared by the two passes -----------------------------------------------

// One 4 KiB tile plus HALO look-ahead bytes in registers: lane owns the 16-byte pieces
// i*1024 + lane*16 (coalesced); lanes < HALO/16 also own one halo piece.
struct TileRegs {
    u32x4 v[4];
    u32x4 h;
    uint32_t m;  // this lane's merge-point offset from the count pass (emit pass only)
};
NXG_DEV void tile_load(TileRegs& r, const uint8_t* __restrict__ wire, uint64_t t0, uint64_t W,
                       uint32_t lane, const uint8_t* moff) {
    if (moff) r.m = moff[lane];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint4 x = ld16_guard(wire, t0 + i * 1024 + lane * 16, W);
        r.v[i] = u32x4{x.x, x.y, x.z, x.w};
    }
    const uint4 x = ld16_guard(wire, t0 + IMG + (lane & (HALO / 16 - 1)) * 16, W);
    r.h = u32x4{x.x, x.y, x.z, x.w};
}
// The same for a tile whose bytes and halo lie inside the frame: straight-line loads only, so
// the compiler can wait for exactly the oldest tile in flight (vmcnt(N), not vmcnt(0)). Lanes
// past the halo re-read its lines instead of branching.
template <bool MOFF>
NXG_DEV void tile_load_full(TileRegs& r, const uint8_t* __restrict__ wire, uint64_t t0,
                            uint32_t lane, const uint8_t* moff) {
    if (MOFF) r.m = moff[lane];
    const u32x4* p = reinterpret_cast<const u32x4*>(wire + t0);
#pragma unroll
    for (int i = 0; i < 4; i++) r.v[i] = p[i * 64 + lane];
    r.h = p[4 * 64 + (lane & (HALO / 16 - 1))];
}
NXG_DEV void tile_store(uint8_t* buf, const TileRegs& r, uint32_t lane) {
#pragma unroll
    for (int i = 0; i < 4; i++) *reinterpret_cast<u32x4*>(buf + i * 1024 + lane * 16) = r.v[i];
    // every lane stores its halo piece; lanes that share a piece write identical bytes (no
    // branch, so the compiler can keep later tiles' loads in flight across this store)
    *reinterpret_cast<u32x4*>(buf + IMG + (lane & (HALO / 16 - 1)) * 16) = r.h;
}

// Merge point X_lane of this lane's chunk [64*lane, 64*lane+64) of `tile` (buf = the tile's
// LDS image): FAIL if the walks starting there do not merge. Lane 63's chunk starts at STRIDE,
// so its merge point is the next tile's X_0 and the tiles join without a gap or overlap.
NXG_DEV uint32_t chunk_merge(const uint8_t* buf, uint64_t tile, uint64_t W, uint32_t lane) {
    if (tile == 0 && lane == 0) {  // the frame's first record starts at byte 0
        uint32_t e0, e1, e2, e3;
        load16(buf, 0, e0, e1, e2, e3);
        return (W == 0 || rec_check(e0, e1, W)) ? 0u : FAIL;
    }
    return merge_point(buf, lane * CHUNK, tile * STRIDE, W);
}

// Records of this lane's chunk [xa, X_lane+1) (lane 63 owns none). Sets `bad` if the chunk is
// not a chain of valid f64 records from merge point to merge point. With POS, the tile-relative
// record starts go to pslot[lane*SLOTS + k].
constexpr int SLOTS = 12;  // records a lane can own: span < CHUNK + WIN bytes, >= 12 B each
template <bool POS>
NXG_DEV uint32_t chunk_walk(const uint8_t* buf, uint32_t xa, uint32_t lane, uint16_t* pslot,
                            bool& bad) {
    const uint32_t xb = __shfl_down(xa, 1, 64);
    bad = (xa == FAIL) | (xb == FAIL) | (xa > xb);
    if (lane == 63) {
        bad = xa == FAIL;
        return 0;
    }
    uint32_t n = 0;
    if (!bad) {
        uint32_t pos = xa;
        while (pos < xb) {
            const uint32_t L = buf[pos];
            if (L - 12u > 3u || n == SLOTS) {
                bad = true;
                break;
            }
            if (POS) pslot[lane * SLOTS + n] = (uint16_t)pos;
            pos += L;
            n++;
        }
        bad |= (pos != xb);
    }
    return bad ? 0u : n;
}

// Tiles [b, e) of run r when `nt` tiles are split into `R` runs (balanced, contiguous).
NXG_DEV uint64_t run_begin(uint64_t first, uint64_t nt, uint32_t R, uint32_t r) {
    return first + nt * r / R;
}

// Walks the run's tiles [b, e) in order: stage(regs, tile) copies a tile into the wave's LDS
// image, then fn(tile) processes it there. Two register sets alternate; a set is refilled with
// the tile after next once its tile has been processed, so the next tile's loads are always in
// flight during processing. The refill is unconditional (past the run's end it re-reads the
// run's last full tile, an L2 hit) and comes after fn's stores, so the compiler's wait before
// each stage is an exact vmcnt(5): the set's own loads (and fn's earlier stores), never the
// other set's. Tiles reaching past the frame's end (at most the last two) are loaded with
// guards after the pipelined loop.
// With MOFF, each tile's 64 merge-point offsets (moff + 64*tile, from the count pass) are
// loaded with its bytes, one per lane, into TileRegs::m.
template <bool MOFF, typename Stage, typename Fn>
NXG_DEV void for_run_tiles(const uint8_t* __restrict__ wire, uint64_t W, uint64_t b, uint64_t e,
                           uint32_t lane, const uint8_t* moff, Stage&& stage, Fn&& fn) {
    // tile t is full (image and halo inside the frame) iff t < nfull
    const uint64_t nfull = W >= IMG + HALO ? (W - IMG - HALO) / STRIDE + 1 : 0;
    const uint64_t ef = e < nfull ? e : (b > nfull ? b : nfull);
    if (b < ef) {
        const uint64_t tl = ef - 1;
        TileRegs A, B;
        tile_load_full<MOFF>(A, wire, b * STRIDE, lane, moff + 64 * b);
        tile_load_full<MOFF>(B, wire, (b + 1 < ef ? b + 1 : tl) * STRIDE, lane,
                             moff + 64 * (b + 1 < ef ? b + 1 : tl));
        for (uint64_t t = b; t < ef; t += 2) {
            stage(A, t);
            fn(t);
            tile_load_full<MOFF>(A, wire, (t + 2 < ef ? t + 2 : tl) * STRIDE, lane,
                                 moff + 64 * (t + 2 < ef ? t + 2 : tl));
            asm volatile("" ::: "memory");  // keep the refill here (not sunk into the next step)
            if (t + 1 >= ef) break;
            stage(B, t + 1);
            fn(t + 1);
            tile_load_full<MOFF>(B, wire, (t + 3 < ef ? t + 3 : tl) * STRIDE, lane,
                                 moff + 64 * (t + 3 < ef ? t + 3 : tl));
            asm volatile("" ::: "memory");
        }
    }
    for (uint64_t t = ef; t < e; t++) {
        TileRegs A;
        tile_load(A, wire, t * STRIDE, W, lane, MOFF ? moff + 64 * t : nullptr);
        stage(A, t);
        fn(t);
    }
}

}  // namespace
