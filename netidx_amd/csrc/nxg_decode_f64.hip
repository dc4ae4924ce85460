// nxg_decode_f64.hip -- single-pass homogeneous-f64 decode for gfx950.
//
// Replaces the receive_batch_fn loop (netidx/src/channel.rs:504-521) for frames in which every
// message is From::Update(Id, F64). Each such message is canonical on the wire (SURVEY.md
// Appendix A):
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
//
// Record numbering is a single-pass decoupled look-back over per-tile record counts. Tiles are
// assigned statically to a persistent, fully resident grid. The 8-byte status granules are
// written and polled with agent-scope relaxed atomics (sc1), the hand-off form in
// MI355X_MICROARCH.md "Valid forms" (R2).
//
// HBM traffic per record: the wire bytes are read once, and 16 bytes (id u64 + f64 bits) are
// written once through an LDS staging buffer, with coalesced stores.
#include "nxg_device.h"

using namespace f64dec;

namespace {

constexpr uint32_t FAIL = 0xffffffffu;

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

// SWAR: 0x80 in every zero byte of x (exact, no borrow propagation)
NXG_DEV uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
}
// gather the 0x80 flags of a zero_bytes() result into 4 bits
NXG_DEV uint32_t nib(uint32_t zb) { return (((zb >> 7) & 0x01010101u) * 0x01020408u) >> 24; }

// Merge point of all record walks starting in [r, r+15) (tile-relative). r is 4-aligned.
NXG_DEV uint32_t merge_point(const uint8_t* buf, uint32_t r, uint64_t t0, uint64_t W) {
    const uint64_t abs_r = t0 + r;
    if (abs_r >= W) return (uint32_t)(W - t0);  // chunk past the end: the END position
    const uint64_t remr = W - abs_r;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(buf + r);
    const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
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

NXG_DEV uint4 ld16_guard(const uint8_t* __restrict__ wire, uint64_t off, uint64_t W) {
    if (off + 16 <= W) return *reinterpret_cast<const uint4*>(wire + off);
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; k++)
        if (off + k < W) v[k >> 2] |= (uint32_t)wire[off + k] << (8 * (k & 3));
    return make_uint4(v[0], v[1], v[2], v[3]);
}

}  // namespace
// One wave per workgroup, one 4 KiB tile per wave iteration. All exchanges between lanes are
// wave-local (shuffles, ballots, the wave's own LDS), so no phase waits for other waves. Many
// waves per CU hide each other's look-back latency.
__global__ __launch_bounds__(TPB) void nxg_dec_f64_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t* __restrict__ oid,
    uint64_t* __restrict__ oval, uint64_t cap, uint64_t* __restrict__ tstat, uint32_t ntiles,
    uint32_t epoch, DevStatus* __restrict__ st, DevStatus* zst) {
    zero_status(zst);
    __shared__ __attribute__((aligned(16))) uint8_t buf[TILE + HALO];
    __shared__ __attribute__((aligned(16))) uint64_t sid[MAXREC];
    __shared__ __attribute__((aligned(16))) uint64_t sval[MAXREC];

    const uint32_t lane = threadIdx.x;
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles) return;

    // register prefetch of the first tile: 4 x 16 B per lane + the halo (8 lanes x 16 B)
    uint4 pre[4], preh = make_uint4(0, 0, 0, 0);
    {
        const uint64_t t0 = (uint64_t)tile * TILE;
#pragma unroll
        for (int i = 0; i < 4; i++) pre[i] = ld16_guard(wire, t0 + i * 1024 + lane * 16, W);
        if (lane < HALO / 16) preh = ld16_guard(wire, t0 + TILE + lane * 16, W);
    }

    for (; tile < ntiles; tile += gridDim.x) {
        const uint64_t t0 = (uint64_t)tile * TILE;
#pragma unroll
        for (int i = 0; i < 4; i++) *reinterpret_cast<uint4*>(buf + i * 1024 + lane * 16) = pre[i];
        if (lane < HALO / 16) *reinterpret_cast<uint4*>(buf + TILE + lane * 16) = preh;
        __syncthreads();  // single-wave workgroup: orders the LDS writes before the reads
        if (ld_agent32(&st->fast_fail)) break;  // another tile already rejected the frame

        // prefetch the next tile while this one is parsed
        const uint32_t nxt = tile + gridDim.x;
        if (nxt < ntiles) {
            const uint64_t n0 = (uint64_t)nxt * TILE;
#pragma unroll
            for (int i = 0; i < 4; i++) pre[i] = ld16_guard(wire, n0 + i * 1024 + lane * 16, W);
            if (lane < HALO / 16) preh = ld16_guard(wire, n0 + TILE + lane * 16, W);
        }

        // 1. merge points of this lane's chunk start and of the next chunk start
        uint32_t xa;
        if (tile == 0 && lane == 0) {
            uint32_t e0, e1, e2, e3;
            load16(buf, 0, e0, e1, e2, e3);
            xa = (W == 0 || rec_check(e0, e1, W)) ? 0u : FAIL;
        } else {
            xa = merge_point(buf, lane * CHUNK, t0, W);
        }
        uint32_t xb = __shfl_down(xa, 1, 64);
        if (lane == TPB - 1) xb = merge_point(buf, TILE, t0, W);

        // 2. count walk over [X_j, X_{j+1})
        uint32_t n = 0;
        bool bad = (xa == FAIL) | (xb == FAIL) | (xa > xb);
        if (!bad) {
            uint32_t pos = xa;
            while (pos < xb) {
                const uint32_t L = buf[pos];
                if (L - 12u > 3u) {
                    bad = true;
                    break;
                }
                pos += L;
                n++;
            }
            bad |= (pos != xb);
        }
        if (bad) n = 0;
        const uint32_t inc = wave_incl_scan(n);
        const uint32_t off = inc - n;
        const uint32_t ntile = __shfl(inc, TPB - 1, 64);

        // 3. publish this tile's aggregate as early as possible
        if (lane == 0) st_agent(&tstat[tile], lb_word(tile == 0 ? kFlagInc : kFlagAgg, epoch, ntile));

        // 4. validate + decode into the LDS staging buffer
        if (!bad) {
            uint32_t pos = xa;
            for (uint32_t k = 0; k < n; k++) {
                uint32_t e0, e1, e2, e3;
                load16(buf, pos, e0, e1, e2, e3);
                const uint32_t L = rec_check(e0, e1, W - (t0 + pos));
                if (!L) {
                    bad = true;
                    break;
                }
                uint64_t id, val;
                rec_decode(e0, e1, e2, e3, L, id, val);
                sid[off + k] = id;
                sval[off + k] = val;
                pos += L;
            }
        }
        bool fail = __any(bad);

        // 5. decoupled look-back for the tile's first record index
        uint64_t base = 0;
        if (tile != 0) {
            int64_t pred = (int64_t)tile - 1;
            const uint64_t t_start = rt_now();
            bool give_up = false;
            for (;;) {
                const int64_t idx = pred - (int64_t)lane;
                uint64_t s = idx >= 0 ? ld_agent(&tstat[idx]) : lb_word(kFlagInc, epoch, 0);
                while (!__all(lb_flag(s, epoch) != 0)) {
                    __builtin_amdgcn_s_sleep(1);
                    if (lb_flag(s, epoch) == 0) s = ld_agent(&tstat[idx]);
                    if (ld_agent32(&st->fast_fail) || rt_now() - t_start > kSpinTicks) {
                        give_up = true;
                        break;
                    }
                }
                if (give_up) break;
                const uint64_t incm = __ballot(lb_flag(s, epoch) == kFlagInc);
                if (incm) {
                    const uint32_t first = (uint32_t)__builtin_ctzll(incm);
                    base += wave_sum<uint64_t>(lane <= first ? (s & kValMask) : 0ull);
                    break;
                }
                base += wave_sum<uint64_t>(s & kValMask);
                pred -= 64;
            }
            if (give_up) {
                if (lane == 0 && !ld_agent32(&st->fast_fail)) atomicOr(&st->timeout, 1u);
                fail = true;
            }
            if (lane == 0) st_agent(&tstat[tile], lb_word(kFlagInc, epoch, base + ntile));
        }
        if (fail) {
            if (lane == 0) atomicOr(&st->fast_fail, 1u);
            break;
        }
        __syncthreads();  // staging writes before the cross-lane reads below

        // 6. coalesced stores of the staged records
        uint32_t lim = ntile;
        if (base + ntile > cap) {
            lim = base < cap ? (uint32_t)(cap - base) : 0u;
            if (lane == 0) atomicOr(&st->capacity, 1u);
        }
        for (uint32_t i = lane; i < lim; i += TPB) {
            oid[base + i] = sid[i];
            oval[base + i] = sval[i];
        }
        if (tile == ntiles - 1 && lane == 0) {
            st->n_rows = base + ntile;
            st->path = 1;
        }
        __syncthreads();  // staging and buf are rewritten by the next tile
    }
}

hipError_t nxg_launch_dec_f64(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                              uint64_t cap, uint64_t* tstat, uint32_t epoch, DevStatus* st,
                              int grid, hipStream_t s) {
    const uint64_t nt = (W + TILE - 1) / TILE;
    if (nt == 0) return hipSuccess;
    // grid <= 0: one workgroup per tile in blockIdx order. Each XCD dispatches its blocks in
    // increasing order, so the lowest unfinished tile is always resident and its predecessor is
    // done (progress). grid > 0: persistent grid of `grid` co-resident workgroups striding over
    // the tiles (the fallback if the watchdog ever fires).
    const uint64_t g = grid <= 0 ? nt : (nt < (uint64_t)grid ? nt : (uint64_t)grid);
    hipLaunchKernelGGL(nxg_dec_f64_kernel, dim3(g), dim3(TPB), 0, s, wire, W, oid, oval, cap,
                       tstat, (uint32_t)nt, epoch, st, nxg_zero_slot);
    return hipGetLastError();
}

int nxg_occupancy_dec_f64() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, nxg_dec_f64_kernel, TPB, 0) != hipSuccess)
        return 1;
    return n;
}
