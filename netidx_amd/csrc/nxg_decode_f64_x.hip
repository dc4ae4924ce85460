// nxg_decode_f64_x.hip -- homogeneous-f64 decode of ANY f64 frame in one pass, for gfx950: the
// decoder for frames whose record lengths vary record to record (ids in arbitrary order: a batch
// updating an arbitrary subset of a publisher's values, netidx/src/publisher/mod.rs:776-845), on
// which the length-run decoder (nxg_decode_f64_run.hip) gives up. Replaces the receive_batch_fn
// loop (netidx/src/channel.rs:504-521) for frames of From::Update(Id, F64) messages with ids of
// 1..5 varint bytes (< 2^35), records of 12..16 bytes.
//
// A wave takes SPW consecutive 4 KiB sub-tiles, a workgroup four waves (64 KiB), and no wave
// waits on a workgroup that may not be running (a decoupled look-back whose unpublished
// predecessors are counted by the waiting workgroup itself), so any number of these decodes can
// share the GPU:
//   1. per sub-tile: its bytes and 64 / 128 around them into LDS (one coalesced pass; dwords
//      stored swizzled, SwzImg, so that the lanes' 64-byte-strided reads do not pile onto two
//      banks). Lane j takes the 64 positions of chunk j: S = the positions where a complete record
//      starts (candidates by SWAR -- a byte in 12..16 then 0x04 -- each checked by rec_check16
//      with independent loads) and the successors of those records (start + length). No walk:
//      the starts ARE the frame's records exactly when every start but the frame's first byte is
//      some start's successor and every successor is a start or the frame end (a start without a
//      predecessor lies inside a record; following successors from byte 0 then visits every
//      start and ends at W). Neighbouring chunks' masks come by DPP; lane 0 and lane 63 check the
//      16 positions before / after the sub-tile themselves. The masks stay in registers;
//   2. a block scan of the counts (popcounts), the workgroup's total to the look-back, its first
//      row from it (one look-back per 64 KiB);
//   3. per sub-tile: the image again (from L2), each start's record decoded (independent loads)
//      into an LDS row image, then the wave's rows leave as coalesced 8-byte column stores.
// A check that fails raises fast_fail, and the host reruns the frame on the mixed/general
// decoders.
#include "nxg_device.h"
#include "nxg_f64_rec16.h"

namespace f64x {
constexpr uint32_t SUB = 4096;          // bytes per sub-tile
constexpr uint32_t HALO = 128;          // look-ahead bytes past the sub-tile
constexpr uint32_t XLO = 64;            // image offset of the sub-tile's first byte
constexpr uint32_t XHI = XLO + SUB;
constexpr uint32_t IMGB = XHI + HALO;   // image bytes
constexpr int TPB = 256;
constexpr int WAVES = TPB / 64;
#ifndef NXG_F64X_SPW
#define NXG_F64X_SPW 4
#endif
constexpr int SPW = NXG_F64X_SPW;       // sub-tiles per wave
constexpr uint64_t WGB = (uint64_t)SUB * SPW * WAVES;  // bytes per workgroup
constexpr uint32_t MAXR = SUB / 12 + 2;  // rows per sub-tile (records start in it, >= 12 bytes)
constexpr uint32_t MAXW = MAXR * SPW;     // rows per wave
static_assert((uint64_t)SUB * SPW <= 65536, "start-list offsets are u16 within the wave's bytes");
#ifndef NXG_F64X_CB
#define NXG_F64X_CB 6
#endif
#ifndef NXG_F64X_OCC
#define NXG_F64X_OCC 4  // waves per SIMD asked of the register allocator (the self-help path
#endif                  // alone would push the kernel to 134 VGPRs, 3 waves)
#ifndef NXG_F64X_CHEAP
#define NXG_F64X_CHEAP 1  // 0: every candidate checked as a record before it counts as a start
#endif                    // (10^7 random-order ids: 128.6 us, against 105.6 us for 1)
#ifndef NXG_F64X_LASTX
#define NXG_F64X_LASTX 1  // 1: the 16 positions after a sub-tile read only after the wave's last (0.121-0.122 vs 0.1245 ms)
#endif
constexpr int CB = NXG_F64X_CB;          // candidates checked together (independent loads)
#ifndef NXG_F64X_EU
#define NXG_F64X_EU 2  // emit rounds with loads in flight together (1 / 2 / 4 with pairs: 0.114 / 0.113 / 0.116 ms)
#endif
#ifndef NXG_F64X_CBATCH
#define NXG_F64X_CBATCH 0
#endif
#ifndef NXG_F64X_PAIRS
#define NXG_F64X_PAIRS 1  // emit two rows per lane as 16-byte stores (0.113 vs 0.118 ms at 10^7)
#endif
#ifndef NXG_F64X_NT
#define NXG_F64X_NT 1  // nontemporal row stores (0.900-0.905 vs 0.928-0.931 ms at 10^8)
#endif
#ifndef NXG_F64X_PFD
#define NXG_F64X_PFD 1  // sub-tile images loading ahead (registers; 2: no faster)
#endif
constexpr int PFD = NXG_F64X_PFD;

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int EU = NXG_F64X_EU;          // emit rounds whose record loads are in flight together
}  // namespace f64x

#ifndef NXG_F64X_PROF
#define NXG_F64X_PROF 0
#endif
#if NXG_F64X_PROF
// diagnostic build only: per workgroup (the first 16384) s_memtime at the kernel's phase edges
// (start, phase 1 done, block scan done, look-back done, emit done) and the XCC / CU it ran on
__device__ unsigned long long nxg_f64x_st[6][16384];
#define XSTAMP(k)                                                                                \
    do {                                                                                         \
        if (threadIdx.x == 0 && blockIdx.x < 16384)                                              \
            nxg_f64x_st[k][blockIdx.x] = __builtin_amdgcn_s_memrealtime();                           \
    } while (0)
#else
#define XSTAMP(k) \
    do {          \
    } while (0)
#endif

namespace {
using namespace f64x;
using namespace f64rec16;

// The decoded range: `wire` is its first byte, W the bytes from there to the frame's end, R <= W
// the range's length (records that START before R are the range's; the bytes after are read as
// look-ahead), `pre` bytes readable before wire[0], `first`: the range starts the frame.
struct XRange {
    uint64_t W, R, pre;
    bool first;
};

// the image of the sub-tile at a0: frame bytes [a0 - 64, a0 + 4096 + 128), dwords swizzled.
// fetch issues the loads into registers (the next sub-tile's, while this one is walked); commit
// stores them into the wave's LDS image.
struct Prefetch {
    uint4 v[(IMGB + 1023) / 1024];
};
NXG_DEV void fetch_image(Prefetch& pf, const uint8_t* __restrict__ wire, uint64_t a0, uint64_t W,
                         uint32_t lane, uint64_t pre = 0) {
    if (a0 >= W) return;
#pragma unroll
    for (uint32_t i = 0; i < (IMGB + 1023) / 1024; i++) {
        const uint32_t off = i * 1024 + lane * 16;
        if (off < IMGB) {
            const int64_t pos = (int64_t)a0 - (int64_t)XLO + (int64_t)off;
            pf.v[i] = pos >= 0 ? ld16g(wire, (uint64_t)pos, W) : ld16_pre(wire, pos, W, pre);
        }
    }
}
NXG_DEV void commit_image(uint8_t* buf, const Prefetch& pf, uint32_t lane) {
    uint32_t* bw = reinterpret_cast<uint32_t*>(buf);
    wave_lds_order();  // the previous image's reads are issued
#pragma unroll
    for (uint32_t i = 0; i < (IMGB + 1023) / 1024; i++) {
        const uint32_t off = i * 1024 + lane * 16;
        if (off < IMGB) {
            const uint32_t q = off >> 2;
            bw[SwzImg::sw(q)] = pf.v[i].x;
            bw[SwzImg::sw(q + 1)] = pf.v[i].y;
            bw[SwzImg::sw(q + 2)] = pf.v[i].z;
            bw[SwzImg::sw(q + 3)] = pf.v[i].w;
        }
    }
    wave_lds_order();
}

// Record starts among the 4 * NDW positions from image offset r (4-aligned; frame position of
// bit 0: fp): S (bit i: a complete record starts at r + i) and the successors of those records
// (bit i of slo: position r + i, of shi: r + 64 + i). Positions at or past W hold none.
template <int NDW>
NXG_DEV void starts_of(const SwzImg& im, uint32_t r, uint64_t fp, uint64_t W, uint64_t& S,
                       uint64_t& slo, uint64_t& shi) {
    const uint32_t q0 = r >> 2;
    uint64_t cm = 0;
    uint32_t a = im.w(q0);
#pragma unroll
    for (int k = 0; k < NDW; k++) {
        const uint32_t b = im.w(q0 + k + 1);
        cm |= (uint64_t)nib(len_bytes(a) & zero_bytes(alignbyte(b, a, 1) ^ 0x04040404u)) << (4 * k);
        a = b;
    }
    if (fp >= W) cm = 0;
    else if (W - fp < 4u * NDW) cm &= (1ull << (W - fp)) - 1ull;
    S = slo = shi = 0;
    if (NXG_F64X_CHEAP) {
        // every candidate (a byte in 12..16 then 04) taken as a start, its successor from its
        // length byte; the records are checked completely where they are decoded
        S = cm;
        if (!NXG_F64X_CBATCH) {
#pragma unroll 1
            for (uint64_t m = cm; m; m &= m - 1) {
                const uint32_t p = (uint32_t)__builtin_ctzll(m);
                const uint32_t nx = p + im.byte(r + p);
                if (nx < 64u) slo |= 1ull << nx;
                else shi |= 1ull << (nx - 64u);
            }
            return;
        }
        // (CB candidates at a time: their length bytes read from LDS together, one wait; A/B:
        // slower, 0.122 vs 0.118 ms at 10^7 with the emit pipelining)
#pragma unroll 1
        for (uint64_t m = cm; m;) {
            uint32_t pp[CB], ll[CB];
#pragma unroll
            for (int i = 0; i < CB; i++) {
                pp[i] = m ? (uint32_t)__builtin_ctzll(m) : 64u;
                m &= m - 1;
            }
#pragma unroll
            for (int i = 0; i < CB; i++) ll[i] = im.byte(r + (pp[i] & 63u));
#pragma unroll
            for (int i = 0; i < CB; i++) {
                if (pp[i] < 64u) {
                    const uint32_t nx = pp[i] + ll[i];
                    if (nx < 64u) slo |= 1ull << nx;
                    else shi |= 1ull << (nx - 64u);
                }
            }
        }
        return;
    }
    // up to CB candidates at a time: positions, then their first 8 bytes, then the checks
#pragma unroll 1
    while (cm) {
        uint32_t pp[CB];
#pragma unroll
        for (int i = 0; i < CB; i++) {
            pp[i] = cm ? (uint32_t)__builtin_ctzll(cm) : 64u;
            cm &= cm - 1;
        }
        uint32_t e0[CB], e1[CB];
#pragma unroll
        for (int i = 0; i < CB; i++) {
            const uint32_t rel = r + (pp[i] & 63u);
            const uint32_t q = rel >> 2, sh = rel & 3u;
            const uint32_t d0 = im.w(q), d1 = im.w(q + 1), d2 = im.w(q + 2);
            e0[i] = alignbyte(d1, d0, sh);
            e1[i] = alignbyte(d2, d1, sh);
        }
#pragma unroll
        for (int i = 0; i < CB; i++) {
            const uint32_t L = pp[i] < 64u ? rec_check16(e0[i], e1[i], W - (fp + pp[i])) : 0u;
            if (L) {
                S |= 1ull << pp[i];
                const uint32_t nx = pp[i] + L;
                if (nx < 64u) slo |= 1ull << nx;
                else shi |= 1ull << (nx - 64u);
            }
        }
    }
}

// the 64-bit value of the previous / next lane (lane 0 / 63: 0), DPP wave_shr / wave_shl
NXG_DEV uint64_t prev64(uint64_t v) { return dpp0_64<0x138, 0xf>(v); }
NXG_DEV uint64_t next64(uint64_t v) { return dpp0_64<0x130, 0xf>(v); }

// Phase 1 of one sub-tile whose image (at a0) is in `buf`: S (the chain's record starts in the
// lane's chunk), n = |S|, the chain's entry into the next sub-tile in q (carried in; ~0 for a
// wave's first sub-tile: found from the merge point before a0). `bad` when the starts are not a
// chain. Wave-collective.
NXG_DEV void subtile_starts(const uint8_t* __restrict__ wire, const XRange& rg, uint8_t* buf,
                            uint64_t a0, bool last_sub, uint32_t lane, uint64_t& q, uint64_t& Sm,
                            uint32_t& n, bool& bad, DevStatus* st) {
    const uint64_t W = rg.W, R = rg.R;
    const SwzImg im{buf};
    const uint64_t ib = a0 - XLO;  // frame position of image byte 0 (wraps for a0 = 0)
    const uint32_t r = XLO + lane * 64;
    const uint64_t fp = ib + r;  // frame position of the lane's chunk
    // The chain's entry into the sub-tile: the frame start, the previous sub-tile's exit, or
    // (the wave's first sub-tile) a walk from the merge point of the 16 bytes at a0 - 64,
    // where the walks from every valid-looking start meet (so on the true chain, records
    // being at most 16 bytes long), to the first start at or past a0. Lane 0 alone.
    if (a0 == 0 && rg.first) {
        q = 0;
    } else if (q == ~0ull) {
        uint32_t x = FAILX;
        if (lane == 0) {
            x = merge16i(im, 0, ib, W);
            while (x < XLO) {
                uint32_t e0, e1, e2, e3;
                lds16i(im, x, e0, e1, e2, e3);
                const uint32_t L = rec_check16(e0, e1, W - (ib + x));
                x = L ? x + L : FAILX;
            }
        }
        x = (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
        if (x == FAILX) bad = true;
        else q = ib + x;
    }
    const uint64_t inc = lane == 0 && q != ~0ull && q - a0 < 64 ? 1ull << (q - a0) : 0ull;
    uint64_t S, slo, shi;
    starts_of<16>(im, r, fp, W, S, slo, shi);
    // lane 63: the starts among the 16 positions after the sub-tile. Inside the wave the next
    // sub-tile's entry check covers them (LASTX), so only the wave's last sub-tile reads them.
    const bool need_x = !NXG_F64X_LASTX || last_sub || a0 + SUB >= W || a0 + SUB >= R;
    uint64_t Sx = 0, xlo, xhi;
    if (need_x) starts_of<4>(im, XHI, ib + XHI, W, Sx, xlo, xhi);
    // False starts -- bytes inside a record that read as one (an f64's bytes may) -- are
    // those no start leads to, or whose only predecessors are false: dropped until every
    // start has a predecessor (in its chunk, the previous chunk, or the entry). What remains
    // is exactly the chain through the sub-tile: each start leads back to the entry.
    // The DPP moves run in every lane, the edge lanes' own terms OR-ed in: a DPP move in a
    // branch reads 0 from a lane that is switched off.
    uint64_t sin = prev64(shi) | inc;
    for (int it = 0;; it++) {
        const uint64_t roots = S & ~(slo | sin);
        if (!__any(roots != 0)) break;
        if (it == 64) {  // a long chain of false starts: the frame is rerun
            bad = true;
            break;
        }
        S &= ~roots;
        slo = shi = 0;
        for (uint64_t m = S; m; m &= m - 1) {
            const uint32_t p = (uint32_t)__builtin_ctzll(m);
            const uint32_t nx = p + im.byte(r + p);
            if (nx < 64u) slo |= 1ull << nx;
            else shi |= 1ull << (nx - 64u);
        }
        sin = prev64(shi) | inc;
    }
    const uint64_t Snx = next64(S) | (lane == 63 ? Sx : 0ull);  // the next chunk's starts
    const uint64_t d = W - fp;  // (fp <= W below: the frame end's bit)
    const uint64_t wlo = fp <= W && d < 64 ? 1ull << d : 0ull;
    const uint64_t whi = fp <= W && d >= 64 && d < 128 ? 1ull << (d - 64) : 0ull;
    const uint64_t shic = need_x || lane != 63 ? shi : 0ull;
    bool b = (slo & ~(S | wlo)) != 0 ||  // a successor that is not a start
             (shic & ~(Snx | whi)) != 0 ||
             (inc & ~(S | wlo)) != 0;    // the entry is not a start
#ifdef NXG_F64X_DIAG
    if (b) nxg_f64x_diag(fp, S, slo, sin, shi, Snx, wlo, whi);
#endif
    bad |= b;
    // the range's records: the starts before R (the chain checks above used them all)
    const uint64_t keep = fp >= R ? 0ull : (R - fp >= 64 ? ~0ull : (1ull << (R - fp)) - 1ull);
    Sm = S & keep;
    n = (uint32_t)__popcll(Sm);
    if (a0 == 0 && lane == 0) st->diag[2] = q + 1;  // the range's entry (+1; 0: unknown)
    // the next sub-tile's entry: lane 63's last start + its length
    uint64_t qn = ~0ull;
    if (lane == 63 && S) {
        const uint32_t pl = 63u - (uint32_t)__builtin_clzll(S);
        qn = fp + pl + im.byte(r + pl);
    }
    q = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)qn, 63) |
        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(qn >> 32), 63) << 32);
    if (R <= a0 + SUB) {
        // the range ends in this sub-tile: its exit is the first start at or past R, else the
        // chain's entry into the next sub-tile
        const uint64_t past = S & ~keep;
        const uint64_t fx = past ? fp + (uint64_t)__builtin_ctzll(past) : ~0ull;
        const uint32_t lo = wave_min_u32((uint32_t)(fx == ~0ull ? 0xffffffffu : (uint32_t)(fx - a0)));
        // (no start at or past R here: the end of the sub-tile's last record -- lane 63 may hold
        // none, where the frame ends inside the sub-tile)
        uint64_t qe = ~0ull;
        if (S) {
            const uint32_t pl = 63u - (uint32_t)__builtin_clzll(S);
            qe = fp + pl + im.byte(r + pl);
        }
        const uint64_t hm = __ballot(S != 0);
        const int hl = hm ? 63 - __builtin_clzll(hm) : 0;
        const uint64_t qlast =
            (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)qe, hl) |
            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(qe >> 32), hl) << 32);
        const uint64_t ex = lo != 0xffffffffu ? a0 + lo : (hm ? qlast : q);
        if (lane == 0) st->diag[3] = ex + 1;  // (+1; 0: unknown)
    }
}

// The record count of workgroup g's bytes, by one wave with its own LDS image `buf` (self-help:
// the look-back's predecessor g has not published it): the f64 decoders' exact path
// (nxg_f64_rec16.h exact_tile: merge points and lane walks), which counts the records that start
// in the range. On a valid frame that is g's own count (both are the true chain's starts in g's
// bytes); if the walks find no chain the frame is rerun (fast_fail), as g itself would.
template <uint32_t T>
NXG_DEV uint64_t unit_count(const uint8_t* __restrict__ wire, const XRange& rg, uint8_t* buf,
                            uint64_t g, uint32_t lane, DevStatus* st) {
    static_assert(IMGB == kXImg && SUB == kXSub && XLO == kXLo, "the exact path's image");
    uint32_t c, en, xx;
    bool b = false, ov = false;
    exact_tile<false, T>(wire, rg.W, rg.R, rg.first, rg.pre, g, buf, lane, 0, nullptr, nullptr, 0,
                         c, en, xx, b, ov);
    if (b && lane == 0) atomicOr(&st->fast_fail, 1u);
    return c;
}
NXG_DEV uint64_t wg_count(const uint8_t* __restrict__ wire, const XRange& rg, uint8_t* buf,
                          uint64_t g, uint32_t lane, DevStatus* st) {
    return unit_count<(uint32_t)WGB>(wire, rg, buf, g, lane, st);
}

__global__ __launch_bounds__(TPB, NXG_F64X_OCC) void nxg_f64x_kernel(const uint8_t* __restrict__ wire,
                                                       XRange rg, uint64_t* __restrict__ oid,
                                                       uint64_t* __restrict__ oval, uint64_t cap,
                                                       uint64_t* tstat, uint32_t epoch,
                                                       DevStatus* __restrict__ st,
                                                       DevStatus* zst, uint32_t patience) {
    zero_status(zst);
    XSTAMP(0);
    const uint64_t W = rg.W, R = rg.R;
    __shared__ __attribute__((aligned(16))) uint8_t img[WAVES][IMGB];
    // the wave's record starts in wire order, as offsets from its first byte (< SUB * SPW)
    __shared__ uint16_t plist[WAVES][MAXW];
    __shared__ uint64_t scan_tmp[WAVES];
    __shared__ uint64_t sh_base;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // (blockIdx order with self-help; a ticket counter measured 0.104 -> 0.120 ms at 10^7)
    const uint32_t bid = blockIdx.x;
    const uint64_t w0 = (uint64_t)bid * WGB + (uint64_t)w * SUB * SPW;  // the wave's bytes
    uint8_t* buf = img[w];
    uint16_t* pl = plist[w];
    bool bad = false;
    // the images of the next PFD sub-tiles in registers while one is checked
    Prefetch pf[PFD];
#pragma unroll
    for (int s = 0; s < PFD && s < SPW; s++)
        if (w0 + (uint64_t)s * SUB < R) fetch_image(pf[s], wire, w0 + (uint64_t)s * SUB, W, lane, rg.pre);
    // q: the frame position of the chain's first record start at or past the sub-tile, carried
    // from sub-tile to sub-tile of the wave (~0: not known -- the wave's first sub-tile)
    uint64_t q = ~0ull;
    uint32_t tw = 0;  // the wave's records so far (wave-uniform)
#pragma unroll
    for (int s = 0; s < SPW; s++) {
        const uint64_t a0 = w0 + (uint64_t)s * SUB;
        if (a0 >= R) break;
        commit_image(buf, pf[s % PFD], lane);
        if (s + PFD < SPW && a0 + PFD * SUB < R)
            fetch_image(pf[s % PFD], wire, a0 + PFD * SUB, W, lane, rg.pre);  // while checking
        uint64_t Sm;
        uint32_t n;
        subtile_starts(wire, rg, buf, a0, s == SPW - 1, lane, q, Sm, n, bad, st);
        // the sub-tile's starts into the wave's list, in wire order (a frame that is not a chain
        // of records can hold more candidates than the list: those are dropped, and the frame is
        // rerun anyway)
        const uint32_t inc = wave_incl_scan<uint32_t>(n);
        uint32_t k = tw + inc - n;
        const uint32_t pb = (uint32_t)s * SUB + lane * 64;
#pragma unroll 1
        for (uint64_t m = Sm; m; m &= m - 1, k++)
            if (k < MAXW) pl[k] = (uint16_t)(pb + (uint32_t)__builtin_ctzll(m));
        tw += wave_last<uint32_t>(inc);
    }
    bad |= tw > MAXW;
    XSTAMP(1);
    const bool wbad = __any(bad);
    if (wbad && lane == 0) atomicOr(&st->fast_fail, 1u);
    // rows: one block scan of the waves' totals, one look-back per workgroup
    uint64_t total;
    const uint64_t excl =
        block_excl_scan<uint64_t, TPB>(lane == 0 ? (uint64_t)tw : 0ull, scan_tmp, &total);
    XSTAMP(2);
    if (w == 0) {
        uint64_t base = 0;
        if (bid == 0) {
            if (lane == 0) st_agent(&tstat[0], lb_word(kFlagInc, epoch, total));
        } else {
            if (lane == 0) st_agent(&tstat[bid], lb_word(kFlagAgg, epoch, total));
            // no wait on a workgroup that may not be running: an unpublished predecessor's count
            // is computed here from its bytes (self-help), in this wave's LDS image
            base = lookback_selfhelp_fn(tstat, bid, epoch, patience, [&](uint64_t g) -> uint64_t {
                return wg_count(wire, rg, buf, g, lane, st);
            });
            if (lane == 0) st_agent(&tstat[bid], lb_word(kFlagInc, epoch, base + total));
        }
        if (lane == 0) sh_base = base;
        if (bid == gridDim.x - 1 && lane == 0) {
            st->n_rows = base + total;
            st->path = 1;
        }
    }
    __syncthreads();
    XSTAMP(3);
    if (wbad) return;  // (a bad sub-tile has raised fast_fail: the frame is rerun)
    // the wave's first row: the block prefix of its lane 0
    const uint64_t row0 =
        sh_base + ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)excl) |
                   ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(excl >> 32)) << 32));
    // emit: one record per lane, 64 consecutive rows per round; the record's 16 bytes by one
    // (unaligned) load from the frame, which the wave read a moment ago (L2), and checked
    // completely (CHEAP: a candidate counted as a start must be a whole record)
    bool over = false, vbad = false;
#if NXG_F64X_PAIRS
    // two consecutive rows per lane, stored as 16-byte pairs (half the store instructions): lane j
    // of a round takes rows 2j, 2j + 1 counted from the even row at or before row0, so the pairs are
    // 16-byte aligned; the half of a pair outside the wave's rows (the first, the last) is skipped
    {
        const uint32_t a = (uint32_t)(row0 & 1u);  // row0 odd: the first pair's first row is not ours
        const uint64_t rb = row0 - a;              // even
        const uint32_t np = tw ? (tw + a + 1) / 2 : 0u;  // pairs (none for a wave without rows)
#pragma unroll 1
        for (uint32_t j0 = 0; j0 < np; j0 += 64 * EU) {
            uint64_t p[EU][2];
            uint4 e[EU][2];
#pragma unroll
            for (int u = 0; u < EU; u++) {
                const uint32_t j = j0 + 64 * u + lane;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int32_t k = (int32_t)(2 * j + h) - (int32_t)a;  // record index in the wave
                    const uint32_t kc = k < 0 || tw == 0 ? 0u : ((uint32_t)k < tw ? (uint32_t)k : tw - 1);
                    p[u][h] = w0 + pl[kc];
                }
            }
#pragma unroll
            for (int u = 0; u < EU; u++) {
                e[u][0] = ld16g(wire, p[u][0], W);
                e[u][1] = ld16g(wire, p[u][1], W);
            }
#pragma unroll
            for (int u = 0; u < EU; u++) {
                const uint32_t j = j0 + 64 * u + lane;
                uint64_t id[2], val[2];
                bool in[2];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int32_t k = (int32_t)(2 * j + h) - (int32_t)a;
                    in[h] = k >= 0 && (uint32_t)k < tw;
                    const uint32_t L = e[u][h].x & 0xffu;
                    if (in[h]) vbad |= rec_check16(e[u][h].x, e[u][h].y, W - p[u][h]) != L;
                    rec_decode16(e[u][h].x, e[u][h].y, e[u][h].z, e[u][h].w, L, id[h], val[h]);
                }
                const uint64_t row = rb + 2 * (uint64_t)j;
                if (in[0] && in[1] && row + 1 < cap) {
                    const v4u iv = {(uint32_t)id[0], (uint32_t)(id[0] >> 32), (uint32_t)id[1],
                                    (uint32_t)(id[1] >> 32)};
                    const v4u vv = {(uint32_t)val[0], (uint32_t)(val[0] >> 32), (uint32_t)val[1],
                                    (uint32_t)(val[1] >> 32)};
                    if (NXG_F64X_NT) {  // (rows are not read again: keep L2 for the frame)
                        __builtin_nontemporal_store(iv, reinterpret_cast<v4u*>(oid + row));
                        __builtin_nontemporal_store(vv, reinterpret_cast<v4u*>(oval + row));
                    } else {
                        *reinterpret_cast<v4u*>(oid + row) = iv;
                        *reinterpret_cast<v4u*>(oval + row) = vv;
                    }
                } else {
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        if (!in[h]) continue;
                        if (row + h < cap) {
                            oid[row + h] = id[h];
                            oval[row + h] = val[h];
                        } else {
                            over = true;
                        }
                    }
                }
            }
        }
    }
#else
    // EU rounds at a time: their loads in flight together
#pragma unroll 1
    for (uint32_t k0 = 0; k0 < tw; k0 += 64 * EU) {
        uint64_t p[EU];
        uint4 e[EU];
#pragma unroll
        for (int u = 0; u < EU; u++) {
            const uint32_t k = k0 + 64 * u + lane;
            p[u] = w0 + pl[k < tw ? k : tw - 1];
        }
#pragma unroll
        for (int u = 0; u < EU; u++) e[u] = ld16g(wire, p[u], W);
#pragma unroll
        for (int u = 0; u < EU; u++) {
            const uint32_t k = k0 + 64 * u + lane;
            if (k < tw) {
                const uint32_t L = e[u].x & 0xffu;
                vbad |= rec_check16(e[u].x, e[u].y, W - p[u]) != L;
                uint64_t id, val;
                rec_decode16(e[u].x, e[u].y, e[u].z, e[u].w, L, id, val);
                const uint64_t row = row0 + k;
                if (row < cap) {
                    oid[row] = id;
                    oval[row] = val;
                } else {
                    over = true;
                }
            }
        }
    }
#endif
    if (__any(over) && lane == 0) atomicOr(&st->capacity, 1u);
    if (__any(vbad) && lane == 0) atomicOr(&st->fast_fail, 1u);  // (CHEAP: a start not a record)
#if NXG_F64X_PROF
    if (threadIdx.x == 0 && blockIdx.x < 16384) {
        nxg_f64x_st[4][blockIdx.x] = __builtin_amdgcn_s_memrealtime();
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        nxg_f64x_st[5][blockIdx.x] = ((uint64_t)xcc << 32) | hw;
    }
#endif
}

}  // namespace

// workgroups of a range of R bytes (one look-back word each)
static uint64_t f64x_wgs(uint64_t R) { return (R + WGB - 1) / WGB; }
// (one look-back per wave instead, 16 KiB units: 0.120 vs 0.110 ms at 10^7 -- the inclusive front
// crosses four times the units)
uint64_t nxg_dec_f64x_groups(uint64_t W) { return f64x_wgs(W); }

#if NXG_F64X_PROF
// diagnostic build only (not ABI): the stamps of the last single-pass decode, 6 x 16384 u64
extern "C" int nxg_debug_f64x_stamps(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(nxg_f64x_st), sizeof(nxg_f64x_st), 0,
                                    hipMemcpyDeviceToHost);
}
#endif

// Decodes the records that start in [begin, end) of a frame of W bytes (a whole frame: 0, W).
// `tstat` holds nxg_dec_f64x_groups(end - begin) epoch-tagged words (no initialisation needed).
// The range's entry (first record start at or past begin) and exit (at or past end), relative to
// begin and + 1, go to DevStatus.diag[2] / diag[3].
hipError_t nxg_launch_dec_f64x_range(const uint8_t* wire, uint64_t W, uint64_t begin,
                                     uint64_t end, uint64_t* oid, uint64_t* oval, uint64_t cap,
                                     uint64_t* tstat, uint32_t epoch, DevStatus* st,
                                     hipStream_t s) {
    if (begin > end || end > W) return hipErrorInvalidValue;
    const uint64_t ng = f64x_wgs(end - begin);
    if (ng == 0) return hipSuccess;
    if (ng > 0x7fffffffull) return hipErrorInvalidValue;
    const XRange rg{W - begin, end - begin, begin < 64 ? begin : 64, begin == 0};
    hipLaunchKernelGGL(nxg_f64x_kernel, dim3((uint32_t)ng), dim3(TPB), 0, s, wire + begin, rg, oid,
                       oval, cap, tstat, epoch, st, nxg_take_zero_slot(), nxg_patience);
    return hipGetLastError();
}

hipError_t nxg_launch_dec_f64x(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                               uint64_t cap, uint64_t* tstat, uint32_t epoch, DevStatus* st,
                               hipStream_t s) {
    return nxg_launch_dec_f64x_range(wire, W, 0, W, oid, oval, cap, tstat, epoch, st, s);
}
