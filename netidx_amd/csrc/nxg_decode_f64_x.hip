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
}  // namespace f64x

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
#pragma unroll 1
        for (uint64_t m = cm; m; m &= m - 1) {
            const uint32_t p = (uint32_t)__builtin_ctzll(m);
            const uint32_t nx = p + im.byte(r + p);
            if (nx < 64u) slo |= 1ull << nx;
            else shi |= 1ull << (nx - 64u);
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
NXG_DEV uint64_t wg_count(const uint8_t* __restrict__ wire, const XRange& rg, uint8_t* buf,
                          uint64_t g, uint32_t lane, DevStatus* st) {
    static_assert(IMGB == kXImg && SUB == kXSub && XLO == kXLo, "the exact path's image");
    uint32_t c, en, xx;
    bool b = false, ov = false;
    exact_tile<false, (uint32_t)WGB>(wire, rg.W, rg.R, rg.first, rg.pre, g, buf, lane, 0, nullptr,
                                     nullptr, 0, c, en, xx, b, ov);
    if (b && lane == 0) atomicOr(&st->fast_fail, 1u);
    return c;
}

__global__ __launch_bounds__(TPB, NXG_F64X_OCC) void nxg_f64x_kernel(const uint8_t* __restrict__ wire,
                                                       XRange rg, uint64_t* __restrict__ oid,
                                                       uint64_t* __restrict__ oval, uint64_t cap,
                                                       uint64_t* tstat, uint32_t epoch,
                                                       DevStatus* __restrict__ st,
                                                       DevStatus* zst, uint32_t patience) {
    zero_status(zst);
    const uint64_t W = rg.W, R = rg.R;
    __shared__ __attribute__((aligned(16))) uint8_t img[WAVES][IMGB];
    __shared__ __attribute__((aligned(16))) uint64_t rows[WAVES][MAXR][2];
    __shared__ uint64_t scan_tmp[WAVES];
    __shared__ uint64_t sh_base;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // (blockIdx order with self-help; a ticket counter measured 0.104 -> 0.120 ms at 10^7)
    const uint32_t bid = blockIdx.x;
    const uint64_t w0 = (uint64_t)bid * WGB + (uint64_t)w * SUB * SPW;  // the wave's bytes
    uint8_t* buf = img[w];
    const SwzImg im{buf};
    uint64_t Sm[SPW];
    uint32_t n[SPW];
    bool bad = false;
    Prefetch pf;
    fetch_image(pf, wire, w0, W, lane, rg.pre);
    // q: the frame position of the chain's first record start at or past the sub-tile, carried
    // from sub-tile to sub-tile of the wave (~0: not known -- the wave's first sub-tile)
    uint64_t q = ~0ull;
#pragma unroll
    for (int s = 0; s < SPW; s++) {
        Sm[s] = 0;
        n[s] = 0;
        const uint64_t a0 = w0 + (uint64_t)s * SUB;
        if (a0 >= R) continue;
        commit_image(buf, pf, lane);
        if (s + 1 < SPW && a0 + SUB < R)
            fetch_image(pf, wire, a0 + SUB, W, lane, rg.pre);  // the next, while checking
        subtile_starts(wire, rg, buf, a0, s == SPW - 1, lane, q, Sm[s], n[s], bad, st);
    }
    const bool wbad = __any(bad);
    if (wbad && lane == 0) atomicOr(&st->fast_fail, 1u);
    // rows: the block scan orders the lanes' counts wave by wave, sub-tile by sub-tile within a
    // wave; here the lane's total, and below each sub-tile's wave-level offsets
    uint32_t ntot = 0;
#pragma unroll
    for (int s = 0; s < SPW; s++) ntot += n[s];
    // the first image of the emit pass, loading during the look-back (waves 1..3; wave 0 runs the
    // look-back, whose self-help path needs the registers)
    if (SPW > 1 && w != 0) fetch_image(pf, wire, w0, W, lane, rg.pre);
    // the start masks wait in the wave's (still unused) row buffer across the look-back, so that
    // they hold no registers there
    uint32_t* stash = reinterpret_cast<uint32_t*>(rows[w]);
#pragma unroll
    for (int s = 0; s < SPW; s++) {
        stash[(3 * s) * 64 + lane] = (uint32_t)Sm[s];
        stash[(3 * s + 1) * 64 + lane] = (uint32_t)(Sm[s] >> 32);
        stash[(3 * s + 2) * 64 + lane] = n[s];
    }
    uint64_t total;
    const uint64_t excl = block_excl_scan<uint64_t, TPB>((uint64_t)ntot, scan_tmp, &total);
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
    if (wbad) return;  // (a bad sub-tile has raised fast_fail: the frame is rerun)
    if (SPW > 1 && w == 0) fetch_image(pf, wire, w0, W, lane, rg.pre);
#pragma unroll
    for (int s = 0; s < SPW; s++) {
        Sm[s] = (uint64_t)stash[(3 * s) * 64 + lane] | ((uint64_t)stash[(3 * s + 1) * 64 + lane] << 32);
        n[s] = stash[(3 * s + 2) * 64 + lane];
    }
    wave_lds_order();  // (the row buffer is written below)
    // the wave's first row: the block prefix of its lane 0
    uint64_t row0 = sh_base + ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)excl) |
                               ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(excl >> 32)) << 32));
    bool over = false, vbad = false;
#pragma unroll
    for (int s = 0; s < SPW; s++) {
        const uint64_t a0 = w0 + (uint64_t)s * SUB;
        if (a0 >= R) break;
        const uint32_t inc = wave_incl_scan<uint32_t>(n[s]);
        const uint32_t nw = wave_last<uint32_t>(inc);
        if (SPW > 1) {
            commit_image(buf, pf, lane);
            if (s + 1 < SPW && a0 + SUB < R) fetch_image(pf, wire, a0 + SUB, W, lane, rg.pre);
        }
        // the lane's records (at most 6 start in 64 bytes), loaded together
        uint32_t k = inc - n[s];
        uint64_t m = Sm[s];
        const uint32_t r = XLO + lane * 64;
        uint32_t pp[6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            pp[i] = m ? (uint32_t)__builtin_ctzll(m) : 0u;
            m &= m - 1;
        }
        uint32_t e[6][4];
#pragma unroll
        for (int i = 0; i < 6; i++) lds16i(im, r + pp[i], e[i][0], e[i][1], e[i][2], e[i][3]);
#pragma unroll
        for (int i = 0; i < 6; i++) {
            if ((uint32_t)i < n[s]) {
                uint64_t id, val;
                if (NXG_F64X_CHEAP)
                    vbad |= rec_check16(e[i][0], e[i][1], W - (a0 + lane * 64 + pp[i])) !=
                            (e[i][0] & 0xffu);
                rec_decode16(e[i][0], e[i][1], e[i][2], e[i][3], e[i][0] & 0xffu, id, val);
                rows[w][k + i][0] = id;
                rows[w][k + i][1] = val;
            }
        }
        wave_lds_order();
        for (uint32_t i = lane; i < nw; i += 64) {
            const uint64_t row = row0 + i;
            if (row < cap) {
                oid[row] = rows[w][i][0];
                oval[row] = rows[w][i][1];
            } else {
                over = true;
            }
        }
        wave_lds_order();
        row0 += nw;
    }
    if (__any(over) && lane == 0) atomicOr(&st->capacity, 1u);
    if (__any(vbad) && lane == 0) atomicOr(&st->fast_fail, 1u);  // (CHEAP: a start not a record)
}

}  // namespace

uint64_t nxg_dec_f64x_groups(uint64_t W) { return (W + WGB - 1) / WGB; }

// Decodes the records that start in [begin, end) of a frame of W bytes (a whole frame: 0, W).
// `tstat` holds nxg_dec_f64x_groups(end - begin) epoch-tagged words (no initialisation needed).
// The range's entry (first record start at or past begin) and exit (at or past end), relative to
// begin and + 1, go to DevStatus.diag[2] / diag[3].
hipError_t nxg_launch_dec_f64x_range(const uint8_t* wire, uint64_t W, uint64_t begin,
                                     uint64_t end, uint64_t* oid, uint64_t* oval, uint64_t cap,
                                     uint64_t* tstat, uint32_t epoch, DevStatus* st,
                                     hipStream_t s) {
    if (begin > end || end > W) return hipErrorInvalidValue;
    const uint64_t ng = nxg_dec_f64x_groups(end - begin);
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
