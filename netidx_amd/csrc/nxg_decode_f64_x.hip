// nxg_decode_f64_x.hip -- homogeneous-f64 decode of ANY f64 frame in one pass, for gfx950: the
// decoder for frames whose record lengths vary record to record (ids in arbitrary order: a batch
// updating an arbitrary subset of a publisher's values, netidx/src/publisher/mod.rs:776-845), on
// which the length-run decoder (nxg_decode_f64_run.hip) gives up. Replaces the receive_batch_fn
// loop (netidx/src/channel.rs:504-521) for frames of From::Update(Id, F64) messages with ids of
// 1..5 varint bytes (< 2^35), records of 12..16 bytes.
//
// A wave takes SPW consecutive 4 KiB sub-tiles, a workgroup four waves (64 KiB), and no wave
// waits on anything but lower-numbered workgroups (a decoupled look-back), so any number of these
// decodes can share the GPU:
//   1. per sub-tile: its bytes and 192 around them into LDS (one coalesced pass; dwords stored
//      swizzled, SwzImg, so that the lanes' 64-byte-strided reads do not pile onto two banks);
//      lane j: the merge point of its 64-byte chunk (nxg_f64_rec16.h) and a walk from it to the
//      next lane's, every record checked completely; lane 0 starts one chunk early, so the walks
//      cover every record that STARTS in the sub-tile, and each is counted by one lane. The
//      walks' ends and counts stay in registers;
//   2. a block scan of the counts, the workgroup's total to the look-back, its first row from it
//      (one look-back per 64 KiB: the wait on the look-back's front is what bounded a workgroup
//      per 16 KiB, at 178 us for 10^7 records);
//   3. per sub-tile: the image again (from L2), the walks again, each record decoded into an LDS
//      row image, then the wave's rows leave as coalesced 8-byte column stores.
// The true chain starts at byte 0 (lane 0 of sub-tile 0 walks from there) and every merge point
// lies on it, so consecutive lanes, waves and workgroups meet by construction: a walk that does
// not land exactly on the next merge point, a record that fails its check, or walks that do not
// merge raise fast_fail, and the host reruns the frame on the mixed/general decoders.
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
}  // namespace f64x

namespace {
using namespace f64x;
using namespace f64rec16;

// the image of the sub-tile at a0: frame bytes [a0 - 64, a0 + 4096 + 128), dwords swizzled
NXG_DEV void load_image(uint8_t* buf, const uint8_t* __restrict__ wire, uint64_t a0, uint64_t W,
                        uint32_t lane) {
    uint32_t* bw = reinterpret_cast<uint32_t*>(buf);
    wave_lds_order();  // the previous image's reads are issued
#pragma unroll
    for (uint32_t i = 0; i < (IMGB + 1023) / 1024; i++) {
        const uint32_t off = i * 1024 + lane * 16;
        if (off < IMGB) {
            const int64_t pos = (int64_t)a0 - (int64_t)XLO + (int64_t)off;
            const uint4 v = pos >= 0 ? ld16g(wire, (uint64_t)pos, W) : ld16_pre(wire, pos, W, 0);
            const uint32_t q = off >> 2;
            bw[SwzImg::sw(q)] = v.x;
            bw[SwzImg::sw(q + 1)] = v.y;
            bw[SwzImg::sw(q + 2)] = v.z;
            bw[SwzImg::sw(q + 3)] = v.w;
        }
    }
    wave_lds_order();
}

__global__ __launch_bounds__(TPB) void nxg_f64x_kernel(const uint8_t* __restrict__ wire,
                                                       uint64_t W, uint64_t* __restrict__ oid,
                                                       uint64_t* __restrict__ oval, uint64_t cap,
                                                       uint64_t* tstat, uint32_t epoch,
                                                       DevStatus* __restrict__ st,
                                                       DevStatus* zst) {
    zero_status(zst);
    __shared__ __attribute__((aligned(16))) uint8_t img[WAVES][IMGB];
    __shared__ __attribute__((aligned(16))) uint64_t rows[WAVES][MAXR][2];
    __shared__ uint64_t scan_tmp[WAVES];
    __shared__ uint64_t sh_base;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t w0 = (uint64_t)blockIdx.x * WGB + (uint64_t)w * SUB * SPW;  // the wave's bytes
    uint8_t* buf = img[w];
    const SwzImg im{buf};
    uint32_t xa[SPW], xb[SPW], n[SPW];
    bool bad = false;
#pragma unroll
    for (int s = 0; s < SPW; s++) {
        xa[s] = xb[s] = n[s] = 0;
        const uint64_t a0 = w0 + (uint64_t)s * SUB;
        if (a0 >= W) continue;
        load_image(buf, wire, a0, W, lane);
        const uint64_t ib = a0 - XLO;  // frame position of image byte 0 (wraps for a0 = 0)
        // segments: lane 0 from the merge point of the chunk before a0 (the frame start for
        // a0 = 0), lane j >= 1 from chunk j's; each ends at the next lane's start, lane 63 at
        // the merge point of the chunk at a0 + 4096
        const uint32_t xhi = XLO + (W - a0 < SUB ? (uint32_t)(W - a0) : SUB);
        uint32_t x0 = lane == 0 ? (a0 == 0 ? XLO : merge16i(im, 0, ib, W))
                                : merge16i(im, XLO + lane * 64, ib, W);
        uint32_t x1 = wave_next(x0);
        if (lane == 63) x1 = merge16i(im, XHI, ib, W);
        bool b = x0 == FAILX || x1 == FAILX || x0 > x1 || (lane == 0 && x0 > XLO);
        uint32_t c = 0;
        if (!b) {
            uint32_t pos = x0;
            int guard = 0;
            while (pos < x1 && guard < 24) {
                uint32_t L;
                if (pos < xhi) {
                    uint32_t e0, e1, e2, e3;
                    lds16i(im, pos, e0, e1, e2, e3);
                    L = rec_check16(e0, e1, W - (ib + pos));
                    if (!L) break;
                    if (pos >= XLO) c++;
                } else {
                    // past the sub-tile: step by the length byte (the next sub-tile checks it)
                    L = im.byte(pos);
                    if (L - 12u > 4u) break;
                }
                pos += L;
                guard++;
            }
            b = pos != x1;
        }
        bad |= b;
        xa[s] = x0;
        xb[s] = x1;
        n[s] = c;
    }
    const bool wbad = __any(bad);
    if (wbad && lane == 0) atomicOr(&st->fast_fail, 1u);
    // rows: the block scan orders the lanes' counts wave by wave, sub-tile by sub-tile within a
    // wave; here the lane's total, and below each sub-tile's wave-level offsets
    uint32_t ntot = 0;
#pragma unroll
    for (int s = 0; s < SPW; s++) ntot += n[s];
    uint64_t total;
    const uint64_t excl = block_excl_scan<uint64_t, TPB>((uint64_t)ntot, scan_tmp, &total);
    if (w == 0) {
        uint64_t base = 0;
        if (blockIdx.x == 0) {
            if (lane == 0) st_agent(&tstat[0], lb_word(kFlagInc, epoch, total));
        } else {
            if (lane == 0) st_agent(&tstat[blockIdx.x], lb_word(kFlagAgg, epoch, total));
            bool give_up;
            base = lookback_prefix<4>(tstat, blockIdx.x, epoch, nullptr, give_up);
            if (give_up) {
                if (lane == 0) {
                    atomicOr(&st->timeout, 1u);
                    atomicOr(&st->fast_fail, 1u);
                }
            } else if (lane == 0) {
                st_agent(&tstat[blockIdx.x], lb_word(kFlagInc, epoch, base + total));
            }
        }
        if (lane == 0) sh_base = base;
        if (blockIdx.x == gridDim.x - 1 && lane == 0) {
            st->n_rows = base + total;
            st->path = 1;
        }
    }
    __syncthreads();
    if (wbad) return;  // (a bad sub-tile has raised fast_fail: the frame is rerun)
    // the wave's first row: the block prefix of its lane 0
    uint64_t row0 = sh_base + ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)excl) |
                               ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(excl >> 32)) << 32));
    bool over = false;
#pragma unroll
    for (int s = 0; s < SPW; s++) {
        const uint64_t a0 = w0 + (uint64_t)s * SUB;
        if (a0 >= W) break;
        const uint32_t inc = wave_incl_scan<uint32_t>(n[s]);
        const uint32_t nw = wave_last<uint32_t>(inc);
        if (SPW > 1) load_image(buf, wire, a0, W, lane);
        const uint32_t xhi = XLO + (W - a0 < SUB ? (uint32_t)(W - a0) : SUB);
        uint32_t k = inc - n[s];
        uint32_t pos = xa[s];
        while (pos < xb[s] && pos < xhi) {
            uint32_t e0, e1, e2, e3;
            lds16i(im, pos, e0, e1, e2, e3);
            const uint32_t L = e0 & 0xffu;
            if (pos >= XLO) {
                uint64_t id, val;
                rec_decode16(e0, e1, e2, e3, L, id, val);
                rows[w][k][0] = id;
                rows[w][k][1] = val;
                k++;
            }
            pos += L;
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
}

}  // namespace

uint64_t nxg_dec_f64x_groups(uint64_t W) { return (W + WGB - 1) / WGB; }

// Decodes a whole frame of W bytes. `tstat` holds nxg_dec_f64x_groups(W) epoch-tagged words (no
// initialisation needed).
hipError_t nxg_launch_dec_f64x(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                               uint64_t cap, uint64_t* tstat, uint32_t epoch, DevStatus* st,
                               hipStream_t s) {
    const uint64_t ng = nxg_dec_f64x_groups(W);
    if (ng == 0) return hipSuccess;
    if (ng > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nxg_f64x_kernel, dim3((uint32_t)ng), dim3(TPB), 0, s, wire, W, oid, oval,
                       cap, tstat, epoch, st, nxg_take_zero_slot());
    return hipGetLastError();
}
