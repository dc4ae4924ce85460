// nxg_decode_f64_x.hip -- homogeneous-f64 decode of ANY f64 frame in one pass, for gfx950: the
// decoder for frames whose record lengths vary record to record (ids in arbitrary order: a batch
// updating an arbitrary subset of a publisher's values, netidx/src/publisher/mod.rs:776-845), on
// which the length-run decoder (nxg_decode_f64_run.hip) gives up. Replaces the receive_batch_fn
// loop (netidx/src/channel.rs:504-521) for frames of From::Update(Id, F64) messages with ids of
// 1..5 varint bytes (< 2^35), records of 12..16 bytes.
//
// One wave per 4 KiB sub-tile, four per workgroup, no wave waits on anything but lower-numbered
// workgroups (a decoupled look-back), so any number of these decodes can share the GPU:
//   1. the sub-tile and 192 bytes around it into LDS (one coalesced pass);
//   2. lane j: the merge point of its 64-byte chunk (nxg_f64_rec16.h) and a walk from it to the
//      next lane's, every record checked completely; lane 0 starts one chunk early, so the walks
//      cover every record that STARTS in the sub-tile, and each is counted by one lane;
//   3. a block scan of the lanes' counts, the workgroup's total to the look-back, its first row
//      from it;
//   4. the walks again (LDS only), each record decoded into an LDS row image, then the wave's rows
//      leave as coalesced 8-byte column stores.
// The true chain starts at byte 0 (lane 0 of sub-tile 0 walks from there) and every merge point
// lies on it, so consecutive lanes, waves and workgroups meet by construction: a walk that does
// not land exactly on the next merge point, a record that fails its check, or walks that do not
// merge raise fast_fail, and the host reruns the frame on the mixed/general decoders.
#include "nxg_device.h"
#include "nxg_f64_rec16.h"

namespace f64x {
constexpr uint32_t SUB = 4096;          // bytes per wave
constexpr uint32_t HALO = 128;          // look-ahead bytes past the sub-tile
constexpr uint32_t XLO = 64;            // image offset of the sub-tile's first byte
constexpr uint32_t XHI = XLO + SUB;
constexpr uint32_t IMGB = XHI + HALO;   // image bytes
constexpr int TPB = 256;
constexpr int WAVES = TPB / 64;
constexpr uint32_t MAXR = SUB / 12 + 2;  // rows per sub-tile (records start in it, >= 12 bytes)
}  // namespace f64x

namespace {
using namespace f64x;
using namespace f64rec16;

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
    const uint64_t a0 = ((uint64_t)blockIdx.x * WAVES + w) * SUB;
    uint8_t* buf = img[w];
    uint32_t xa = 0, xb = 0, n = 0;
    bool bad = false;
    if (a0 < W) {
        const uint64_t ib = a0 - XLO;  // frame position of image byte 0 (wraps for a0 = 0)
#pragma unroll
        for (uint32_t i = 0; i < (IMGB + 1023) / 1024; i++) {
            const uint32_t off = i * 1024 + lane * 16;
            if (off < IMGB) {
                const int64_t pos = (int64_t)a0 - (int64_t)XLO + (int64_t)off;
                const uint4 v = pos >= 0 ? ld16g(wire, (uint64_t)pos, W) : ld16_pre(wire, pos, W, 0);
                *reinterpret_cast<uint4*>(buf + off) = v;
            }
        }
        wave_lds_order();
        // segments: lane 0 from the merge point of the chunk before a0 (the frame start for
        // a0 = 0), lane j >= 1 from chunk j's; each ends at the next lane's start, lane 63 at the
        // merge point of the chunk at a0 + 4096
        const uint32_t xhi = XLO + (W - a0 < SUB ? (uint32_t)(W - a0) : SUB);
        xa = lane == 0 ? (a0 == 0 ? XLO : merge16(buf, 0, ib, W)) : merge16(buf, XLO + lane * 64, ib, W);
        xb = wave_next(xa);
        if (lane == 63) xb = merge16(buf, XHI, ib, W);
        bad = xa == FAILX || xb == FAILX || xa > xb || (lane == 0 && xa > XLO);
        if (!bad) {
            uint32_t pos = xa;
            int guard = 0;
            while (pos < xb && guard < 24) {
                uint32_t L;
                if (pos < xhi) {
                    uint32_t e0, e1, e2, e3;
                    lds16(buf, pos, e0, e1, e2, e3);
                    L = rec_check16(e0, e1, W - (ib + pos));
                    if (!L) break;
                    if (pos >= XLO) n++;
                } else {
                    // past the sub-tile: step by the length byte (the next sub-tile checks it)
                    L = buf[pos];
                    if (L - 12u > 4u) break;
                }
                pos += L;
                guard++;
            }
            bad = pos != xb;
        }
    }
    const bool wbad = __any(bad);
    if (wbad && lane == 0) atomicOr(&st->fast_fail, 1u);
    // rows: this lane's first row within the workgroup, the workgroup's first row in the frame
    uint64_t total;
    const uint64_t excl = block_excl_scan<uint64_t, TPB>((uint64_t)n, scan_tmp, &total);
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
    if (a0 >= W || wbad) return;  // (a bad sub-tile has raised fast_fail: the frame is rerun)
    // the wave's rows: [wbase, wbase + nw) of the frame; lane's rows from (excl - wexcl) within
    const uint64_t wexcl = (uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)excl) |
                           ((uint64_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(excl >> 32)) << 32);
    const uint64_t wbase = sh_base + wexcl;
    const uint32_t nw = (uint32_t)wave_sum<uint32_t>(n);
    {
        const uint32_t xhi = XLO + (W - a0 < SUB ? (uint32_t)(W - a0) : SUB);
        uint32_t k = (uint32_t)(excl - wexcl);
        uint32_t pos = xa;
        while (pos < xb && pos < xhi) {
            uint32_t e0, e1, e2, e3;
            lds16(buf, pos, e0, e1, e2, e3);
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
    }
    wave_lds_order();
    bool over = false;
    for (uint32_t i = lane; i < nw; i += 64) {
        const uint64_t row = wbase + i;
        if (row < cap) {
            oid[row] = rows[w][i][0];
            oval[row] = rows[w][i][1];
        } else {
            over = true;
        }
    }
    if (__any(over) && lane == 0) atomicOr(&st->capacity, 1u);
}

}  // namespace

uint64_t nxg_dec_f64x_groups(uint64_t W) {
    return (W + (uint64_t)SUB * WAVES - 1) / ((uint64_t)SUB * WAVES);
}

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
