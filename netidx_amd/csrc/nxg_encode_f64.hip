// nxg_encode_f64.hip -- single-pass encode of (id u64[N], f64 bits u64[N]) to wire bytes.
//
// Replaces the handle_updates -> queue_send loop (netidx/src/publisher/server.rs:610-612,
// netidx/src/channel.rs:177-202) for a batch of From::Update(Id, F64). It emits, per record,
// exactly what len_wrapped_encode (pack.rs:527-535) + the derived enum encode
// (netidx-derive/src/lib.rs:289-381) + Value::encode (netidx-value/src/lib.rs:404-407) write:
//     varint(L) 04 varint(id) 09 f64be,   L = lw(1 + vl(id) + 9)
//
// One tile = 1024 records: 256 threads x 4 records.
// 1. Each thread loads its records (16-byte vector loads) and computes their lengths.
// 2. A block scan gives each record's offset inside the tile.
// 3. A decoupled look-back over tile byte counts gives the tile's output offset.
// 4. Records are serialised into LDS at their final 16-byte phase. The tile then leaves LDS as
//    aligned 16-byte stores, plus byte stores for the two partial 16-byte blocks it shares with
//    its neighbours.
#include "nxg_device.h"

using namespace f64enc;

namespace {
constexpr int MAXB_ALL = TILE * 21 + 32;  // worst case: 10-byte ids -> 21-byte records

NXG_DEV uint32_t rec_len(uint64_t id) { return (uint32_t)lwlen(1 + vl64(id) + 9); }

NXG_DEV uint32_t put_rec(uint8_t* stg, uint32_t o, uint64_t id, uint64_t val) {
    const uint32_t L = rec_len(id);
    stg[o++] = (uint8_t)L;  // L <= 21 < 128: one varint byte
    stg[o++] = 4;
    uint64_t v = id;
    while (v >= 0x80) {
        stg[o++] = (uint8_t)((v & 0x7f) | 0x80);
        v >>= 7;
    }
    stg[o++] = (uint8_t)v;
    stg[o++] = 9;
#pragma unroll
    for (int i = 7; i >= 0; i--) stg[o++] = (uint8_t)(val >> (8 * i));
    return o;
}
}  // namespace

__global__ __launch_bounds__(TPB) void nxg_enc_f64_kernel(
    const uint64_t* __restrict__ id, const uint64_t* __restrict__ val, uint64_t n,
    uint8_t* __restrict__ out, uint64_t cap, uint64_t* __restrict__ tstat, uint32_t ntiles,
    uint32_t epoch, DevStatus* __restrict__ st, DevStatus* zst) {
    zero_status(zst);
    __shared__ __attribute__((aligned(16))) uint8_t stg[MAXB_ALL];
    __shared__ uint32_t scan_tmp[4];
    __shared__ uint64_t sh_base;

    const uint32_t tid = threadIdx.x, lane = tid & 63;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t r0 = (uint64_t)tile * TILE + (uint64_t)tid * RPT;
        uint64_t ids[RPT], vals[RPT];
        if (r0 + RPT <= n) {
            const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(id + r0);
            const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(id + r0 + 2);
            const ulonglong2 c = *reinterpret_cast<const ulonglong2*>(val + r0);
            const ulonglong2 d = *reinterpret_cast<const ulonglong2*>(val + r0 + 2);
            ids[0] = a.x; ids[1] = a.y; ids[2] = b.x; ids[3] = b.y;
            vals[0] = c.x; vals[1] = c.y; vals[2] = d.x; vals[3] = d.y;
        } else {
#pragma unroll
            for (int k = 0; k < RPT; k++) {
                ids[k] = r0 + k < n ? id[r0 + k] : 0;
                vals[k] = r0 + k < n ? val[r0 + k] : 0;
            }
        }
        uint32_t mylen = 0;
#pragma unroll
        for (int k = 0; k < RPT; k++) mylen += (r0 + k < n) ? rec_len(ids[k]) : 0u;
        uint32_t tbytes;
        const uint32_t off = block_excl_scan<uint32_t, TPB>(mylen, scan_tmp, &tbytes);
        if (tid == 0) st_agent(&tstat[tile], lb_word(tile == 0 ? kFlagInc : kFlagAgg, epoch, tbytes));

        // decoupled look-back over tile byte counts (wave 0)
        if (tid < 64) {
            uint64_t base = 0;
            if (tile != 0) {
                bool give_up;
                base = lookback_prefix<LB_U>(tstat, tile, epoch, nullptr, give_up);
                if (give_up && lane == 0) atomicOr(&st->timeout, 1u);
                if (lane == 0) st_agent(&tstat[tile], lb_word(kFlagInc, epoch, base + tbytes));
            }
            if (lane == 0) sh_base = base;
        }
        __syncthreads();
        const uint64_t base = sh_base;
        const uint32_t phase = (uint32_t)(base & 15u);

        if (out) {
            uint32_t o = phase + off;
#pragma unroll
            for (int k = 0; k < RPT; k++)
                if (r0 + k < n) o = put_rec(stg, o, ids[k], vals[k]);
            __syncthreads();
            const uint64_t end = base + tbytes;
            if (end > cap) {
                if (tid == 0) atomicOr(&st->capacity, 1u);
            } else if (tbytes) {
                const uint64_t gb0 = base & ~15ull;
                const uint32_t nblk = (uint32_t)((end - gb0 + 15) >> 4);
                for (uint32_t b = tid; b < nblk; b += TPB) {
                    const uint64_t g = gb0 + 16ull * b;
                    const uint8_t* src = stg + 16 * b;
                    if (g >= base && g + 16 <= end) {
                        *reinterpret_cast<uint4*>(out + g) = *reinterpret_cast<const uint4*>(src);
                    } else {
                        for (int k = 0; k < 16; k++)
                            if (g + k >= base && g + k < end) out[g + k] = src[k];
                    }
                }
            }
        }
        if (tile == ntiles - 1 && tid == 0) {
            st->total_bytes = base + tbytes;
            st->n_rows = n;
        }
        __syncthreads();
    }
}

hipError_t nxg_launch_enc_f64(const uint64_t* id, const uint64_t* val, uint64_t n, uint8_t* out,
                              uint64_t cap, uint64_t* tstat, uint32_t epoch, DevStatus* st,
                              int grid, hipStream_t s) {
    const uint64_t nt = (n + TILE - 1) / TILE;
    if (nt == 0) return hipSuccess;
    const uint64_t g = grid <= 0 ? nt : (nt < (uint64_t)grid ? nt : (uint64_t)grid);
    hipLaunchKernelGGL(nxg_enc_f64_kernel, dim3(g), dim3(TPB), 0, s, id, val, n, out, cap, tstat,
                       (uint32_t)nt, epoch, st, nxg_zero_slot);
    return hipGetLastError();
}

int nxg_occupancy_enc_f64() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, nxg_enc_f64_kernel, TPB, 0) != hipSuccess)
        return 1;
    return n;
}
