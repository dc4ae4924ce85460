// nxg_encode_f64.hip -- single-pass encode of (id u64[N], f64 bits u64[N]) to wire bytes.
//
// Replaces the handle_updates -> queue_send loop (netidx/src/publisher/server.rs:610-612,
// netidx/src/channel.rs:177-202) for a batch of From::Update(Id, F64). It emits, per record,
// exactly what len_wrapped_encode (pack.rs:527-535) + the derived enum encode
// (netidx-derive/src/lib.rs:289-381) + Value::encode (netidx-value/src/lib.rs:404-407) write:
//     varint(L) 04 varint(id) 09 f64be,   L = lw(1 + vl(id) + 9)
//
// One tile = TPB threads x RPT records.
// 1. Each thread loads its records (16-byte vector loads) and computes their lengths.
// 2. A block scan gives each record's offset inside the tile.
// 3. A decoupled look-back over tile byte counts gives the tile's output offset.
// 4. Records are serialised into LDS at their final 16-byte phase. The tile then leaves LDS as aligned 16-byte stores, plus byte stores for the two partial
//    16-byte blocks it shares with its neighbours. The staging holds STGB bytes per record; a
//    tile that needs more (ids >= 2^28 throughout) writes its records to global memory byte by
//    byte instead.
#include "nxg_device.h"

using namespace f64enc;

namespace {
// Tuning (scripts/probe_enc.hip, profiles/r01f_probe_enc_1e7.log; 10^7 records on one box):
// 4 -> 8 records per thread 0.098 -> 0.081 ms (6, 12, 16: 0.087, 0.086, 0.098), staging 21 -> 15
// bytes per record (5 workgroups per CU by LDS instead of 3), nontemporal frame stores
// 0.081 -> 0.070 ms; nontemporal column loads were slower (0.094), and so were dword LDS writes.
#ifndef NXG_ENC_RPT
#define NXG_ENC_RPT 8
#endif
#ifndef NXG_ENC_STGB
#define NXG_ENC_STGB 15
#endif
#ifndef NXG_ENC_NT
#define NXG_ENC_NT 2  // bit 0: nontemporal column loads, bit 1: nontemporal frame stores
#endif
constexpr int ERPT = NXG_ENC_RPT;
constexpr int ETILE = TPB * ERPT;
constexpr int MAXB_ALL = ETILE * NXG_ENC_STGB + 32;
static_assert(NXG_ENC_STGB >= 12 && NXG_ENC_STGB <= 21, "staging bytes per record");

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

// The slow path for a tile whose records exceed the staging: bytes straight to the frame.
NXG_DEV void put_rec_global(uint8_t* out, uint64_t o, uint64_t id, uint64_t val) {
    const uint32_t L = rec_len(id);
    out[o++] = (uint8_t)L;
    out[o++] = 4;
    uint64_t v = id;
    while (v >= 0x80) {
        out[o++] = (uint8_t)((v & 0x7f) | 0x80);
        v >>= 7;
    }
    out[o++] = (uint8_t)v;
    out[o++] = 9;
#pragma unroll
    for (int i = 7; i >= 0; i--) out[o++] = (uint8_t)(val >> (8 * i));
}
// The exclusive byte prefix of `tile`, by wave 0 of its workgroup: a decoupled look-back over
// the tiles' published byte counts (lane l polls tile pred - l) that never depends on another
// workgroup being scheduled. A predecessor that has published nothing after kPatience polls has
// its byte count computed here from its ids (16 KiB of reads), so the look-back always
// progresses: dispatch is in order only per XCD, and on a GPU shared by several processes an XCD
// can fall behind with the awaited workgroup not yet dispatched (seen with 2-3 processes on one
// device); a ticket counter instead cost 66 us at 10^7 records (one contended atomic per tile).
NXG_DEV uint64_t lookback_selfhelp(const uint64_t* tstat, uint32_t tile, uint32_t epoch,
                                   const uint64_t* __restrict__ id, uint64_t n, uint32_t lane,
                                   uint32_t patience) {
    // a hole's byte count from its ids
    return lookback_selfhelp_fn(tstat, tile, epoch, patience, [&](uint64_t t) -> uint64_t {
        const uint64_t r0 = t * ETILE;
        uint64_t b = 0;
        for (uint64_t r = r0 + lane; r < r0 + ETILE && r < n; r += 64) b += rec_len(id[r]);
        return wave_sum<uint64_t>(b);
    });
}
}  // namespace

__global__ __launch_bounds__(TPB) void nxg_enc_f64_kernel(
    const uint64_t* __restrict__ id, const uint64_t* __restrict__ val, uint64_t n,
    uint8_t* __restrict__ out, uint64_t cap, uint64_t* __restrict__ tstat, uint32_t ntiles,
    uint32_t epoch, DevStatus* __restrict__ st, DevStatus* zst, uint32_t patience) {
    zero_status(zst);
    __shared__ __attribute__((aligned(16))) uint8_t stg[MAXB_ALL];
    __shared__ uint32_t scan_tmp[4];
    __shared__ uint64_t sh_base;

    const uint32_t tid = threadIdx.x, lane = tid & 63;
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t r0 = (uint64_t)tile * ETILE + (uint64_t)tid * ERPT;
        uint64_t ids[ERPT], vals[ERPT];
        if (r0 + ERPT <= n) {
#pragma unroll
            for (int k = 0; k < ERPT; k += 2) {
                if (NXG_ENC_NT & 1) {
                    typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
                    const u64x2 a = __builtin_nontemporal_load(
                        reinterpret_cast<const u64x2*>(id + r0 + k));
                    const u64x2 c = __builtin_nontemporal_load(
                        reinterpret_cast<const u64x2*>(val + r0 + k));
                    ids[k] = a.x; ids[k + 1] = a.y;
                    vals[k] = c.x; vals[k + 1] = c.y;
                } else {
                    const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(id + r0 + k);
                    const ulonglong2 c = *reinterpret_cast<const ulonglong2*>(val + r0 + k);
                    ids[k] = a.x; ids[k + 1] = a.y;
                    vals[k] = c.x; vals[k + 1] = c.y;
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < ERPT; k++) {
                ids[k] = r0 + k < n ? id[r0 + k] : 0;
                vals[k] = r0 + k < n ? val[r0 + k] : 0;
            }
        }
        uint32_t mylen = 0;
#pragma unroll
        for (int k = 0; k < ERPT; k++) mylen += (r0 + k < n) ? rec_len(ids[k]) : 0u;
        uint32_t tbytes;
        const uint32_t off = block_excl_scan<uint32_t, TPB>(mylen, scan_tmp, &tbytes);
        if (tid == 0) st_agent(&tstat[tile], lb_word(tile == 0 ? kFlagInc : kFlagAgg, epoch, tbytes));

        // decoupled look-back over tile byte counts (wave 0)
        if (tid < 64) {
            uint64_t base = 0;
            if (tile != 0) {
                base = lookback_selfhelp(tstat, tile, epoch, id, n, lane, patience);
                if (lane == 0) st_agent(&tstat[tile], lb_word(kFlagInc, epoch, base + tbytes));
            }
            if (lane == 0) sh_base = base;
        }
        __syncthreads();
        const uint64_t base = sh_base;
        const uint32_t phase = (uint32_t)(base & 15u);

        const uint64_t end = base + tbytes;
        if (base <= kMaxBatch && kMaxBatch < end) {  // the first frame boundary is in this tile
            uint64_t o = base + off;
#pragma unroll
            for (int k = 0; k < ERPT; k++)
                if (r0 + k < n) {
                    note_split(st, o, rec_len(ids[k]));
                    o += rec_len(ids[k]);
                }
        }
        if (out && end > cap) {
            if (tid == 0) atomicOr(&st->capacity, 1u);
        } else if (out && phase + tbytes > (uint32_t)(MAXB_ALL - 16)) {
            // more bytes than the staging holds: straight to the frame, byte by byte
            uint64_t o = base + off;
#pragma unroll
            for (int k = 0; k < ERPT; k++)
                if (r0 + k < n) {
                    put_rec_global(out, o, ids[k], vals[k]);
                    o += rec_len(ids[k]);
                }
        } else if (out) {
            uint32_t o = phase + off;
#pragma unroll
            for (int k = 0; k < ERPT; k++)
                if (r0 + k < n) o = put_rec(stg, o, ids[k], vals[k]);
            __syncthreads();
            if (tbytes) {
                const uint64_t gb0 = base & ~15ull;
                const uint32_t nblk = (uint32_t)((end - gb0 + 15) >> 4);
                for (uint32_t b = tid; b < nblk; b += TPB) {
                    const uint64_t g = gb0 + 16ull * b;
                    const uint8_t* src = stg + 16 * b;
                    if (g >= base && g + 16 <= end) {
                        typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
                        const u32x4v x = *reinterpret_cast<const u32x4v*>(src);
                        if (NXG_ENC_NT & 2)
                            __builtin_nontemporal_store(x, reinterpret_cast<u32x4v*>(out + g));
                        else
                            *reinterpret_cast<u32x4v*>(out + g) = x;
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

uint64_t nxg_enc_f64_tiles(uint64_t n) { return (n + ETILE - 1) / ETILE; }

hipError_t nxg_launch_enc_f64(const uint64_t* id, const uint64_t* val, uint64_t n, uint8_t* out,
                              uint64_t cap, uint64_t* tstat, uint32_t epoch, DevStatus* st,
                              int grid, hipStream_t s) {
    const uint64_t nt = nxg_enc_f64_tiles(n);
    if (nt == 0) return hipSuccess;
    const uint64_t g = grid <= 0 ? nt : (nt < (uint64_t)grid ? nt : (uint64_t)grid);
    hipLaunchKernelGGL(nxg_enc_f64_kernel, dim3(g), dim3(TPB), 0, s, id, val, n, out, cap, tstat,
                       (uint32_t)nt, epoch, st, nxg_take_zero_slot(), nxg_patience);
    return hipGetLastError();
}

int nxg_occupancy_enc_f64() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, nxg_enc_f64_kernel, TPB, 0) != hipSuccess)
        return 1;
    return n;
}
