// nxg_decode_f64_1p.hip -- single-pass homogeneous-f64 decode for gfx950 (record format:
// nxg_f64_rec.h). Replaces the receive_batch_fn loop (netidx/src/channel.rs:504-521) for frames
// in which every message is From::Update(Id, F64); anything else raises fast_fail and the host
// reruns the frame on the general decoder.
//
// Record boundaries: the merge points of nxg_f64_rec.h (the same exact, adversarially safe
// machinery as the two-pass decoder): lane j's walk from its chunk's merge point must land on the
// next lane's merge point; anything unprovable raises fast_fail.
//
// Pipeline (one launch)
// ---------------------
// Block 0 is a scanner; every other wave is a worker. Worker v of V handles tiles v, v+V, ...
// (tiles start 4032 bytes apart; lane 63's merge point is the next tile's first). Step k, with
// LAG = 1 (NXG_1P_LAG) and LAG + 1 LDS slots per wave:
//   1. stage tile t_k in LDS slot k mod (LAG+1) (its bytes were loaded during step k-1) and
//      issue the loads of t_{k+1};
//   2. merge points; each lane's chain of record starts, one length byte per step; then the
//      lane's records (at most 6) are loaded together and checked and decoded without branches
//      (32-bit id: ids of f64 records are < 2^28; 64-bit value); a wave scan numbers them; the
//      decoded records then replace the tile's image in its LDS slot, in record order; publish
//      the tile's count (agg[t_k]);
//   3. wait for t_{k-LAG}'s first record index (pre[t_{k-LAG}], published by the scanner
//      meanwhile) and copy its slot to the id / value columns with coalesced stores.
// The scanner turns agg[] into pre[] in tile order. Each step waits on the prefix of the tile
// from LAG steps before, so a slow wave elsewhere does not stall the others at once (and the
// waves stay on a compact address window, which HBM rewards); every spin is bounded (watchdog)
// and gives up once fast_fail is raised. Two 4.2 KiB slots per wave (image and decoded records
// share a slot): four 4-wave workgroups per CU.
#include "nxg_f64_rec.h"

#ifdef NXG_1P_PROBE  // scripts/probe_f64.hip only: phase cycle counters and ablation flags
__device__ uint32_t g_1p_dbg;                  // bit 0: no wait for pre[], bit 1: no stores
__device__ unsigned long long g_1p_cyc[8];     // per-phase s_memtime cycles, all waves
#define P1_FLAGS g_1p_dbg
#define P1_STAMP(i)                                    \
    do {                                               \
        const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
        cyc##i += t_ - tprev;                          \
        tprev = t_;                                    \
    } while (0)
#else
#define P1_FLAGS 0u
#define P1_STAMP(i) \
    do {            \
    } while (0)
#endif

namespace {

#ifndef NXG_1P_TPB
#define NXG_1P_TPB 256
#endif
constexpr int TPB1 = NXG_1P_TPB;
constexpr int WAVES1 = TPB1 / 64;
#ifndef NXG_1P_LAG
#define NXG_1P_LAG 1
#endif
constexpr int LAG = NXG_1P_LAG;
constexpr int NSLOT = LAG + 1;
constexpr int MAXR = f64dec::STRIDE / 12 + 1;  // records per tile (>= 12 bytes each): 337
constexpr int SCAN_K = 8;                      // scanner: tiles per thread per step
constexpr int MAXL = 6;  // records a lane owns: its span is < 64 + 15 bytes, >= 12 B each
constexpr uint32_t SLOTB = f64dec::IMG + f64dec::HALO;  // image, then its decoded records
constexpr uint32_t VALOFF = (MAXR * 4 + 7) & ~7u;       // decoded: u32 ids, then u64 values
constexpr uint32_t CNTOFF = SLOTB - 4;                  // decoded: the tile's record count
static_assert(VALOFF + MAXR * 8 <= CNTOFF, "decoded records fit the image they replace");

struct WaveLds {
    uint8_t slot[NSLOT][SLOTB] __attribute__((aligned(16)));
};
static_assert(sizeof(WaveLds) * WAVES1 <= 80 * 1024, "two workgroups per CU at least");

}  // namespace

// ---- scanner: pre[i] = records in tiles [0, i), for the longest published prefix of agg[] ----
// Steps of up to TPB1*SCAN_K tiles; never waits for a tile beyond the first unpublished one, so
// it cannot wait on a worker that waits on it. Loads and stores are coalesced (tile
// c + k*TPB1 + tid); `stg` (TPB1*SCAN_K words of LDS) holds the transpose to per-thread runs.
NXG_DEV void f64_scan(uint64_t nt, const uint64_t* agg, uint64_t* pre, uint32_t epoch,
                      DevStatus* __restrict__ st, uint64_t* stg, uint64_t t_start) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    __shared__ uint64_t scan_tmp[WAVES1];
    __shared__ uint64_t wmin[WAVES1];
    uint64_t running = 0;
    uint64_t c = 0;
    while (c < nt) {
        uint64_t v[SCAN_K];
        uint64_t fu = nt;  // first unpublished tile of the step (nt if none)
#pragma unroll
        for (int k = 0; k < SCAN_K; k++) {
            const uint64_t i = c + (uint64_t)k * TPB1 + tid;
            v[k] = i < nt ? ld_agent(&agg[i]) : lb_word(kFlagAgg, epoch, 0);
        }
#pragma unroll
        for (int k = SCAN_K - 1; k >= 0; k--) {
            const uint64_t i = c + (uint64_t)k * TPB1 + tid;
            if (i < nt && lb_flag(v[k], epoch) == 0) fu = i < fu ? i : fu;
        }
        // tile indices fit 32 bits (nt < 2^32: frames are < 2^44 bytes)
        fu = wave_min_u32(fu < 0xffffffffull ? (uint32_t)fu : 0xffffffffu);
        if (lane == 0) wmin[w] = fu;
#pragma unroll
        for (int k = 0; k < SCAN_K; k++) stg[k * TPB1 + tid] = v[k] & kValMask;
        __syncthreads();
        uint64_t F = wmin[0];
#pragma unroll
        for (int i = 1; i < WAVES1; i++) F = wmin[i] < F ? wmin[i] : F;
        const uint64_t cend = c + (uint64_t)TPB1 * SCAN_K;
        if (F > cend) F = cend;
        if (F == c) {  // nothing new: back off, then poll again
            const int stop = __syncthreads_or(
                tid == 0 && (ld_agent32(&st->fast_fail) || rt_now() - t_start > kSpinTicks));
            if (stop) {
                if (tid == 0 && !ld_agent32(&st->fast_fail)) {
                    atomicOr(&st->timeout, 1u);
                    atomicOr(&st->fast_fail, 1u);
                }
                return;
            }
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        // thread tid owns tiles c + tid*SCAN_K + [0, SCAN_K) of the transpose
        const uint64_t j0 = c + (uint64_t)tid * SCAN_K;
        uint64_t x[SCAN_K], local = 0;
#pragma unroll
        for (int k = 0; k < SCAN_K; k++) {
            x[k] = j0 + k < F ? stg[tid * SCAN_K + k] : 0ull;
            local += x[k];
        }
        uint64_t total;
        uint64_t p = running + block_excl_scan<uint64_t, TPB1>(local, scan_tmp, &total);
#pragma unroll
        for (int k = 0; k < SCAN_K; k++) {
            stg[tid * SCAN_K + k] = p;
            p += x[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < SCAN_K; k++) {
            const uint64_t i = c + (uint64_t)k * TPB1 + tid;
            if (i < F) st_agent(&pre[i], lb_word(kFlagInc, epoch, stg[k * TPB1 + tid]));
        }
        running += total;
        c = F;
        __syncthreads();  // stg is rewritten by the next step
    }
    if (tid == 0) {
        st->n_rows = running;
        st->path = 1;
    }
}

// ---- worker wave v of V ------------------------------------------------------------------------
NXG_DEV void f64_work(const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt,
                      uint64_t* __restrict__ oid, uint64_t* __restrict__ oval, uint64_t cap,
                      uint64_t* agg, const uint64_t* pre, uint32_t epoch,
                      DevStatus* __restrict__ st, uint64_t v, uint64_t V, WaveLds& L,
                      uint64_t t_start) {
    const uint32_t lane = threadIdx.x & 63;
    if (v >= nt) return;
    const uint64_t K = (nt - v + V - 1) / V;  // this wave's tiles
    const uint64_t nfull = W >= f64dec::IMG + f64dec::HALO
                               ? (W - f64dec::IMG - f64dec::HALO) / f64dec::STRIDE + 1
                               : 0;
#ifdef NXG_1P_PROBE
    uint64_t tprev = __builtin_amdgcn_s_memtime(), cyc0 = 0, cyc1 = 0, cyc2 = 0, cyc3 = 0,
             cyc4 = 0;
#endif
    TileRegs R;
    if (v < nfull) tile_load_full<false>(R, wire, v * f64dec::STRIDE, lane, nullptr);
    else tile_load(R, wire, v * f64dec::STRIDE, W, lane, nullptr);
    bool over = false;
#pragma unroll 1
    for (uint64_t k = 0; k < K + LAG; k++) {
        if (k < K) {
            const uint64_t t = k * V + v;
            P1_STAMP(4);
            wave_lds_order();
            uint8_t* img = L.slot[k % NSLOT];
            tile_store(img, R, lane);
            wave_lds_order();
            P1_STAMP(0);
            const uint64_t tn = t + V;
            if (k + 1 < K) {
                if (tn < nfull) tile_load_full<false>(R, wire, tn * f64dec::STRIDE, lane, nullptr);
                else tile_load(R, wire, tn * f64dec::STRIDE, W, lane, nullptr);
            }
            // 2. merge points, then one walk per lane from its merge point to the next lane's,
            // decoding into registers as it goes (at most MAXL records; each fully checked:
            // variant, id varint, value tag); it must land exactly on the next merge point
            const uint32_t xa = chunk_merge(img, t, W, lane);
            const uint32_t xb = wave_next(xa);
            const bool owner = lane != 63;  // lane 63's merge point is the next tile's first
            bool bad = (xa == FAIL) | (owner & ((xb == FAIL) | (xa > xb)));
            const uint64_t t0 = t * f64dec::STRIDE;
            // the chain of record starts reads one length byte per step; the records are then
            // loaded together (independent reads) and each is fully checked (rec_check: its
            // length must be the byte the chain stepped by)
            uint32_t ps[MAXL];
            uint32_t pos = xa, n = 0;
            const bool walk = owner && !bad;
#pragma unroll
            for (int q = 0; q < MAXL; q++) {
                ps[q] = walk && pos < xb ? pos : 0u;
                if (walk && pos < xb) {
                    const uint32_t Lb = img[pos];
                    bad |= Lb - 12u > 3u;
                    pos += Lb - 12u > 3u ? 12u : Lb;
                    n++;
                }
            }
            bad |= owner && pos != xb;
            uint32_t rid[MAXL];
            uint64_t rval[MAXL];
            const uint32_t remt = W - t0 < 0xffffffffull ? (uint32_t)(W - t0) : 0xffffffffu;
#pragma unroll
            for (int q = 0; q < MAXL; q++) {
                uint32_t e0, e1, e2, e3;
                load16(img, ps[q], e0, e1, e2, e3);
                const uint32_t Lr = rec_check32(e0, e1, remt - ps[q]);
                bad |= (uint32_t)q < n && Lr == 0;
                uint64_t id, val;
                rec_decode(e0, e1, e2, e3, Lr ? Lr : 12u, id, val);
                rid[q] = (uint32_t)id;
                rval[q] = val;
            }
            if (__any(bad)) {
                if (lane == 0) atomicOr(&st->fast_fail, 1u);
                return;
            }
            P1_STAMP(1);
            const uint32_t inc = wave_incl_scan(n);
            const uint32_t ntile = wave_last(inc);
            // the decoded records replace the image (u32 ids at 0, u64 values at VALOFF, in
            // record order) once every lane has read its records
            wave_lds_order();
            uint32_t* did = reinterpret_cast<uint32_t*>(img);
            uint64_t* dval = reinterpret_cast<uint64_t*>(img + VALOFF);
            const uint32_t i0 = inc - n;
#pragma unroll
            for (int q = 0; q < MAXL; q++) {
                if ((uint32_t)q < n) {
                    did[i0 + q] = rid[q];
                    dval[i0 + q] = rval[q];
                }
            }
            if (lane == 0) st_agent(&agg[t], lb_word(kFlagAgg, epoch, ntile));
            const int sl = (int)(k % NSLOT);
            if (lane == 0) *reinterpret_cast<uint32_t*>(img + CNTOFF) = ntile;
            P1_STAMP(2);
        }
        if (k >= LAG) {
            // 3. columns of tile t_{k-LAG} at its first record index
            const uint64_t ke = k - LAG;
            const uint64_t te = ke * V + v;
            const int se = (int)(ke % NSLOT);
            const uint32_t ne = *reinterpret_cast<const uint32_t*>(L.slot[se] + CNTOFF);
            const uint32_t* sid = reinterpret_cast<const uint32_t*>(L.slot[se]);
            const uint64_t* sval = reinterpret_cast<const uint64_t*>(L.slot[se] + VALOFF);
            P1_STAMP(4);
            uint64_t pw = (P1_FLAGS & 1u) ? lb_word(kFlagInc, epoch, te * 270) : ld_agent(&pre[te]);
            while (lb_flag(pw, epoch) == 0) {
                __builtin_amdgcn_s_sleep(1);
                if (ld_agent32(&st->fast_fail) || rt_now() - t_start > kSpinTicks) {
                    if (lane == 0 && !ld_agent32(&st->fast_fail)) {
                        atomicOr(&st->timeout, 1u);
                        atomicOr(&st->fast_fail, 1u);
                    }
                    return;
                }
                pw = ld_agent(&pre[te]);
            }
            const uint64_t base = pw & kValMask;
            uint32_t lim = ne;
            if (base + ne > cap) {
                lim = base < cap ? (uint32_t)(cap - base) : 0u;
                over = true;
            }
            P1_STAMP(3);
            wave_lds_order();
            if (!(P1_FLAGS & 2u)) {
                for (uint32_t i = lane; i < lim; i += 64) {
                    oid[base + i] = sid[i];  // widened to the u64 column
                    oval[base + i] = sval[i];
                }
            }
            P1_STAMP(4);
        }
    }
    if (over && lane == 0) atomicOr(&st->capacity, 1u);
#ifdef NXG_1P_PROBE
    if (lane == 0) {
        atomicAdd(&g_1p_cyc[0], (unsigned long long)cyc0);
        atomicAdd(&g_1p_cyc[1], (unsigned long long)cyc1);
        atomicAdd(&g_1p_cyc[2], (unsigned long long)cyc2);
        atomicAdd(&g_1p_cyc[3], (unsigned long long)cyc3);
        atomicAdd(&g_1p_cyc[4], (unsigned long long)cyc4);
    }
#endif
}

__global__ __launch_bounds__(TPB1) void nxg_f64_1p_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, uint64_t* __restrict__ oid,
    uint64_t* __restrict__ oval, uint64_t cap, uint64_t* agg, uint64_t* pre, uint32_t epoch,
    DevStatus* __restrict__ st, DevStatus* zst) {
    zero_status(zst);
    const uint64_t t_start = rt_now();
    __shared__ WaveLds lds[WAVES1];
    static_assert(TPB1 * SCAN_K * 8 <= sizeof(WaveLds) * WAVES1, "scanner staging");
    if (blockIdx.x == 0) {
        f64_scan(nt, agg, pre, epoch, st, reinterpret_cast<uint64_t*>(&lds[0]), t_start);
        return;
    }
    const uint32_t w = threadIdx.x >> 6;
    f64_work(wire, W, nt, oid, oval, cap, agg, pre, epoch, st,
             (uint64_t)(blockIdx.x - 1) * WAVES1 + w, (uint64_t)(gridDim.x - 1) * WAVES1, lds[w],
             t_start);
}

uint64_t nxg_dec_f64_1p_tiles(uint64_t W) { return (W + f64dec::STRIDE - 1) / f64dec::STRIDE; }

hipError_t nxg_launch_dec_f64_1p(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                                 uint64_t cap, uint64_t* tstat, uint32_t epoch, int wgs,
                                 DevStatus* st, hipStream_t s) {
    const uint64_t nt = nxg_dec_f64_1p_tiles(W);
    if (nt == 0) return hipSuccess;
    if (wgs < 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nxg_f64_1p_kernel, dim3(wgs), dim3(TPB1), 0, s, wire, W, nt, oid, oval, cap,
                       tstat, tstat + nt, epoch, st, nxg_take_zero_slot());
    return hipGetLastError();
}

// Every workgroup must be resident at once (workers and the scanner wait on each other): the
// occupancy answer, with one workgroup of margin per 8 CUs.
int nxg_dec_f64_1p_wgs(int ncu) {
    int a = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, nxg_f64_1p_kernel, TPB1, 0) !=
            hipSuccess ||
        a < 1)
        return 0;
    return ncu * a - ncu / 8;
}
