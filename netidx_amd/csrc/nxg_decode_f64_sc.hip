// nxg_decode_f64_sc.hip -- single-pass homogeneous-f64 decode with a scanner workgroup.
//
// Persistent grid: block 0 is the scanner, every other wave a worker. Worker wave v owns tiles
// v, v+V, v+2V, ... (V worker waves), so round k = tiles [kV, (k+1)V) is spread over all
// waves. A worker stages a tile in its LDS image, counts and numbers its records, publishes the
// count (agg[t]), and issues the loads of its next tile; it then waits for the tile's first
// record index (pre[t]), decodes the records from LDS with coalesced column stores, and stages
// the next tile. The scanner turns agg[] into pre[] in tile order, 256*SCAN_K tiles per step,
// so no worker ever walks a look-back chain; the chain's throughput is the scanner's.
//
// agg[] and pre[] words are epoch-tagged 8-byte granules (nxg_internal.h) written with one
// agent-scope store and polled with agent-scope loads (MI355X_MICROARCH.md "Valid forms", R2).
// Every spin is bounded (watchdog) and gives up when DevStatus.fast_fail is raised, so a
// rejected frame or a stuck grid ends the kernel; the host then runs the general decoder.
#include "nxg_f64_rec.h"

#ifdef NXG_PROBE_TRACE  // scripts/probe_f64.hip only: per-tile timeline (s_memrealtime, 10 ns)
__device__ uint64_t* g_probe_trace;  // [nt][4]: published, prefix seen, decoded, scanner wrote
#define PROBE_MARK(tile, k, v) \
    do { g_probe_trace[(uint64_t)(tile) * 4 + (k)] = (v); } while (0)
#else
#define PROBE_MARK(tile, k, v) do {} while (0)
#endif

namespace {
constexpr int SCAN_K = 8;  // tiles per scanner thread per step (up to 2048 per step)

// Wave-uniform spin on an epoch-tagged word until it carries `flag`; false on abort/timeout.
NXG_DEV bool wait_word(const uint64_t* p, uint32_t epoch, const uint32_t* abort, uint64_t t_start,
                       uint64_t& v) {
    v = ld_agent(p);
    while (lb_flag(v, epoch) == 0) {
        __builtin_amdgcn_s_sleep(2);
        if (ld_agent32(abort) || rt_now() - t_start > kSpinTicks) return false;
        v = ld_agent(p);
    }
    return true;
}
}  // namespace

// ---- scanner: publishes pre[] for the longest published prefix of agg[], in steps of up to
// TPB*SCAN_K tiles (never waiting for a tile beyond the first unpublished one, so it cannot wait
// on a worker that waits on it). Loads and stores are coalesced (tile c + k*TPB + tid); `stg`
// (TPB*SCAN_K words of LDS) holds the transpose to per-thread runs. One full workgroup.
NXG_DEV void sc_scan(uint64_t nt, const uint64_t* agg, uint64_t* pre, uint32_t epoch,
                     DevStatus* __restrict__ st, uint64_t* stg, uint64_t t_start) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
            __shared__ uint64_t scan_tmp[WAVES];
            __shared__ uint64_t wmin[WAVES];
            uint64_t running = 0;
            uint64_t c = 0;
            while (c < nt) {
                uint64_t v[SCAN_K];
                uint64_t fu = nt;  // first unpublished tile of the step (nt if none)
    #pragma unroll
                for (int k = 0; k < SCAN_K; k++) {
                    const uint64_t i = c + (uint64_t)k * TPB + tid;
                    v[k] = i < nt ? ld_agent(&agg[i]) : lb_word(kFlagAgg, epoch, 0);
                }
    #pragma unroll
                for (int k = SCAN_K - 1; k >= 0; k--) {
                    const uint64_t i = c + (uint64_t)k * TPB + tid;
                    if (i < nt && lb_flag(v[k], epoch) == 0) fu = i < fu ? i : fu;
                }
    #pragma unroll
                for (int d = 32; d >= 1; d >>= 1) {
                    const uint64_t o = __shfl_xor(fu, d, 64);
                    fu = o < fu ? o : fu;
                }
                if (lane == 0) wmin[w] = fu;
    #pragma unroll
                for (int k = 0; k < SCAN_K; k++) stg[k * TPB + tid] = v[k] & kValMask;
                __syncthreads();
                uint64_t F = wmin[0];
    #pragma unroll
                for (int i = 1; i < WAVES; i++) F = wmin[i] < F ? wmin[i] : F;
                const uint64_t cend = c + (uint64_t)TPB * SCAN_K;
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
                    __builtin_amdgcn_s_sleep(2);
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
                uint64_t p = running + block_excl_scan<uint64_t, TPB>(local, scan_tmp, &total);
    #pragma unroll
                for (int k = 0; k < SCAN_K; k++) {
                    stg[tid * SCAN_K + k] = p;
                    p += x[k];
                }
                __syncthreads();
    #pragma unroll
                for (int k = 0; k < SCAN_K; k++) {
                    const uint64_t i = c + (uint64_t)k * TPB + tid;
                    if (i < F) {
                        st_agent(&pre[i], lb_word(kFlagInc, epoch, stg[k * TPB + tid]));
                        PROBE_MARK(i, 3, rt_now());
                    }
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

// ---- worker wave v of V: tiles v, v+V, v+2V, ...; buf/rpos/pslot are the wave's LDS ----
NXG_DEV void sc_work(const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt,
                     uint64_t* __restrict__ oid, uint64_t* __restrict__ oval, uint64_t cap,
                     uint64_t* agg, const uint64_t* pre, uint32_t epoch, DevStatus* __restrict__ st,
                     uint64_t v, uint64_t V, uint8_t* buf, uint16_t* rpos, uint16_t* pslot,
                     uint64_t t_start) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t t = v;
    if (t >= nt) return;
    const uint64_t nfull = W >= IMG + HALO ? (W - IMG - HALO) / STRIDE + 1 : 0;

    // stage + number tile t (LDS image, rpos); returns the tile's record count, sets bad
    auto number = [&](const TileRegs& regs, uint64_t tile, bool& bad) __attribute__((always_inline)) {
        wave_lds_order();
        tile_store(buf, regs, lane);
        wave_lds_order();
        const uint32_t n = chunk_walk<true>(buf, chunk_merge(buf, tile, W, lane), lane, pslot, bad);
        const uint32_t inc = wave_incl_scan(n);
        const uint32_t off = inc - n;
        for (uint32_t q = 0; q < n; q++) rpos[off + q] = pslot[lane * SLOTS + q];
        wave_lds_order();
        return __shfl(inc, 63, 64);
    };

    TileRegs R;
    if (t < nfull) tile_load_full<false>(R, wire, t * STRIDE, lane, nullptr);
    else tile_load(R, wire, t * STRIDE, W, lane, nullptr);
    bool bad;
    uint32_t ntile = number(R, t, bad);
    if (__any(bad)) {
        if (lane == 0) atomicOr(&st->fast_fail, 1u);
        return;
    }
    if (lane == 0) st_agent(&agg[t], lb_word(kFlagAgg, epoch, ntile));
    if (lane == 0) PROBE_MARK(t, 0, rt_now());
    bool over = false;
    for (;;) {
        const uint64_t tn = t + V;
        if (tn < nfull) tile_load_full<false>(R, wire, tn * STRIDE, lane, nullptr);
        else if (tn < nt) tile_load(R, wire, tn * STRIDE, W, lane, nullptr);
        uint64_t pw;
        if (!wait_word(&pre[t], epoch, &st->fast_fail, t_start, pw)) {
            if (lane == 0 && !ld_agent32(&st->fast_fail)) {
                atomicOr(&st->timeout, 1u);
                atomicOr(&st->fast_fail, 1u);
            }
            return;
        }
        const uint64_t base = pw & kValMask;
        if (lane == 0) PROBE_MARK(t, 1, rt_now());
        const uint64_t t0 = t * STRIDE;
        uint32_t lim = ntile;
        if (base + ntile > cap) {
            lim = base < cap ? (uint32_t)(cap - base) : 0u;
            over = true;
        }
        bool badrec = false;
        for (uint32_t i = lane; i < lim; i += 64) {
            const uint32_t p = rpos[i];
            uint32_t e0, e1, e2, e3;
            load16(buf, p, e0, e1, e2, e3);
            const uint32_t L = rec_check(e0, e1, W - (t0 + p));
            badrec |= L == 0;
            uint64_t id, val;
            rec_decode(e0, e1, e2, e3, L ? L : 12u, id, val);
            oid[base + i] = id;
            oval[base + i] = val;
        }
        if (__any(badrec)) {
            if (lane == 0) atomicOr(&st->fast_fail, 1u);
            return;
        }
        if (lane == 0) PROBE_MARK(t, 2, rt_now());
        if (tn >= nt) break;
        t = tn;
        ntile = number(R, t, bad);
        if (__any(bad)) {
            if (lane == 0) atomicOr(&st->fast_fail, 1u);
            return;
        }
        if (lane == 0) st_agent(&agg[t], lb_word(kFlagAgg, epoch, ntile));
        if (lane == 0) PROBE_MARK(t, 0, rt_now());
    }
    if (over && lane == 0) atomicOr(&st->capacity, 1u);
}

// Fused form: block 0 scans, every other wave works.
__global__ __launch_bounds__(TPB) void nxg_f64_sc_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, uint64_t* __restrict__ oid,
    uint64_t* __restrict__ oval, uint64_t cap, uint64_t* agg, uint64_t* pre, uint32_t epoch,
    DevStatus* __restrict__ st, DevStatus* zst) {
    zero_status(zst);
    const uint64_t t_start = rt_now();
    __shared__ __attribute__((aligned(16))) uint8_t bufs[WAVES][TILE + HALO];
    __shared__ uint16_t rposs[WAVES][MAXREC];
    __shared__ uint16_t pslots[WAVES][64 * SLOTS];
    static_assert(TPB * SCAN_K * 8 <= WAVES * (TILE + HALO), "scanner staging");
    if (blockIdx.x == 0) {
        sc_scan(nt, agg, pre, epoch, st, reinterpret_cast<uint64_t*>(&bufs[0][0]), t_start);
        return;
    }
    const uint32_t w = threadIdx.x >> 6;
    sc_work(wire, W, nt, oid, oval, cap, agg, pre, epoch, st,
            (uint64_t)(blockIdx.x - 1) * WAVES + w, (uint64_t)(gridDim.x - 1) * WAVES, bufs[w],
            rposs[w], pslots[w], t_start);
}

// Split form: the scanner is its own one-workgroup kernel (run on a stream whose CU mask
// leaves it a CU of its own), the workers another.
__global__ __launch_bounds__(TPB) void nxg_f64_scan_kernel(uint64_t nt, const uint64_t* agg,
                                                           uint64_t* pre, uint32_t epoch,
                                                           DevStatus* __restrict__ st) {
    __shared__ uint64_t stg[TPB * SCAN_K];
    sc_scan(nt, agg, pre, epoch, st, stg, rt_now());
}
__global__ __launch_bounds__(TPB) void nxg_f64_work_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, uint64_t* __restrict__ oid,
    uint64_t* __restrict__ oval, uint64_t cap, uint64_t* agg, const uint64_t* pre,
    uint32_t epoch, DevStatus* __restrict__ st, DevStatus* zst) {
    zero_status(zst);
    __shared__ __attribute__((aligned(16))) uint8_t bufs[WAVES][TILE + HALO];
    __shared__ uint16_t rposs[WAVES][MAXREC];
    __shared__ uint16_t pslots[WAVES][64 * SLOTS];
    const uint32_t w = threadIdx.x >> 6;
    sc_work(wire, W, nt, oid, oval, cap, agg, pre, epoch, st, (uint64_t)blockIdx.x * WAVES + w,
            (uint64_t)gridDim.x * WAVES, bufs[w], rposs[w], pslots[w], rt_now());
}

hipError_t nxg_launch_dec_f64_sc(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                                 uint64_t cap, uint64_t* tstat, uint32_t epoch, int wgs,
                                 DevStatus* st, hipStream_t s) {
    const uint64_t nt = (W + STRIDE - 1) / STRIDE;
    if (nt == 0) return hipSuccess;
    if (wgs < 2) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nxg_f64_sc_kernel, dim3(wgs), dim3(TPB), 0, s, wire, W, nt, oid, oval, cap,
                       tstat, tstat + nt, epoch, st, nxg_zero_slot);
    return hipGetLastError();
}

hipError_t nxg_launch_dec_f64_sc2(const uint8_t* wire, uint64_t W, uint64_t* oid,
                                  uint64_t* oval, uint64_t cap, uint64_t* tstat, uint32_t epoch,
                                  int wgs, DevStatus* st, hipStream_t s_scan, hipStream_t s_work) {
    const uint64_t nt = (W + STRIDE - 1) / STRIDE;
    if (nt == 0) return hipSuccess;
    hipLaunchKernelGGL(nxg_f64_scan_kernel, dim3(1), dim3(TPB), 0, s_scan, nt, tstat, tstat + nt,
                       epoch, st);
    hipLaunchKernelGGL(nxg_f64_work_kernel, dim3(wgs), dim3(TPB), 0, s_work, wire, W, nt, oid,
                       oval, cap, tstat, tstat + nt, epoch, st, nxg_zero_slot);
    return hipGetLastError();
}

int nxg_dec_f64_sc2_wgs(int ncu) {
    int a = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, nxg_f64_work_kernel, TPB, 0) !=
            hipSuccess || a < 1)
        return 0;
    return ncu * a - ncu / 8;
}

int nxg_dec_f64_sc_wgs(int ncu) {
    int a = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, nxg_f64_sc_kernel, TPB, 0) != hipSuccess ||
        a < 1)
        return 0;
    // every workgroup must be resident at once (workers and the scanner wait on each other);
    // keep one workgroup of margin per 8 CUs under the occupancy answer
    return ncu * a - ncu / 8;
}
