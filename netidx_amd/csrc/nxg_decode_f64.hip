// nxg_decode_f64.hip -- homogeneous-f64 decode for gfx950 (record format and merge points:
// nxg_f64_rec.h).
//
// Replaces the receive_batch_fn loop (netidx/src/channel.rs:504-521) for frames in which every
// message is From::Update(Id, F64).
//
// Two launches on one persistent grid of `wgs` workgroups x 4 waves; wave v owns a contiguous
// run of tiles in both. count: merge points + record counts per run (reads W bytes). emit: each
// run's first record index from the count pass's totals, then numbering and decode with
// coalesced column stores (reads W bytes again, writes 16 B per record). The kernel boundary is
// the only grid-wide synchronisation; there is no look-back chain and no spin-wait.
#include "nxg_f64_rec.h"

// ---- pass 1: count ----------------------------------------------------------------------------
// Wave v of the grid owns run v: a contiguous run of the frame's tiles. It counts the run's
// records (wcnt[v]); the workgroup stores the sum of its four runs (gcnt). It also keeps each
// lane's merge point (moff), so the emit pass does not search for them again. Pure streaming:
// no inter-workgroup communication inside the launch.
__global__ __launch_bounds__(TPB) void nxg_f64_count_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, uint32_t* __restrict__ wcnt,
    uint32_t* __restrict__ gcnt, uint8_t* __restrict__ moff, DevStatus* __restrict__ st,
    DevStatus* zst) {
    zero_status(zst);
    __shared__ __attribute__((aligned(16))) uint8_t bufs[WAVES][IMG + HALO];
    __shared__ uint32_t wsum[WAVES];

    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t R = gridDim.x * WAVES, r = blockIdx.x * WAVES + w;
    uint8_t* buf = bufs[w];
    uint32_t total = 0;
    bool anybad = false;
    for_run_tiles<false>(
        wire, W, run_begin(0, nt, R, r), run_begin(0, nt, R, r + 1), lane, nullptr,
        [&](const TileRegs& regs, uint64_t) __attribute__((always_inline)) {
            wave_lds_order();
            tile_store(buf, regs, lane);
            wave_lds_order();
        },
        [&](uint64_t tile) __attribute__((always_inline)) {
            bool bad;
            const uint32_t xa = chunk_merge(buf, tile, W, lane);
            total += chunk_walk<false>(buf, xa, lane, nullptr, bad);
            anybad |= bad;
            // read by the emit pass: offset in the chunk (< WIN), or 0xff for a chunk that starts
            // at or past the frame's end (its merge point is the END position W - t0)
            moff[tile * 64 + lane] = xa >= lane * CHUNK ? (uint8_t)(xa - lane * CHUNK) : 0xffu;
        });
    total = wave_sum<uint32_t>(total);
    if (__any(anybad) && lane == 0) atomicOr(&st->fast_fail, 1u);
    if (lane == 0) {
        wcnt[r] = total;
        wsum[w] = total;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t g = 0;
        for (int i = 0; i < WAVES; i++) g += wsum[i];
        gcnt[blockIdx.x] = g;
    }
}

// ---- pass 2: emit -----------------------------------------------------------------------------
// Same runs as the count pass. Each workgroup first sums the counts of all earlier workgroups
// (gcnt, at most MAX_WGS words: one round trip, no serial scan anywhere), so every run knows its
// first record index. The wave then walks its tiles again from the count pass's merge points to
// number the records; lane i decodes records i, i+64, ... of a tile, so both column stores are
// coalesced.
constexpr int SCAN_PER = MAX_WGS / TPB;  // per-workgroup counts each thread sums
static_assert(MAX_WGS % TPB == 0, "prefix geometry");
__global__ __launch_bounds__(TPB) void nxg_f64_emit_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, const uint32_t* __restrict__ wcnt,
    const uint32_t* __restrict__ gcnt, const uint8_t* __restrict__ moff,
    uint64_t* __restrict__ oid, uint64_t* __restrict__ oval, uint64_t cap,
    DevStatus* __restrict__ st) {
    if (ld_agent32(&st->fast_fail)) return;  // the count pass rejected the frame
    __shared__ uint64_t red[2][WAVES];
    __shared__ __attribute__((aligned(16))) uint8_t bufs[WAVES][IMG + HALO];
    __shared__ uint16_t rposs[WAVES][MAXREC];
    __shared__ uint16_t pslots[WAVES][64 * SLOTS];

    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t G = gridDim.x, R = G * WAVES, r = blockIdx.x * WAVES + w;
    uint8_t* buf = bufs[w];
    uint16_t* rpos = rposs[w];
    uint16_t* pslot = pslots[w];
    {
        // records before this workgroup (and in the whole frame): all loads issued up front
        uint32_t v[SCAN_PER];
#pragma unroll
        for (int k = 0; k < SCAN_PER; k++) {
            const uint32_t q = k * TPB + tid;
            v[k] = q < G ? gcnt[q] : 0u;
        }
        uint64_t before = 0, all = 0;
#pragma unroll
        for (int k = 0; k < SCAN_PER; k++) {
            before += (k * TPB + tid < blockIdx.x) ? v[k] : 0u;
            all += v[k];
        }
        before = wave_sum<uint64_t>(before);
        all = wave_sum<uint64_t>(all);
        if (lane == 0) {
            red[0][w] = before;
            red[1][w] = all;
        }
        __syncthreads();
    }
    uint64_t rbase = 0, total = 0;
#pragma unroll
    for (int i = 0; i < WAVES; i++) {
        rbase += red[0][i];
        total += red[1][i];
    }
    for (uint32_t i = 0; i < w; i++) rbase += wcnt[blockIdx.x * WAVES + i];
    if (blockIdx.x == 0 && tid == 0) {
        st->n_rows = total;
        st->path = 1;
    }
    uint64_t base = rbase;
    bool anybad = false, over = false;
    uint32_t xa = 0;
    for_run_tiles<true>(
        wire, W, run_begin(0, nt, R, r), run_begin(0, nt, R, r + 1), lane, moff,
        [&](const TileRegs& regs, uint64_t tile) __attribute__((always_inline)) {
            wave_lds_order();
            tile_store(buf, regs, lane);
            wave_lds_order();
            xa = lane * CHUNK + regs.m;  // merge point found by the count pass
            if (regs.m == 0xffu) xa = (uint32_t)(W - (uint64_t)tile * STRIDE);
        },
        [&](uint64_t tile) __attribute__((always_inline)) {
            const uint64_t t0 = tile * STRIDE;
            bool bad;
            const uint32_t n = chunk_walk<true>(buf, xa, lane, pslot, bad);
            const uint32_t inc = wave_incl_scan(n);
            const uint32_t off = inc - n;
            const uint32_t ntile = wave_last(inc);
            for (uint32_t q = 0; q < n; q++) rpos[off + q] = pslot[lane * SLOTS + q];
            wave_lds_order();
            uint32_t lim = ntile;
            if (base + ntile > cap) {
                lim = base < cap ? (uint32_t)(cap - base) : 0u;
                over = true;
            }
            for (uint32_t i = lane; i < lim; i += 64) {
                const uint32_t p = rpos[i];
                uint32_t e0, e1, e2, e3;
                load16(buf, p, e0, e1, e2, e3);
                const uint32_t L = rec_check(e0, e1, W - (t0 + p));
                bad |= L == 0;
                uint64_t id, val;
                rec_decode(e0, e1, e2, e3, L ? L : 12u, id, val);
                oid[base + i] = id;
                oval[base + i] = val;
            }
            anybad |= bad;
            base += ntile;
        });
    anybad |= base - rbase != wcnt[r];  // the count pass saw the same records
    if (__any(anybad) && lane == 0) atomicOr(&st->fast_fail, 1u);
    if (over && lane == 0) atomicOr(&st->capacity, 1u);
}

uint64_t nxg_dec_f64_tiles(uint64_t W) { return (W + STRIDE - 1) / STRIDE; }

hipError_t nxg_launch_dec_f64(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                              uint64_t cap, uint64_t* scratch, uint8_t* moff, int wgs,
                              DevStatus* st, hipStream_t s) {
    const uint64_t nt = nxg_dec_f64_tiles(W);
    if (nt == 0) return hipSuccess;
    if (wgs <= 0 || wgs > MAX_WGS) return hipErrorInvalidValue;
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(scratch);
    uint32_t* gcnt = reinterpret_cast<uint32_t*>(scratch + MAX_WGS * WAVES / 2);
    hipLaunchKernelGGL(nxg_f64_count_kernel, dim3(wgs), dim3(TPB), 0, s, wire, W, nt, wcnt, gcnt,
                       moff, st, nxg_take_zero_slot());
    hipLaunchKernelGGL(nxg_f64_emit_kernel, dim3(wgs), dim3(TPB), 0, s, wire, W, nt, wcnt, gcnt,
                       moff, oid, oval, cap, st);
    return hipGetLastError();
}

int nxg_dec_f64_wgs(int ncu) {
    int a = 0, b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, nxg_f64_count_kernel, TPB, 0) !=
            hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, nxg_f64_emit_kernel, TPB, 0) != hipSuccess)
        return ncu;
    const int occ = std::max(1, std::min(a, b));
    return std::min(MAX_WGS, ncu * occ);
}
