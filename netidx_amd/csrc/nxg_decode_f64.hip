// nxg_decode_f64.hip -- homogeneous-f64 decode for gfx950 (record format and merge points:
// nxg_f64_rec.h).
//
// Replaces the receive_batch_fn loop (netidx/src/channel.rs:504-521) for frames in which every
// message is From::Update(Id, F64).
#include "nxg_f64_rec.h"

// ---- pass 1: count ----------------------------------------------------------------------------
// Wave v of the grid owns run v: a contiguous run of the segment's tiles. It counts the run's
// records (wcnt); the workgroup publishes the sum of its four runs (gcnt), and the workgroup that
// arrives last (agent-scope ticket) turns the per-workgroup counts into first-record indices
// (gpre), continuing the running total of the call's earlier segments.
constexpr int SCAN_PER = MAX_WGS / TPB;  // per-workgroup counts each scanning thread owns
static_assert(MAX_WGS % TPB == 0, "scan geometry");
__global__ __launch_bounds__(TPB) void nxg_f64_count_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t first, uint64_t nt, int last_seg,
    uint32_t* __restrict__ wcnt, uint32_t* gcnt, uint64_t* __restrict__ gpre, uint64_t* running,
    uint32_t* ticket, DevStatus* __restrict__ st, DevStatus* zst) {
    zero_status(zst);
    __shared__ __attribute__((aligned(16))) uint8_t bufs[WAVES][TILE + HALO];
    __shared__ uint32_t wsum[WAVES];
    __shared__ uint32_t sh_last;
    __shared__ uint64_t scan_tmp[WAVES];

    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t R = gridDim.x * WAVES, r = blockIdx.x * WAVES + w;
    uint8_t* buf = bufs[w];
    uint32_t total = 0;
    bool anybad = false;
    for_run_tiles(
        wire, W, run_begin(first, nt, R, r), run_begin(first, nt, R, r + 1), lane,
        [&](const TileRegs& regs, uint64_t) __attribute__((always_inline)) {
            wave_lds_order();
            tile_store(buf, regs, lane);
            wave_lds_order();
        },
        [&](uint64_t tile) __attribute__((always_inline)) {
            bool bad;
            total += chunk_walk<false>(buf, tile, W, lane, nullptr, bad);
            anybad |= bad;
        });
    total = wave_sum<uint32_t>(total);
    if (__any(anybad) && lane == 0) atomicOr(&st->fast_fail, 1u);
    if (lane == 0) {
        wcnt[r] = total;  // read by the emit pass (next launch)
        wsum[w] = total;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t g = 0;
        for (int i = 0; i < WAVES; i++) g += wsum[i];
        __hip_atomic_store(&gcnt[blockIdx.x], g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        drain_stores();
        sh_last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                  gridDim.x - 1;
    }
    __syncthreads();
    if (!sh_last) return;
    // last workgroup: exclusive scan of the per-workgroup counts (all loads issued up front)
    const uint32_t G = gridDim.x;
    const uint64_t base = ld_agent(running);
    uint32_t v[SCAN_PER];
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        const uint32_t q = tid * SCAN_PER + k;
        v[k] = q < G ? ld_agent32(&gcnt[q]) : 0u;
    }
    uint64_t local = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) local += v[k];
    uint64_t sum;
    uint64_t pre = block_excl_scan<uint64_t, TPB>(local, scan_tmp, &sum);
#pragma unroll
    for (int k = 0; k < SCAN_PER; k++) {
        const uint32_t q = tid * SCAN_PER + k;
        if (q < G) gpre[q] = base + pre;
        pre += v[k];
    }
    if (tid == 0) {
        *ticket = 0;  // ready for the next launch (every other workgroup has arrived)
        st_agent(running, last_seg ? 0ull : base + sum);  // the next call starts from 0 again
        if (last_seg) {
            st->n_rows = base + sum;
            st->path = 1;
        }
    }
}

// ---- pass 2: emit -----------------------------------------------------------------------------
// Same runs as the count pass. The wave numbers its tiles' records from the run's first index,
// walking again to find each record start; lane i then decodes records i, i+64, ... of the tile,
// so both column stores are coalesced.
__global__ __launch_bounds__(TPB) void nxg_f64_emit_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t first, uint64_t nt,
    const uint32_t* __restrict__ wcnt, const uint64_t* __restrict__ gpre,
    uint64_t* __restrict__ oid, uint64_t* __restrict__ oval, uint64_t cap,
    DevStatus* __restrict__ st) {
    if (ld_agent32(&st->fast_fail)) return;  // the count pass rejected the frame
    __shared__ __attribute__((aligned(16))) uint8_t bufs[WAVES][TILE + HALO];
    __shared__ uint16_t rposs[WAVES][MAXREC];
    __shared__ uint16_t pslots[WAVES][64 * SLOTS];

    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t R = gridDim.x * WAVES, r = blockIdx.x * WAVES + w;
    uint8_t* buf = bufs[w];
    uint16_t* rpos = rposs[w];
    uint16_t* pslot = pslots[w];
    uint64_t rbase = gpre[blockIdx.x];
    for (uint32_t i = 0; i < w; i++) rbase += wcnt[blockIdx.x * WAVES + i];
    uint64_t base = rbase;
    bool anybad = false, over = false;
    for_run_tiles(
        wire, W, run_begin(first, nt, R, r), run_begin(first, nt, R, r + 1), lane,
        [&](const TileRegs& regs, uint64_t) __attribute__((always_inline)) {
            wave_lds_order();
            tile_store(buf, regs, lane);
            wave_lds_order();
        },
                  [&](uint64_t tile) __attribute__((always_inline)) {
                      const uint64_t t0 = tile * TILE;
                      bool bad;
                      const uint32_t n = chunk_walk<true>(buf, tile, W, lane, pslot, bad);
                      const uint32_t inc = wave_incl_scan(n);
                      const uint32_t off = inc - n;
                      const uint32_t ntile = __shfl(inc, 63, 64);
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

hipError_t nxg_launch_dec_f64(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                              uint64_t cap, uint64_t* scratch, uint32_t* ticket, int wgs,
                              DevStatus* st, hipStream_t s) {
    const uint64_t nt = (W + TILE - 1) / TILE;
    if (nt == 0) return hipSuccess;
    if (wgs <= 0 || wgs > MAX_WGS) return hipErrorInvalidValue;
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(scratch);
    uint32_t* gcnt = reinterpret_cast<uint32_t*>(scratch + MAX_WGS * WAVES / 2);
    uint64_t* gpre = scratch + MAX_WGS * WAVES / 2 + MAX_WGS / 2;
    uint64_t* running = gpre + MAX_WGS;
    // Segment by segment (each at most SEG_TILES tiles, all of equal size): count, then emit,
    // while the segment's bytes are still in the Infinity Cache.
    const uint64_t nseg = (nt + SEG_TILES - 1) / SEG_TILES;
    for (uint64_t k = 0; k < nseg; k++) {
        const uint64_t b = nt * k / nseg, e = nt * (k + 1) / nseg;
        hipLaunchKernelGGL(nxg_f64_count_kernel, dim3(wgs), dim3(TPB), 0, s, wire, W, b, e - b,
                           (int)(k + 1 == nseg), wcnt, gcnt, gpre, running, ticket, st,
                           k == 0 ? nxg_zero_slot : nullptr);
        hipLaunchKernelGGL(nxg_f64_emit_kernel, dim3(wgs), dim3(TPB), 0, s, wire, W, b, e - b,
                           wcnt, gpre, oid, oval, cap, st);
    }
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
