// nxg_partition.hip -- the type-partitioned view of decoded mixed columns (the
// optional output; BASELINE configs[2]'s "LDS histogram + scan"), for gfx950.
//
// A subscriber that handles values by type does, per value, the 28-way `match` of Value::decode
// (netidx-value/src/lib.rs:470-506) and of whatever consumes the value. This view groups the rows
// by their wire tag once, on the device: dense per-tag runs of the fixed / aux columns (rows of a
// tag in record order), the dense index -> row map, and the record -> (tag, rank) map (the tag is
// the row's own tag column, rank its index among the rows of that tag). Integer work only:
// HBM-bound, no MFMA.
//
//   count  per 4096-row tile: one LDS histogram per wave, filled a round of 64 rows at a time --
//          the round's distinct tags found by ballots (readfirstlane of the first unclaimed lane,
//          then a ballot of the lanes holding that tag), so a round costs one LDS update per
//          distinct tag, not per row -- summed per tile into counts[bin][tile] (bin-major)
//   scan   one workgroup per bin: the exclusive scan of its tiles' counts (tile bases) and the
//          bin's total; then one workgroup scans the 256 totals into the per-tag offsets
//   place  per tile: the tags again, the waves' histograms again, a prefix over the four waves
//          per bin, then each round ranks its rows by the same ballots (mbcnt of the tag's lane
//          mask) and writes rank[row], row_of[dest], fixed and aux at dest =
//          off[tag] + tile base + wave prefix + rank in the wave.
#include "nxg_device.h"

namespace part {
constexpr int TPB = 256;
constexpr int WAVES = TPB / 64;
#ifndef NXG_PART_TROWS
#define NXG_PART_TROWS 4096  // (A/B at 10^7: 4096 0.149-0.150, 2048 0.156-0.158, 1024 0.169-0.171 ms)
#endif
constexpr uint32_t TROWS = NXG_PART_TROWS;  // rows per tile
constexpr uint32_t WROWS = TROWS / WAVES;   // rows per wave (4096: 16 rounds of 64)
constexpr uint32_t ROUNDS = WROWS / 64;
constexpr uint32_t NB = 256;                // tag bins (the tag column is u8)
constexpr uint32_t NOTAG = 0x100;           // a lane past the last row
constexpr int KU = 8;                       // distinct tags per round handled unrolled

// The round's distinct tags one after another (readfirstlane of the first unclaimed lane, a ballot
// of the lanes holding that tag): f(k, leader lane, tag, lane mask) for each. The first KU are
// unrolled (each LDS operation f issues gets its own registers, so nothing waits between them);
// more than KU distinct tags in one round of 64 rows take the rolled loop.
template <typename F>
NXG_DEV void each_tag(uint32_t t, F&& f) {
    uint64_t rem = __ballot(t != NOTAG);
#pragma unroll
    for (int k = 0; k < KU; k++) {
        if (rem) {
            const uint32_t l = (uint32_t)__builtin_ctzll(rem);
            const uint32_t tv = (uint32_t)__builtin_amdgcn_readlane((int)t, (int)l);
            const uint64_t m = __ballot(t == tv);
            f(k, l, tv, m);
            rem &= ~m;
        }
    }
#pragma unroll 1
    while (rem) {
        const uint32_t l = (uint32_t)__builtin_ctzll(rem);
        const uint32_t tv = (uint32_t)__builtin_amdgcn_readlane((int)t, (int)l);
        const uint64_t m = __ballot(t == tv);
        f(KU, l, tv, m);
        rem &= ~m;
    }
}

// the wave's rows' tags (16 rounds of 64; NOTAG past n), all loads in flight together
NXG_DEV void load_tags(const uint8_t* __restrict__ tag, uint64_t r0, uint64_t n, uint32_t lane,
                       uint32_t (&t)[ROUNDS]) {
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; r++) {
        const uint64_t row = r0 + r * 64 + lane;
        t[r] = row < n ? (uint32_t)tag[row] : NOTAG;
    }
}

// the wave's per-bin counts into its LDS histogram h (zeroed by the caller): one LDS add per
// distinct tag of a round, with no return (nothing waits on it)
NXG_DEV void wave_hist(const uint32_t (&t)[ROUNDS], uint32_t* h, uint32_t lane) {
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; r++)
        each_tag(t[r], [&](int, uint32_t l, uint32_t tv, uint64_t m) {
            if (lane == l) atomicAdd(&h[tv], (uint32_t)__popcll(m));
        });
}
}  // namespace part

using namespace part;

__global__ __launch_bounds__(TPB) void nxg_part_count_kernel(const uint8_t* __restrict__ tag,
                                                             uint64_t n, uint32_t ntiles,
                                                             uint32_t* __restrict__ counts) {
    __shared__ uint32_t hist[WAVES][NB];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t tile = blockIdx.x;
#pragma unroll
    for (uint32_t b = tid; b < WAVES * NB; b += TPB) (&hist[0][0])[b] = 0;
    __syncthreads();
    uint32_t t[ROUNDS];
    load_tags(tag, (uint64_t)tile * TROWS + (uint64_t)w * WROWS, n, lane, t);
    wave_hist(t, hist[w], lane);
    __syncthreads();
    // tile totals, bin-major (the scan reads a bin's tiles contiguously)
    const uint32_t b = tid;
    counts[(uint64_t)b * ntiles + tile] = hist[0][b] + hist[1][b] + hist[2][b] + hist[3][b];
}

// one workgroup per bin: exclusive scan over the tiles -> bases (in place), the bin's total
__global__ __launch_bounds__(TPB) void nxg_part_scan_kernel(uint32_t* __restrict__ counts,
                                                            uint32_t ntiles,
                                                            uint64_t* __restrict__ totals) {
    __shared__ uint32_t tmp[WAVES];
    const uint32_t b = blockIdx.x;
    uint32_t* c = counts + (uint64_t)b * ntiles;
    uint32_t run = 0;
#pragma unroll 1
    for (uint32_t i0 = 0; i0 < ntiles; i0 += TPB) {
        const uint32_t i = i0 + threadIdx.x;
        const uint32_t v = i < ntiles ? c[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan<uint32_t, TPB>(v, tmp, &tot);
        if (i < ntiles) c[i] = run + ex;
        run += tot;
    }
    if (threadIdx.x == 0) totals[b] = run;
}

// one workgroup: the per-tag offsets off[0..NB] (exclusive scan of the totals; off[NB] = rows)
__global__ __launch_bounds__(TPB) void nxg_part_offsets_kernel(const uint64_t* __restrict__ totals,
                                                               uint64_t* __restrict__ off) {
    __shared__ uint64_t tmp[WAVES];
    const uint32_t b = threadIdx.x;
    uint64_t tot;
    const uint64_t ex = block_excl_scan<uint64_t, TPB>(totals[b], tmp, &tot);
    off[b] = ex;
    if (b == 0) off[NB] = tot;
}

__global__ __launch_bounds__(TPB) void nxg_part_place_kernel(
    const uint8_t* __restrict__ tag, const uint64_t* __restrict__ fixed,
    const uint32_t* __restrict__ aux, uint64_t n, uint32_t ntiles,
    const uint32_t* __restrict__ bases, const uint64_t* __restrict__ off,
    uint32_t* __restrict__ rank, uint32_t* __restrict__ row_of, uint64_t* __restrict__ dfixed,
    uint32_t* __restrict__ daux) {
    __shared__ uint32_t hist[WAVES][NB];  // then: each wave's next slot per bin
    __shared__ uint32_t offl[NB];         // the per-tag offsets (rows < 2^32)
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t tile = blockIdx.x;
#pragma unroll
    for (uint32_t b = tid; b < WAVES * NB; b += TPB) (&hist[0][0])[b] = 0;
    offl[tid] = (uint32_t)off[tid];
    __syncthreads();
    const uint64_t r0 = (uint64_t)tile * TROWS + (uint64_t)w * WROWS;
    uint32_t t[ROUNDS];
    load_tags(tag, r0, n, lane, t);
    // the rows' values, every round's loads in flight together (a round that waited for its own
    // loads paid a memory round trip per 64 rows: 113 us at 10^7 rows)
    uint64_t fv[ROUNDS];
    uint32_t av[ROUNDS];
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; r++) {
        const uint64_t row = r0 + r * 64 + lane;
        fv[r] = row < n ? fixed[row] : 0ull;
        av[r] = row < n ? aux[row] : 0u;
    }
    wave_hist(t, hist[w], lane);
    __syncthreads();
    {  // per bin: the tile's base within the tag, then the waves' starts (rank within the tag)
        const uint32_t b = tid;
        uint32_t s = bases[(uint64_t)b * ntiles + tile];
#pragma unroll
        for (uint32_t k = 0; k < WAVES; k++) {
            const uint32_t c = hist[k][b];
            hist[k][b] = s;
            s += c;
        }
    }
    __syncthreads();
    uint32_t* nx = hist[w];
#pragma unroll
    for (uint32_t r = 0; r < ROUNDS; r++) {
        const uint64_t row = r0 + r * 64 + lane;
        const bool in = t[r] != NOTAG;
        // per distinct tag of the round: its leader lane takes the tag's slots with one LDS
        // fetch-and-add into a register of its own (the adds of a round issue back to back; LDS
        // applies them in order), each lane notes its leader and its tag's lane mask; then one
        // ds_bpermute hands every lane its leader's base
        uint32_t bk[KU + 1];
#pragma unroll
        for (int k = 0; k <= KU; k++) bk[k] = 0;
        uint32_t ldr = 0;
        uint64_t mine = 0;
        each_tag(t[r], [&](int k, uint32_t l, uint32_t tv, uint64_t m) {
            if (lane == l) {
                const uint32_t v = atomicAdd(&nx[tv], (uint32_t)__popcll(m));
                if (k < KU) bk[k] = v;
                else bk[KU] = v;  // (the rolled loop: its adds wait on each other)
            }
            if (t[r] == tv) {
                ldr = l;
                mine = m;
            }
        });
        uint32_t b = 0;
#pragma unroll
        for (int k = 0; k <= KU; k++) b |= bk[k];  // (each lane leads at most one tag)
        const uint32_t base = (uint32_t)__shfl((int)b, (int)ldr, 64);
        const uint32_t rk = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
        if (in) {
            const uint64_t dest = (uint64_t)offl[t[r]] + rk;
            rank[row] = rk;
            row_of[dest] = (uint32_t)row;
            dfixed[dest] = fv[r];
            daux[dest] = av[r];
        }
    }
}

uint64_t nxg_part_tiles(uint64_t n) { return (n + TROWS - 1) / TROWS; }
// scratch: counts / bases (u32 per bin and tile), totals and offsets (u64)
uint64_t nxg_part_scratch_bytes(uint64_t n) {
    return 4ull * NB * nxg_part_tiles(n) + 8ull * (2 * NB + 1) + 64;
}

// off_out: NB + 1 device u64 (the per-tag offsets, off[NB] = n), in the scratch's tail
hipError_t nxg_launch_partition(const uint8_t* tag, const uint64_t* fixed, const uint32_t* aux,
                                uint64_t n, uint8_t* scratch, uint32_t* rank, uint32_t* row_of,
                                uint64_t* dfixed, uint32_t* daux, uint64_t** off_out,
                                hipStream_t s) {
    const uint64_t nt = nxg_part_tiles(n);
    if (nt > 0xffffffffull) return hipErrorInvalidValue;
    uint32_t* counts = reinterpret_cast<uint32_t*>(scratch);
    uint64_t* totals = reinterpret_cast<uint64_t*>(scratch + ((4ull * NB * nt + 15) & ~15ull));
    uint64_t* off = totals + NB;
    *off_out = off;
    if (nt == 0) return hipMemsetAsync(off, 0, 8 * (NB + 1), s);
    hipLaunchKernelGGL(nxg_part_count_kernel, dim3((uint32_t)nt), dim3(TPB), 0, s, tag, n,
                       (uint32_t)nt, counts);
    hipLaunchKernelGGL(nxg_part_scan_kernel, dim3(NB), dim3(TPB), 0, s, counts, (uint32_t)nt,
                       totals);
    hipLaunchKernelGGL(nxg_part_offsets_kernel, dim3(1), dim3(TPB), 0, s, totals, off);
    hipLaunchKernelGGL(nxg_part_place_kernel, dim3((uint32_t)nt), dim3(TPB), 0, s, tag, fixed, aux,
                       n, (uint32_t)nt, counts, off, rank, row_of, dfixed, daux);
    return hipGetLastError();
}
