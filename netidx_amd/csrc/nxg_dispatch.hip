// nxg_dispatch.hip -- subscriber update dispatch for gfx950: the decoded Update rows fanned out
// to the subscriber's channels. Replaces ConnectionCtx::process_updates_batch
// (netidx/src/subscriber/connection.rs:546-567): per update, in batch order, the Id -> Sub lookup
// (a dense table here: publisher Ids count up from 0, netidx-core/src/utils.rs:130-134), one
// (SubId, update) entry per stream of the subscription appended to that stream's channel batch
// (by_chan, connection.rs:551-557), and the subscription's `last` (connection.rs:559-561).
//
// Output is grouped by channel, each channel's batch in batch order (CSR, chan_off). Three
// launches, deterministic (no atomics decide an order):
//   count    one wave per segment of SEG rows (64 rows per step); one counter increment per
//            (row, stream), order-free. Counters end in hist[chan * n_seg + seg] (channel-major).
//            Also: last_row (atomicMax of row + 1), unmatched rows. (NXG_DISP_LASTP: a plain store
//            that the scatter raises to the slot's last row, measured slower.)
//   scan     exclusive scan of hist in that order: the first entry of every (channel, segment)
//            pair; chan_off[c] is the (c, 0) value.
//   scatter  the rows again; an entry's position is the wave's running count for its channel
//            plus its rank within the 64-row step: each (row, stream) sets its lane's bit in its
//            channel's LDS mask and counts the lower bits (a row names a channel at most once,
//            connection.rs:328-356); steps with a repeated channel in one row, or rows with more
//            than RF streams, use a "match" loop instead (wave minimum of each lane's next
//            channel, an inclusive scan over lanes per channel). Entries come out in row order.
// Counters live in LDS when there are at most LCH channels, in global memory otherwise.
#include "nxg_device.h"
#include "nxg_internal.h"

namespace {

constexpr int TPB = 256;
constexpr int WAVES = TPB / 64;
constexpr uint32_t LCH = 1024;        // channels with LDS counters (u64 per channel per wave)
constexpr uint32_t NONE = 0xffffffffu;
constexpr int SCAN_K = 16;            // scan: elements per thread
constexpr uint32_t SCAN_B = TPB * SCAN_K;

constexpr uint32_t RF = 4;  // streams per row held in registers (more: read from memory)
#ifndef NXG_DISP_U
#define NXG_DISP_U 2  // (round 5, 1024-row segments: 1 / 2 / 4 steps 0.433 / 0.415 / 0.401-0.418 ms;
// round 6, one segment per wave: 128 rows x 2 steps 0.346-0.351, 256 x 4 0.337-0.360, 256 x 2
// 0.365-0.369, 512 x 8 0.418-0.422 ms, 1024 x 4 on a capped grid 0.366-0.384 ms)
#endif
constexpr int DU = NXG_DISP_U;  // 64-row steps whose lookups are in flight together
// (entries stored nontemporal measured 0.56 vs 0.40 ms: scattered 8-byte stores need the L2 to
// merge them into lines)

struct Row {
    uint32_t k0, k1;  // the row's streams [k0, k1) in stream_chan (empty: no subscription)
    uint32_t slot;
    uint32_t c[RF];   // their channels (NONE past k1 or >= n_chans), when k1 - k0 <= RF
};

// Per-row routing (publisher commit, nxg_publish.hip): mode 0 = through the Id's slot, 1 = not
// pushed (an unchanged UpdateChanged), 2 = to client to_client[i] only. `mode` null: all 0.
struct Route {
    const uint8_t* mode;
    const uint32_t* to_client;
};

NXG_DEV Row row_of(const NxgSubTable& tb, const Route& rt, const uint64_t* __restrict__ id,
                   uint64_t i, uint64_t n, bool& unmatched) {
    Row r{0, 0, NONE, {NONE, NONE, NONE, NONE}};
    unmatched = false;
    if (i < n) {
        const uint32_t m = rt.mode ? rt.mode[i] : 0u;
        if (m == 2) {  // one stream: the named client
            const uint32_t c = rt.to_client[i];
            r.k1 = 1;
            r.c[0] = c < tb.n_chans ? c : NONE;
            return r;
        }
        if (m == 1) return r;
        const uint64_t x = id[i];
        const uint32_t s = x < tb.n_ids ? tb.slot_of_id[x] : NONE;
        unmatched = s == NONE;
        if (s != NONE) {
            r.slot = s;
            r.k0 = tb.slot_stream_off[s];
            r.k1 = tb.slot_stream_off[s + 1];
#pragma unroll
            for (uint32_t j = 0; j < RF; j++) {
                const uint32_t c = r.k0 + j < r.k1 ? tb.stream_chan[r.k0 + j] : NONE;
                r.c[j] = c < tb.n_chans ? c : NONE;  // channels past n_chans: ignored
            }
        }
    }
    return r;
}

// the smallest channel above `prev` among the row's streams (NONE: none), and how many of the
// row's streams name channel `d`
NXG_DEV uint32_t next_chan(const NxgSubTable& tb, const Row& r, uint32_t prev, bool first) {
    uint32_t m = NONE;
    if (r.k1 - r.k0 <= RF) {
#pragma unroll
        for (uint32_t j = 0; j < RF; j++)
            if ((first || r.c[j] > prev) && r.c[j] < m) m = r.c[j];
        return m;
    }
    for (uint32_t k = r.k0; k < r.k1; k++) {
        const uint32_t c = tb.stream_chan[k];
        if ((first || c > prev) && c < m && c < tb.n_chans) m = c;  // others: ignored
    }
    return m;
}
NXG_DEV uint32_t count_chan(const NxgSubTable& tb, const Row& r, uint32_t d) {
    uint32_t n = 0;
    if (r.k1 - r.k0 <= RF) {
#pragma unroll
        for (uint32_t j = 0; j < RF; j++) n += r.c[j] == d;
        return n;
    }
    for (uint32_t k = r.k0; k < r.k1; k++) n += tb.stream_chan[k] == d;
    return n;
}

NXG_DEV uint32_t wave_min(uint32_t v) { return wave_min_u32(v); }

// The count pass's lookups kept for the scatter (NXG_DISP_CACHE): per row its slot and the
// channels of up to two streams (a 16-bit half each, kNoChan: none; kLookup in the low half: more
// streams, the scatter looks the row up again), so the scatter's chain of dependent loads is the
// cache and the SubId instead of Id -> slot -> stream offsets -> channel. Null pointers: no cache
// (kLookup channels or more). `narrow` (fewer than 254 channels): the two channels in the bytes
// of a 16-bit word (0xff none, 0xfe look up), 6 bytes per row instead of 8.
#ifndef NXG_DISP_CACHE
#define NXG_DISP_CACHE 1
#endif
constexpr uint16_t kNoChan = 0xffff, kLookup = 0xfffe;
struct RowCache {
    uint32_t* slot;
    void* ch;
    bool narrow;
};
#ifndef NXG_DISP_CNT
#define NXG_DISP_CNT 0  // 1: the cache stored nontemporal (A/B: 0.333-0.338 vs 0.334-0.341 ms, equal)
#endif
template <typename T>
NXG_DEV void cache_st(T* p, T v) {
    if (NXG_DISP_CNT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
NXG_DEV void cache_put(const RowCache& rc, uint64_t i, uint32_t slot, uint32_t ns, uint32_t c0,
                       uint32_t c1) {  // c0, c1: channels or NONE
    cache_st(&rc.slot[i], slot);
    if (rc.narrow)
        cache_st(&static_cast<uint16_t*>(rc.ch)[i],
                 (uint16_t)(ns > 2u ? 0xfeu
                                    : (c0 == NONE ? 0xffu : c0) | ((c1 == NONE ? 0xffu : c1) << 8)));
    else
        cache_st(&static_cast<uint32_t*>(rc.ch)[i],
                 ns > 2u ? (uint32_t)kLookup
                         : (c0 == NONE ? kNoChan : c0) | ((c1 == NONE ? kNoChan : c1) << 16));
}
// false: look the row up again; else its two channels (NONE: none)
NXG_DEV bool cache_get(const RowCache& rc, uint64_t i, uint32_t& c0, uint32_t& c1) {
    if (rc.narrow) {
        const uint32_t w = static_cast<const uint16_t*>(rc.ch)[i];
        c0 = w & 0xffu;
        c1 = w >> 8;
        if (c0 == 0xfeu) return false;
        c0 = c0 == 0xffu ? NONE : c0;
        c1 = c1 == 0xffu ? NONE : c1;
    } else {
        const uint32_t w = static_cast<const uint32_t*>(rc.ch)[i];
        c0 = w & 0xffffu;
        c1 = w >> 16;
        if (c0 == kLookup) return false;
        c0 = c0 == kNoChan ? NONE : c0;
        c1 = c1 == kNoChan ? NONE : c1;
    }
    return true;
}

}  // namespace

// ---- pass 1: per (channel, segment) entry counts ---------------------------------------------
#ifndef NXG_DISP_SKIP
#define NXG_DISP_SKIP 0  // timing experiments only: 1 last_row, 2 counters, 4 the row cache
#endif
#ifndef NXG_DISP_A32
#define NXG_DISP_A32 0  // 1: last_row's atomicMax on its low 32-bit word while rows fit 32 bits
// (A/B at 10^7, 16 channels: 0.316-0.321 vs 0.317-0.328 ms, equal)
#endif
#ifndef NXG_DISP_LASTP
#define NXG_DISP_LASTP 0  // 1: plain last_row stores finished by the scatter (measured slower: 0.353-0.363
// vs 0.337-0.350 ms sequential, 1.40-1.42 vs 1.10 ms random Ids at 10^7, 16 channels)
#endif
#ifndef NXG_DISP_COCC
#define NXG_DISP_COCC 1  // waves per SIMD asked of the register allocation (A/B)
#endif
__global__ __launch_bounds__(TPB, NXG_DISP_COCC) void nxg_disp_count_kernel(
    NxgSubTable tb, Route rt, const uint64_t* __restrict__ id, uint64_t n, uint64_t seg_rows,
    uint64_t n_seg,
    uint32_t* __restrict__ hist, uint64_t* __restrict__ last_row, uint64_t* __restrict__ unmatched,
    RowCache rc, bool plain_last) {
    // (dynamic LDS: n_chans counters per wave, sized at launch, so that few channels leave room
    // for more workgroups per CU)
    extern __shared__ __attribute__((aligned(16))) uint64_t dyn_lds[];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool lds = tb.n_chans <= LCH;
    uint32_t* cnt = reinterpret_cast<uint32_t*>(dyn_lds) + (size_t)w * tb.n_chans;
    uint64_t um = 0;
#pragma unroll 1
    for (uint64_t seg = (uint64_t)blockIdx.x * WAVES + w; seg < n_seg;
         seg += (uint64_t)gridDim.x * WAVES) {
        if (lds) {
            for (uint32_t c = lane; c < tb.n_chans; c += 64) cnt[c] = 0;
            wave_lds_order();
        }
        const uint64_t r0 = seg * seg_rows, r1 = r0 + seg_rows < n ? r0 + seg_rows : n;
#pragma unroll 1
        for (uint64_t b0 = r0; b0 < r1; b0 += 64 * DU) {
          // DU steps' rows looked up together (their dependent loads in flight at once)
          Row rows[DU];
          bool unms[DU];
#pragma unroll
          for (int u = 0; u < DU; u++) rows[u] = row_of(tb, rt, id, b0 + 64 * u + lane, r1, unms[u]);
#pragma unroll
          for (int u = 0; u < DU; u++) {
            const uint64_t i = b0 + 64 * u + lane;
            const bool unm = unms[u];
            const Row& r = rows[u];
            um += unm;
            if (!(NXG_DISP_SKIP & 4) && rc.slot && i < r1) {
                const uint32_t ns = r.k1 - r.k0;
                cache_put(rc, i, r.slot, ns, ns >= 1u ? r.c[0] : NONE, ns >= 2u ? r.c[1] : NONE);
            }
            if (!(NXG_DISP_SKIP & 1) && r.slot != NONE && (!tb.slot_has_last || tb.slot_has_last[r.slot])) {
                if (plain_last) last_row[r.slot] = i + 1;
                else if (NXG_DISP_A32 && n < 0xffffffffull)  // the low word (high words are 0)
                    atomicMax(reinterpret_cast<unsigned*>(&last_row[r.slot]), (unsigned)(i + 1));
                else atomicMax((unsigned long long*)&last_row[r.slot], (unsigned long long)(i + 1));
            }
            // order-free: one atomic per (row, stream)
            if (NXG_DISP_SKIP & 2) {
            } else if (r.k1 - r.k0 <= RF) {
#pragma unroll
                for (uint32_t j = 0; j < RF; j++) {
                    if (r.c[j] == NONE) continue;
                    if (lds) atomicAdd(&cnt[r.c[j]], 1u);
                    else atomicAdd(&hist[(uint64_t)r.c[j] * n_seg + seg], 1u);
                }
            } else {
                for (uint32_t k = r.k0; k < r.k1; k++) {
                    const uint32_t c = tb.stream_chan[k];
                    if (c >= tb.n_chans) continue;
                    if (lds) atomicAdd(&cnt[c], 1u);
                    else atomicAdd(&hist[(uint64_t)c * n_seg + seg], 1u);
                }
            }
          }
        }
        if (lds) {
            wave_lds_order();
            for (uint32_t c = lane; c < tb.n_chans; c += 64) hist[(uint64_t)c * n_seg + seg] = cnt[c];
            wave_lds_order();
        }
    }
    um = wave_sum<uint64_t>(um);
    if (lane == 0 && um) atomicAdd((unsigned long long*)unmatched, (unsigned long long)um);
}

// ---- pass 2: exclusive scan of hist (M values) into off (u64), block totals in bsum ----------
__global__ __launch_bounds__(TPB) void nxg_disp_scan_block_kernel(
    const uint32_t* __restrict__ hist, uint64_t M, uint64_t* __restrict__ off,
    uint64_t* __restrict__ bsum) {
    __shared__ uint64_t tmp[WAVES];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_B + (uint64_t)threadIdx.x * SCAN_K;
    uint64_t v[SCAN_K], local = 0;
#pragma unroll
    for (int k = 0; k < SCAN_K; k++) {
        v[k] = base + k < M ? hist[base + k] : 0u;
        local += v[k];
    }
    uint64_t total;
    uint64_t p = block_excl_scan<uint64_t, TPB>(local, tmp, &total);
#pragma unroll
    for (int k = 0; k < SCAN_K; k++) {
        if (base + k < M) off[base + k] = p;
        p += v[k];
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// one workgroup: exclusive scan of the block totals (nb values), grand total in bsum[nb]
__global__ __launch_bounds__(1024) void nxg_disp_scan_top_kernel(uint64_t* __restrict__ bsum,
                                                                 uint64_t nb) {
    __shared__ uint64_t tmp[16];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
#pragma unroll 1
    for (uint64_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint64_t i = b0 + threadIdx.x;
        const uint64_t v = i < nb ? bsum[i] : 0;
        uint64_t total;
        const uint64_t p = block_excl_scan<uint64_t, 1024>(v, tmp, &total);
        const uint64_t c = carry;
        if (i < nb) bsum[i] = c + p;
        __syncthreads();
        if (threadIdx.x == 0) carry = c + total;
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[nb] = carry;
}

// NXG_DISP_FUSE: the top scan also writes chan_off (each channel's first entry: its segment 0's
// block-local offset plus its block's prefix), and the scatter adds the block prefixes itself, so
// neither the scan_add launch nor chan_off's memset runs (LDS counters only; more channels keep
// the global cursors, which the scatter rewrites, and the add pass)
#ifndef NXG_DISP_FUSE
#define NXG_DISP_FUSE 1
#endif
__global__ __launch_bounds__(1024) void nxg_disp_scan_top_chan_kernel(
    uint64_t* __restrict__ bsum, uint64_t nb, const uint64_t* __restrict__ off, uint64_t n_seg,
    uint32_t n_chans, uint64_t* __restrict__ chan_off) {
    __shared__ uint64_t tmp[16];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
#pragma unroll 1
    for (uint64_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint64_t i = b0 + threadIdx.x;
        const uint64_t v = i < nb ? bsum[i] : 0;
        uint64_t total;
        const uint64_t p = block_excl_scan<uint64_t, 1024>(v, tmp, &total);
        const uint64_t c = carry;
        if (i < nb) bsum[i] = c + p;
        __syncthreads();
        if (threadIdx.x == 0) carry = c + total;
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[nb] = carry;
#pragma unroll 1
    for (uint32_t c = threadIdx.x; c < n_chans; c += 1024) {
        const uint64_t i = (uint64_t)c * n_seg;
        chan_off[c] = off[i] + bsum[i / SCAN_B];
    }
    if (threadIdx.x == 0) chan_off[n_chans] = carry;
}

__global__ __launch_bounds__(TPB) void nxg_disp_scan_add_kernel(
    uint64_t* __restrict__ off, uint64_t M, const uint64_t* __restrict__ bsum, uint64_t nb,
    uint64_t n_seg, uint32_t n_chans, uint64_t* __restrict__ chan_off) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i < M) {
        const uint64_t x = off[i] + bsum[i / SCAN_B];
        off[i] = x;
        if (i % n_seg == 0) chan_off[i / n_seg] = x;
    }
    if (i == 0) chan_off[n_chans] = bsum[nb];
}

// ---- pass 3: entries --------------------------------------------------------------------------
#ifndef NXG_DISP_SOCC
#define NXG_DISP_SOCC 1  // waves per SIMD asked of the register allocation (A/B)
#endif
__global__ __launch_bounds__(TPB, NXG_DISP_SOCC) void nxg_disp_scatter_kernel(
    NxgSubTable tb, Route rt, const uint64_t* __restrict__ id, uint64_t n, uint64_t seg_rows,
    uint64_t n_seg,
    uint64_t* __restrict__ off, uint64_t* __restrict__ ent_sub, uint64_t* __restrict__ ent_row,
    uint64_t cap, RowCache rc, uint64_t* __restrict__ last_row, bool plain_last,
    const uint64_t* __restrict__ bpre) {
    // (dynamic LDS: a cursor and a lane mask per channel and wave, sized at launch)
    extern __shared__ __attribute__((aligned(16))) uint64_t dyn_lds[];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool lds = tb.n_chans <= LCH;
    uint64_t* cur = dyn_lds + (size_t)w * 2 * tb.n_chans;
    uint64_t* mask = cur + tb.n_chans;
    const uint64_t lt = (1ull << lane) - 1;
#pragma unroll 1
    for (uint64_t seg = (uint64_t)blockIdx.x * WAVES + w; seg < n_seg;
         seg += (uint64_t)gridDim.x * WAVES) {
        if (lds) {
            for (uint32_t c = lane; c < tb.n_chans; c += 64) {
                const uint64_t i = (uint64_t)c * n_seg + seg;
                cur[c] = off[i] + (bpre ? bpre[i / SCAN_B] : 0ull);  // (bpre: the add pass skipped)
                mask[c] = 0;
            }
            wave_lds_order();
        }
        const uint64_t r0 = seg * seg_rows, r1 = r0 + seg_rows < n ? r0 + seg_rows : n;
#pragma unroll 1
        for (uint64_t b0 = r0; b0 < r1; b0 += 64 * DU) {
          // DU steps' rows and SubIds looked up together, then the steps in order
          Row rows[DU];
          uint64_t subs[DU], lastv[DU];
#pragma unroll
          for (int u = 0; u < DU; u++) {
            const uint64_t i = b0 + 64 * u + lane;
            bool unm;
            if (rc.slot) {
                uint32_t c0 = NONE, c1 = NONE;
                if (i < r1 && !cache_get(rc, i, c0, c1)) rows[u] = row_of(tb, rt, id, i, r1, unm);
                else rows[u] = Row{0u, 2u, i < r1 ? rc.slot[i] : NONE, {c0, c1, NONE, NONE}};
            } else {
                rows[u] = row_of(tb, rt, id, i, r1, unm);
            }
            // the entry's tag: the subscription's SubId, or (no SubId table) the row's own Id
            subs[u] = !tb.slot_sub_id ? (i < r1 ? id[i] : 0)
                      : (rows[u].slot != NONE ? tb.slot_sub_id[rows[u].slot] : 0);
            // the count pass's last_row of a kept slot (~0: none to check)
            lastv[u] = ~0ull;
            if (plain_last && rows[u].slot != NONE &&
                (!tb.slot_has_last || tb.slot_has_last[rows[u].slot]))
                lastv[u] = last_row[rows[u].slot];
          }
#pragma unroll
          for (int u = 0; u < DU; u++) {
            const uint64_t i = b0 + 64 * u + lane;
            const Row& r = rows[u];
            const uint64_t sub = subs[u];
            if (lastv[u] < i + 1)  // a later row of the slot than the count pass's store
                atomicMax((unsigned long long*)&last_row[r.slot], (unsigned long long)(i + 1));
            const bool dup = (r.c[0] != NONE && (r.c[0] == r.c[1] || r.c[0] == r.c[2] ||
                                                 r.c[0] == r.c[3])) ||
                             (r.c[1] != NONE && (r.c[1] == r.c[2] || r.c[1] == r.c[3])) ||
                             (r.c[2] != NONE && r.c[2] == r.c[3]);
            if (lds && !__any(r.k1 - r.k0 > RF || dup)) {
                // each (row, stream) sets its lane's bit in its channel's mask; a row names a
                // channel at most once here, so the entry's rank among the step's entries for
                // that channel is the number of lower lanes in the mask (row order)
#pragma unroll
                for (uint32_t j = 0; j < RF; j++)
                    if (r.c[j] != NONE) atomicOr((unsigned long long*)&mask[r.c[j]], 1ull << lane);
                wave_lds_order();
                uint64_t m[RF];
#pragma unroll
                for (uint32_t j = 0; j < RF; j++) {
                    m[j] = r.c[j] != NONE ? mask[r.c[j]] : 0ull;
                    if (r.c[j] != NONE) {
                        const uint64_t e = cur[r.c[j]] + __popcll(m[j] & lt);
                        if (e < cap) {
                            ent_sub[e] = sub;
                            ent_row[e] = i;
                        }
                    }
                }
                wave_lds_order();
                // the channel's highest lane advances its cursor and clears its mask
#pragma unroll
                for (uint32_t j = 0; j < RF; j++) {
                    if (r.c[j] != NONE && 63u - (uint32_t)__builtin_clzll(m[j]) == lane) {
                        cur[r.c[j]] += __popcll(m[j]);
                        mask[r.c[j]] = 0;
                    }
                }
                wave_lds_order();
                continue;
            }
            uint32_t prev = 0;
            bool first = true;
#pragma unroll 1
            for (;;) {
                const uint32_t d = wave_min(next_chan(tb, r, prev, first));
                if (d == NONE) break;
                const uint32_t c = count_chan(tb, r, d);
                const uint32_t inc = wave_incl_scan(c);
                // the wave owns this (channel, segment) cursor; in global memory it is read and
                // written past the L1 (the same wave reads its own store back next)
                uint64_t* gcur = &off[(uint64_t)d * n_seg + seg];
                const uint64_t base = lds ? cur[d] : ld_agent(gcur);
                for (uint32_t j = 0; j < c; j++) {
                    const uint64_t e = base + inc - c + j;
                    if (e < cap) {
                        ent_sub[e] = sub;
                        ent_row[e] = i;
                    }
                }
                const uint64_t nb = base + wave_last(inc);
                wave_lds_order();
                if (lane == 0) {
                    if (lds) cur[d] = nb;
                    else {
                        st_agent(gcur, nb);
                        drain_stores();
                    }
                }
                wave_lds_order();
                prev = d;
                first = false;
            }
          }
        }
    }
}

// ---- launch -------------------------------------------------------------------------------------
namespace {
constexpr uint64_t MAX_M = 1ull << 26;  // (channel, segment) counters
}

#ifndef NXG_DISP_SEG
#define NXG_DISP_SEG 128  // rows per segment (one group of NXG_DISP_U 64-row steps)
#endif
#ifndef NXG_DISP_GCAP
#define NXG_DISP_GCAP 0  // workgroups per CU at most (0: one segment per wave, no grid-stride)
#endif
uint64_t nxg_disp_seg_rows(uint64_t n, uint32_t n_chans) {
    uint64_t seg = NXG_DISP_SEG;
    const uint64_t ch = n_chans ? n_chans : 1;
    while (((n + seg - 1) / seg) * ch > MAX_M) seg *= 2;
    return seg;
}

uint64_t nxg_disp_scratch_bytes(uint64_t n, uint32_t n_chans) {
    const uint64_t seg = nxg_disp_seg_rows(n, n_chans);
    const uint64_t M = ((n + seg - 1) / seg) * (uint64_t)n_chans;
    const uint64_t nb = (M + SCAN_B - 1) / SCAN_B;
    return M * 4 + M * 8 + (nb + 1) * 8 + 64 + (NXG_DISP_CACHE ? n * 8 + 16 : 0);
}

hipError_t nxg_launch_dispatch(const NxgSubTable& tb, const uint64_t* id, uint64_t n,
                               uint8_t* scratch, uint64_t* chan_off, uint64_t* ent_sub,
                               uint64_t* ent_row, uint64_t cap, uint64_t* last_row,
                               uint64_t* unmatched, int ncu, hipStream_t s,
                               const uint8_t* row_mode, const uint32_t* to_client) {
    const Route rt{row_mode, to_client};
    const uint64_t seg = nxg_disp_seg_rows(n, tb.n_chans);
    const uint64_t n_seg = (n + seg - 1) / seg;
    const uint64_t M = n_seg * (uint64_t)tb.n_chans;
    const uint64_t nb = (M + SCAN_B - 1) / SCAN_B;
    uint32_t* hist = reinterpret_cast<uint32_t*>(scratch);
    uint64_t* off = reinterpret_cast<uint64_t*>(scratch + ((M * 4 + 7) & ~7ull));
    uint64_t* bsum = off + M;
#ifndef NXG_DISP_NARROW
#define NXG_DISP_NARROW 1
#endif
    RowCache rc{nullptr, nullptr, NXG_DISP_NARROW && tb.n_chans < 0xfeu};
    if (NXG_DISP_CACHE && tb.n_chans < kLookup) {
        rc.slot = reinterpret_cast<uint32_t*>(bsum + nb + 1);
        rc.ch = rc.slot + n;
    }
    hipError_t e;
    if ((e = hipMemsetAsync(unmatched, 0, 8, s)) != hipSuccess) return e;
    if (tb.n_slots && (e = hipMemsetAsync(last_row, 0, tb.n_slots * 8, s)) != hipSuccess) return e;
    const bool fuse = NXG_DISP_FUSE && M != 0 && tb.n_chans <= LCH;
    if (!fuse && (e = hipMemsetAsync(chan_off, 0, ((uint64_t)tb.n_chans + 1) * 8, s)) != hipSuccess)
        return e;
    if (n == 0) return hipSuccess;
    if (tb.n_chans > LCH && (e = hipMemsetAsync(hist, 0, M * 4, s)) != hipSuccess) return e;
    // one segment per wave: the hardware hands workgroups to CUs as they free up, so a wave's
    // chain of dependent lookups (Id -> slot -> streams -> channel) does not leave a tail of CUs
    // working a second segment while the others idle (round 6: 1024-row segments on a grid of
    // 8 workgroups per CU measured count 127 / scatter 185 us at 10^7 rows, 16 channels)
    const uint64_t want = (n_seg + WAVES - 1) / WAVES;
    const uint64_t gcap = NXG_DISP_GCAP ? (uint64_t)ncu * NXG_DISP_GCAP : 0x7fffffffull;
    const uint32_t g = (uint32_t)(want < gcap ? want : gcap);
    const bool in_lds = tb.n_chans <= LCH;
    // (no channels: no scatter to finish last_row, the count pass takes the atomics)
    const bool plain_last = NXG_DISP_LASTP && M != 0;
    const size_t lds_count = in_lds ? (size_t)WAVES * tb.n_chans * 4 : 0;
    const size_t lds_scatter = in_lds ? (size_t)WAVES * tb.n_chans * 16 : 0;
    hipLaunchKernelGGL(nxg_disp_count_kernel, dim3(g), dim3(TPB), lds_count, s, tb, rt, id, n, seg,
                       n_seg, hist, last_row, unmatched, rc, plain_last);
    if (M) {
        hipLaunchKernelGGL(nxg_disp_scan_block_kernel, dim3((uint32_t)nb), dim3(TPB), 0, s, hist, M,
                           off, bsum);
        if (fuse) {
            hipLaunchKernelGGL(nxg_disp_scan_top_chan_kernel, dim3(1), dim3(1024), 0, s, bsum, nb,
                               off, n_seg, tb.n_chans, chan_off);
        } else {
            hipLaunchKernelGGL(nxg_disp_scan_top_kernel, dim3(1), dim3(1024), 0, s, bsum, nb);
            hipLaunchKernelGGL(nxg_disp_scan_add_kernel, dim3((uint32_t)((M + TPB - 1) / TPB)),
                               dim3(TPB), 0, s, off, M, bsum, nb, n_seg, tb.n_chans, chan_off);
        }
        hipLaunchKernelGGL(nxg_disp_scatter_kernel, dim3(g), dim3(TPB), lds_scatter, s, tb, rt, id,
                           n, seg, n_seg, off, ent_sub, ent_row, cap, rc, last_row, plain_last,
                           fuse ? (const uint64_t*)bsum : nullptr);
    }
    return hipGetLastError();
}
