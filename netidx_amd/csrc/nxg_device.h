// nxg_device.h -- device-side primitives shared by the gfx950 codec kernels.
//
// These are re-statements of the reference's scalar rules, written for the device:
//   varint_len            netidx-core/src/pack.rs:472-474
//   decode_varint         pack.rs:504-520 (reads <= 10 bytes from the Take-limited chunk)
//   len_wrapped_len       pack.rs:522-525
//   zigzag                pack.rs:488-502
//   str::from_utf8        pack.rs:462
//   DateTime::from_timestamp validity  pack.rs:1572 (chrono >= 0.4.35 rules)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nxg_internal.h"

#define NXG_DEV __device__ __forceinline__

// ---- inter-workgroup hand-off (MI355X_MICROARCH.md "Valid forms"): 8-byte granules written
// with one agent-scope relaxed atomic store (sc1) and polled with agent-scope relaxed loads.
NXG_DEV uint64_t ld_agent(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
NXG_DEV uint32_t ld_agent32(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
NXG_DEV void st_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// drain this wave's outstanding stores before a flag store (guide: asm wait, never builtin)
NXG_DEV void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// watchdog: 100 MHz s_memrealtime, bound every spin (deadlock => NXG_TIMEOUT, never a hang)
NXG_DEV uint64_t rt_now() { return __builtin_amdgcn_s_memrealtime(); }
constexpr uint64_t kSpinTicks = 200ull * 1000 * 1000;  // 2 s at 100 MHz
constexpr uint32_t kSpinPolls = 1u << 20;               // ~1 s of polls at ~1 us each
// A bounded spin ends when BOTH 2 s have passed and about 1 s of polls were made: the clock
// alone would also count time the queue spent switched out (GPUs shared by several processes,
// compute wave save/restore), during which the waited-for workgroup cannot make progress either.
NXG_DEV bool spin_expired(uint64_t t_start, uint32_t polls) {
    return polls > kSpinPolls && rt_now() - t_start > kSpinTicks;
}

NXG_DEV uint32_t vl64(uint64_t v) {
    uint32_t hb = 63u - (uint32_t)__clzll((long long)(v | 1ull));
    return (hb * 9u + 73u) >> 6;
}
NXG_DEV uint64_t lwlen(uint64_t n) { return n + vl64(n + vl64(n)); }
NXG_DEV uint32_t zz32(int32_t n) { return ((uint32_t)n << 1) ^ (uint32_t)(n >> 31); }
NXG_DEV uint64_t zz64(int64_t n) { return ((uint64_t)n << 1) ^ (uint64_t)(n >> 63); }

NXG_DEV uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbyte(hi, lo, s);
}
NXG_DEV uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// SWAR: 0x80 in every zero byte of x (exact, no borrow propagation)
NXG_DEV uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
}
// gather the 0x80 flags of a zero_bytes() result into 4 bits
NXG_DEV uint32_t nib(uint32_t zb) { return (((zb >> 7) & 0x01010101u) * 0x01020408u) >> 24; }

// A wave's LDS image is private to it and LDS operations of one wave complete in order, so only
// the compiler has to be kept from moving accesses across this point.
NXG_DEV void wave_lds_order() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// ---- wave/block scans (wave64) -----------------------------------------------------------
NXG_DEV uint32_t lane_id() { return __lane_id(); }

// Wave scans with DPP (no LDS round trips; __shfl_up/__shfl_xor would compile to
// ds_bpermute_b32, one dependent LDS trip per step). The GFX9 inclusive scan: row_shr 1, 2, 4, 8
// within each 16-lane row, then row_bcast:15 into rows 1 and 3, row_bcast:31 into rows 2 and 3.
// A lane whose source is outside its row reads 0 (old = 0, bound_ctrl off). All 64 lanes must be
// active.
template <int CTRL, int ROWS>
NXG_DEV uint32_t dpp0(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS>
NXG_DEV uint64_t dpp0_64(uint64_t v) {
    return (uint64_t)dpp0<CTRL, ROWS>((uint32_t)v) | ((uint64_t)dpp0<CTRL, ROWS>((uint32_t)(v >> 32)) << 32);
}
template <typename T>
NXG_DEV T wave_incl_scan(T v) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit");
    if constexpr (sizeof(T) == 4) {
        uint32_t x = (uint32_t)v;
        x += dpp0<0x111, 0xf>(x);
        x += dpp0<0x112, 0xf>(x);
        x += dpp0<0x114, 0xf>(x);
        x += dpp0<0x118, 0xf>(x);
        x += dpp0<0x142, 0xa>(x);
        x += dpp0<0x143, 0xc>(x);
        return (T)x;
    } else {
        uint64_t x = (uint64_t)v;
        x += dpp0_64<0x111, 0xf>(x);
        x += dpp0_64<0x112, 0xf>(x);
        x += dpp0_64<0x114, 0xf>(x);
        x += dpp0_64<0x118, 0xf>(x);
        x += dpp0_64<0x142, 0xa>(x);
        x += dpp0_64<0x143, 0xc>(x);
        return (T)x;
    }
}

// wave minimum (uniform), by the same DPP pattern with all-ones as the identity
template <int CTRL, int ROWS>
NXG_DEV uint32_t dppmax(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, CTRL, ROWS, 0xf, false);
}
NXG_DEV uint32_t wave_min_u32(uint32_t x) {
    x = min(x, dppmax<0x111, 0xf>(x));
    x = min(x, dppmax<0x112, 0xf>(x));
    x = min(x, dppmax<0x114, 0xf>(x));
    x = min(x, dppmax<0x118, 0xf>(x));
    x = min(x, dppmax<0x142, 0xa>(x));
    x = min(x, dppmax<0x143, 0xc>(x));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// wave OR (uniform), the same DPP pattern with 0 as the identity
NXG_DEV uint32_t wave_or_u32(uint32_t x) {
    x |= dpp0<0x111, 0xf>(x);
    x |= dpp0<0x112, 0xf>(x);
    x |= dpp0<0x114, 0xf>(x);
    x |= dpp0<0x118, 0xf>(x);
    x |= dpp0<0x142, 0xa>(x);
    x |= dpp0<0x143, 0xc>(x);
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

// the next lane's value (lane 63: 0) -- DPP wave_shl:1
NXG_DEV uint32_t wave_next(uint32_t v) { return dpp0<0x130, 0xf>(v); }

// lane 63's value, wave-uniform (a scalar read, no LDS)
template <typename T>
NXG_DEV T wave_last(T v) {
    if constexpr (sizeof(T) == 4) {
        return (T)__builtin_amdgcn_readlane((int)v, 63);
    } else {
        const uint64_t x = (uint64_t)v;
        return (T)((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63) |
                   ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63) << 32));
    }
}

template <typename T>
NXG_DEV T wave_sum(T v) {
    return wave_last<T>(wave_incl_scan<T>(v));
}

// ---- decoupled look-back with a wide window ---------------------------------------------------
// The next tile of a look-back kernel for this workgroup, handed out by an atomic ticket in the
// order workgroups actually start. The hardware dispatches in order only per XCD: on a GPU that
// several processes share, one XCD can fall behind, and a workgroup whose look-back waits on a
// lower blockIdx not yet dispatched there would spin until the watchdog (seen with 2-3 processes
// on one device). With tickets every tile waited on was taken by a running workgroup.
// Block-wide (contains __syncthreads); `sh` is a __shared__ word.
NXG_DEV uint32_t next_tile(unsigned long long* ticket, uint32_t* sh) {
    __syncthreads();  // every thread has read the previous ticket
    if (threadIdx.x == 0) *sh = (uint32_t)atomicAdd(ticket, 1ull);
    __syncthreads();
    return *sh;
}

// Exclusive prefix of `tile` over the epoch-tagged tile words tstat[0..tile). Called by one full
// wave. The first poll covers the 64 nearest predecessors (lane l owns tile-1-l); when none of
// them is inclusive yet, later polls cover 64*U predecessors at once (word tile-1-64u-l for
// u = 0..U-1, each load instruction still one contiguous 512-byte run), so the inclusive front
// advances 64*U tiles per memory round trip instead of 64. Sets `give_up` on the watchdog or when
// *abort becomes non-zero (abort may be null).
template <int U>
NXG_DEV uint64_t lookback_prefix(const uint64_t* tstat, uint32_t tile, uint32_t epoch,
                                 const uint32_t* abort, bool& give_up) {
    const uint32_t lane = lane_id();
    uint64_t base = 0;
    int64_t pred = (int64_t)tile - 1;
    const uint64_t t_start = rt_now();
    uint32_t polls = 0;
    give_up = false;
    int nu = 1;  // rows of 64 words polled in this step
    while (pred >= 0) {
        uint64_t s[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int64_t idx = pred - 64 * u - (int64_t)lane;
            s[u] = (u < nu && idx >= 0) ? ld_agent(&tstat[idx]) : lb_word(kFlagInc, epoch, 0);
        }
        int uf;          // row of the nearest inclusive word (nu: none)
        uint32_t lf;     // its lane
        for (;;) {
            uf = nu;
            lf = 64;
            bool hole = false;
#pragma unroll
            for (int u = 0; u < U; u++) {
                if (u >= nu || uf < nu) break;
                const uint64_t f = lb_flag(s[u], epoch);
                const uint64_t m = __ballot(f == kFlagInc);
                if (m) {
                    uf = u;
                    lf = (uint32_t)__builtin_ctzll(m);
                    hole |= (f == 0) && lane < lf;
                } else {
                    hole |= (f == 0);
                }
            }
            if (!__any(hole)) break;
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int64_t idx = pred - 64 * u - (int64_t)lane;
                if (u < nu && lb_flag(s[u], epoch) == 0) s[u] = ld_agent(&tstat[idx]);
            }
            if ((abort && ld_agent32(abort)) || spin_expired(t_start, ++polls)) {
                give_up = true;
                return 0;
            }
        }
        uint64_t part = 0;
#pragma unroll
        for (int u = 0; u < U; u++)
            if (u < uf || (u == uf && lane <= lf)) part += s[u] & kValMask;
        base += wave_sum<uint64_t>(part);
        if (uf < nu) break;
        pred -= 64 * nu;
        nu = U;
    }
    return base;
}

// Exclusive prefix of `tile` over the epoch-tagged words tstat[0..tile), by one full wave, that
// never depends on another workgroup being scheduled: a predecessor that has published nothing
// after `patience` polls has its aggregate computed here by `count(t)` (wave-collective, returns
// the wave-uniform aggregate of tile t, exactly what tile t itself publishes). Dispatch is in order
// only per XCD: on a GPU shared by several processes an XCD can fall behind with the awaited
// workgroup not yet dispatched, and a plain look-back would wait on it until the watchdog.
template <typename F>
NXG_DEV uint64_t lookback_selfhelp_fn(const uint64_t* tstat, uint32_t tile, uint32_t epoch,
                                      uint32_t patience, F&& count) {
    const uint32_t lane = lane_id();
    uint64_t base = 0;
    int64_t pred = (int64_t)tile - 1;
#pragma unroll 1
    while (pred >= 0) {
        const int64_t idx = pred - (int64_t)lane;
        uint64_t s = idx >= 0 ? ld_agent(&tstat[idx]) : lb_word(kFlagInc, epoch, 0);
        uint32_t polls = 0;
#pragma unroll 1
        for (;;) {
            const uint64_t f = lb_flag(s, epoch);
            const uint64_t im = __ballot(f == kFlagInc);
            const uint32_t lf = im ? (uint32_t)__builtin_ctzll(im) : 64u;
            const uint64_t holes = __ballot(f == 0 && lane < lf);
            if (!holes) break;  // every tile up to the nearest inclusive one has its count
            if (++polls > patience) {
                // the nearest hole's aggregate, computed here
                const uint32_t h = (uint32_t)__builtin_ctzll(holes);
                const uint64_t agg = count((uint64_t)(pred - (int64_t)h));
                if (lane == h) s = lb_word(kFlagAgg, epoch, agg);
                polls = 0;
                continue;
            }
            __builtin_amdgcn_s_sleep(1);
            if (f == 0 && idx >= 0) s = ld_agent(&tstat[idx]);
        }
        const uint64_t im = __ballot(lb_flag(s, epoch) == kFlagInc);
        const uint32_t lf = im ? (uint32_t)__builtin_ctzll(im) : 64u;
        base += wave_sum<uint64_t>(lane <= lf ? (s & kValMask) : 0ull);
        if (im) break;
        pred -= 64;
    }
    return base;
}

// f() for each (active) lane with `want`, one lane at a time (uniform loop; the others wait):
// lanes that share one per-wave resource (an LDS stack) take turns
template <typename F>
NXG_DEV void one_lane_at_a_time(bool want, F&& f) {
    uint64_t m = __ballot(want);
#pragma unroll 1
    while (m) {
        const uint32_t j = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        if (lane_id() == j) f();
    }
}

// exclusive scan over a 256-thread block; `tmp` = 4 (or more) T in LDS. Returns the exclusive
// prefix, sets *total. Contains __syncthreads().
template <typename T, int NT>
NXG_DEV T block_excl_scan(T v, T* tmp, T* total) {
    const uint32_t tid = threadIdx.x, w = tid >> 6, l = tid & 63;
    T inc = wave_incl_scan(v);
    if (l == 63) tmp[w] = inc;
    __syncthreads();
    T wbase = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) {
        T x = tmp[i];
        if ((uint32_t)i < w) wbase += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return wbase + inc - v;
}

// ---- UTF-8 (std::str::from_utf8) over an arbitrary byte source -----------------------------
template <typename Src>
NXG_DEV bool utf8_valid(const Src& s, uint64_t p, uint64_t n) {
    uint64_t i = 0;
    while (i < n) {
        uint32_t c = s.byte(p + i);
        if (c < 0x80) {
            i++;
            continue;
        }
        uint32_t lo = 0x80, hi = 0xBF, need;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c == 0xE0) { need = 2; lo = 0xA0; }
        else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) need = 2;
        else if (c == 0xED) { need = 2; hi = 0x9F; }
        else if (c == 0xF0) { need = 3; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) need = 3;
        else if (c == 0xF4) { need = 3; hi = 0x8F; }
        else return false;
        if (i + need >= n) return false;
        uint32_t c1 = s.byte(p + i + 1);
        if (c1 < lo || c1 > hi) return false;
        for (uint32_t k = 2; k <= need; k++)
            if ((s.byte(p + i + k) & 0xC0) != 0x80) return false;
        i += need + 1;
    }
    return true;
}

// ---- chrono DateTime::from_timestamp validity ----------------------------------------------
// days-from-CE bounds of NaiveDate::MIN (-262143-01-01) and MAX (262142-12-31)
constexpr int64_t kMinDaysCE = -95746129;  // days_from_civil(-262143,1,1) + 719163
constexpr int64_t kMaxDaysCE = 95745399;   // days_from_civil(262142,12,31) + 719163
NXG_DEV bool datetime_valid(int64_t secs, uint32_t ns) {
    if (ns >= 2000000000u) return false;
    // |secs| < 2^42 (about 139,000 years) lies inside the range below: no day arithmetic, and
    // the leap-second test needs only secs mod 60 (86400 is a multiple of 60)
    if (secs > -(1ll << 42) && secs < (1ll << 42)) {
        if (ns < 1000000000u) return true;
        const int32_t hi = (int32_t)(secs >> 21);  // secs = hi * 2^21 + lo, exactly
        const int32_t lo = (int32_t)(secs & ((1 << 21) - 1));
        // 2^21 mod 60 = 32; floored mod of hi * 32 + lo, all within 32 bits
        int32_t m = ((hi % 60) * 32 + lo % 60) % 60;
        if (m < 0) m += 60;
        return m == 59;
    }
    int64_t days = secs / 86400;
    int64_t sod = secs % 86400;
    if (sod < 0) {
        sod += 86400;
        days -= 1;
    }
    int64_t dce = days + 719163;
    if (dce < kMinDaysCE || dce > kMaxDaysCE) return false;
    if (ns >= 2000000000u) return false;
    if (ns >= 1000000000u && (sod % 60) != 59) return false;
    return true;
}
