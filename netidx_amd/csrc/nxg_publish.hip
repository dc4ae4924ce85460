// nxg_publish.hip -- the publisher's commit for gfx950: UpdateBatch::commit
// (netidx/src/publisher/mod.rs:776-845). Queued messages, in batch order:
//   Update(None, id, v)   if id is published (pb.by_id), From::Update(id, v) goes to every
//                         subscribed client's batch and becomes the value's `current`;
//   UpdateChanged(id, v)  the same, only if current != v (Value::eq, netidx-value/src/op.rs:133-172);
//   Update(Some(cl), ..)  From::Update(id, v) to client cl only.
// The per-client batches are built by the dispatch kernels (nxg_dispatch.hip) with per-row
// routing; this file decides the routing of the UpdateChanged rows.
//
// UpdateChanged without a sequential loop. Value::eq is an equivalence relation (NaN == NaN,
// +0 == -0, otherwise exact), and `current` only ever takes values of the rows that are pushed,
// each of which differs from the value before it. So `current != v` at row i equals
// `prev(i) != v`, where prev(i) is the previous row of the same Id in the batch (any Update(None)
// or UpdateChanged row, pushed or not: an unpushed one equals current), or the table's current
// value when there is none. prev() is found by a stable LSD radix sort of (slot, row) -- only
// when some slot occurs twice in a batch that has UpdateChanged rows.
//
// Equality is Value::eq on every variant, over the columnar contract: text, Decimal and Abstract
// bytes in the heap, the elements of Array / Map / Error(Value) as child slots. Containers are
// compared by an explicit stack (no device recursion), off the scalar path. Map entries are
// compared in column order: the reference's encoder writes a map's entries sorted by key and
// unique, so two encodings of equal maps hold the same entries in the same order.
#include <algorithm>

#include "nxg_device.h"
#include "nxg_internal.h"

namespace {

constexpr int TPB = 256;
constexpr int WAVES = TPB / 64;
constexpr uint32_t NONE = 0xffffffffu;
constexpr uint32_t SEG = 1024;  // radix pass: items per wave segment (64 per step)
constexpr uint32_t BINS = 256;
constexpr int MAX_DEPTH = 32;  // NXG_MAX_DEPTH: deeper values fail the call (NXG_UNSUPPORTED)

// a source of values: top-level slots (tag null: all F64, aux null: 0) and their child slots
struct VSrc {
    const uint8_t* tag;
    const uint64_t* fixed;
    const uint32_t* aux;
    const uint8_t* ctag;
    const uint64_t* cfixed;
    const uint32_t* caux;
    const uint8_t* heap;
};

NXG_DEV bool heavy(uint32_t t) { return t == 19 || t == 20 || t == 21 || t == 22 || t == 27; }

NXG_DEV int float_eq(uint32_t t, uint64_t fa, uint64_t fb) {
    if (t == 8) {  // F32: NaN == NaN, otherwise IEEE == (+0 == -0)
        const float l = __uint_as_float((uint32_t)fa), r = __uint_as_float((uint32_t)fb);
        return (l != l && r != r) || l == r;
    }
    const double l = __longlong_as_double((long long)fa), r = __longlong_as_double((long long)fb);
    return (l != l && r != r) || l == r;
}

NXG_DEV int bytes_eq(const uint8_t* p, const uint8_t* q, uint32_t n) {
    for (uint32_t k = 0; k < n; k++)
        if (p[k] != q[k]) return 0;
    return 1;
}

// Value::eq for the scalar tags (no Decimal, container or Abstract): 1 equal, 0 different
NXG_DEV int scalar_eq(uint32_t ta, uint64_t fa, uint32_t aa, const uint8_t* ha, uint32_t tb,
                      uint64_t fb, uint32_t ab, const uint8_t* hb) {
    if (ta == 17) ta = 16;  // the old Ok decodes to Null
    if (tb == 17) tb = 16;
    if (ta != tb) return 0;  // different Typ, or Bool(true) vs Bool(false)
    switch (ta) {
    case 8: case 9: return float_eq(ta, fa, fb);
    case 10: case 11: return fa == fb && aa == ab;  // DateTime / Duration
    case 12: case 13: case 18: return aa == ab && bytes_eq(ha + fa, hb + fb, aa);
    case 14: case 15: case 16: return 1;
    default: return fa == fb;  // integers (signed sign-extended), V32/Z32 as stored
    }
}

NXG_DEV uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// rust_decimal's PartialEq (Decimal::serialize bytes: flags, lo, mid, hi little-endian; scale =
// flags bits 16..23, sign = bit 31): numeric equality, exact for any scale byte -- a mantissa
// below 2^96 < 10^29 cannot equal a non-zero one scaled by 10^29 or more.
NXG_DEV int decimal_eq(const uint8_t* a, const uint8_t* b) {
    const uint32_t fa = le32(a), fb = le32(b);
    uint32_t ma0 = le32(a + 4), ma1 = le32(a + 8), ma2 = le32(a + 12);
    uint32_t mb0 = le32(b + 4), mb1 = le32(b + 8), mb2 = le32(b + 12);
    const bool za = !(ma0 | ma1 | ma2), zb = !(mb0 | mb1 | mb2);
    if (za || zb) return za && zb;
    if ((fa >> 31) != (fb >> 31)) return 0;
    uint32_t sa = (fa >> 16) & 0xffu, sb = (fb >> 16) & 0xffu;
    if (sa > sb) {  // scale the smaller-scale side: m_small * 10^d == m_large
        uint32_t t = ma0; ma0 = mb0; mb0 = t;
        t = ma1; ma1 = mb1; mb1 = t;
        t = ma2; ma2 = mb2; mb2 = t;
        t = sa; sa = sb; sb = t;
    }
    const uint32_t d = sb - sa;
    if (d > 28) return 0;
    uint64_t w0 = ma0, w1 = ma1, w2 = ma2, w3 = 0;  // 128 bits suffice: m < 2^96, 10^28 < 2^94
    for (uint32_t k = 0; k < d; k++) {                 // but the product may reach 2^190: keep
        uint64_t x = w0 * 10;                          // the top limb saturating
        w0 = x & 0xffffffffu;
        x = w1 * 10 + (x >> 32);
        w1 = x & 0xffffffffu;
        x = w2 * 10 + (x >> 32);
        w2 = x & 0xffffffffu;
        w3 = (x >> 32) | (w3 ? 1u : 0u);  // any bit above 96 makes the product unequal
    }
    return w0 == mb0 && w1 == mb1 && w2 == mb2 && !w3;
}

NXG_DEV void slot_at(const VSrc& s, bool child, uint64_t i, uint32_t& t, uint64_t& f, uint32_t& a) {
    if (child) {
        t = s.ctag[i];
        f = s.cfixed[i];
        a = s.caux[i];
    } else {
        t = s.tag ? s.tag[i] : 9u;
        f = s.fixed[i];
        a = s.aux ? s.aux[i] : 0u;
    }
}

// Error(String) has two spellings in the columns: tag 18, or tag 22 over a String child
NXG_DEV void norm_error(const VSrc& s, uint32_t& t, uint64_t& f, uint32_t& a) {
    if (t == 22 && s.ctag && s.ctag[f] == 12) {
        const uint64_t c = f;
        t = 18;
        f = s.cfixed[c];
        a = s.caux[c];
    }
}

// one node of the comparison: 0 different, 1 equal, 2 equal so far with `n` child pairs to
// compare at child slots fa.., fb..; -1 a container whose source has no child columns
NXG_DEV int node_eq(const VSrc& A, uint32_t ta, uint64_t fa, uint32_t aa, const VSrc& B,
                    uint32_t tb, uint64_t fb, uint32_t ab, uint64_t& n) {
    if (ta == 22) norm_error(A, ta, fa, aa);
    if (tb == 22) norm_error(B, tb, fb, ab);
    if (!heavy(ta) && !heavy(tb)) return scalar_eq(ta, fa, aa, A.heap, tb, fb, ab, B.heap);
    if (ta != tb) return 0;
    switch (ta) {
    case 20: return decimal_eq(A.heap + fa, B.heap + fb);
    case 27: return aa == ab && bytes_eq(A.heap + fa, B.heap + fb, aa);  // Abstract: its bytes
    case 19: case 21:  // Array elements / Map entries (key, value) in column order
        if (aa != ab) return 0;
        if (aa && (!A.ctag || !B.ctag)) return -1;  // no child columns: the call fails
        n = ta == 19 ? (uint64_t)aa : 2ull * aa;
        return 2;
    default:  // Error(Value): the inner value
        if (!A.ctag || !B.ctag) return -1;
        n = 1;
        return 2;
    }
}

// Value::eq with containers: 1 equal, 0 different, -1 nested deeper than MAX_DEPTH (or no
// child columns). Without a stack (stk null) only one level of children is walked, and a child
// container gives DEEP_MORE; with one, stk holds 3 * (MAX_DEPTH + 1) words of pending child
// ranges (a per-wave LDS stack: the callers take turns, one_lane_at_a_time).
constexpr int DEEP_MORE = 3;
NXG_DEV int deep_eq(const VSrc& A, uint64_t ia, const VSrc& B, uint64_t ib, uint64_t* stk) {
    uint32_t ta, aa, tb, ab;
    uint64_t fa, fb, n = 0;
    slot_at(A, false, ia, ta, fa, aa);
    slot_at(B, false, ib, tb, fb, ab);
    int r = node_eq(A, ta, fa, aa, B, tb, fb, ab, n);
    if (r < 2) return r;
    if (!stk) {  // the common case: a flat container, walked in registers
        const uint64_t a0 = fa, b0 = fb;
        for (uint64_t k = 0; k < n; k++) {
            uint64_t m;
            slot_at(A, true, a0 + k, ta, fa, aa);
            slot_at(B, true, b0 + k, tb, fb, ab);
            r = node_eq(A, ta, fa, aa, B, tb, fb, ab, m);
            if (r <= 0) return r;
            if (r == 2) return DEEP_MORE;
        }
        return 1;
    }
    uint64_t* sa = stk;
    uint64_t* sb = stk + (MAX_DEPTH + 1);
    uint64_t* sn = stk + 2 * (MAX_DEPTH + 1);
    int sp = 0;
    sa[0] = fa, sb[0] = fb, sn[0] = n, sp = 1;
    while (sp > 0) {
        const int k = sp - 1;
        if (sn[k] == 0) {
            sp--;
            continue;
        }
        if (sp > MAX_DEPTH) return -1;  // the next child sits at depth sp
        const uint64_t ca = sa[k]++, cb = sb[k]++;
        sn[k]--;
        slot_at(A, true, ca, ta, fa, aa);
        slot_at(B, true, cb, tb, fb, ab);
        r = node_eq(A, ta, fa, aa, B, tb, fb, ab, n);
        if (r <= 0) return r;
        if (r == 2) sa[sp] = fa, sb[sp] = fb, sn[sp] = n, sp++;
    }
    return 1;
}

struct PubIn {
    const uint64_t* id;
    const uint8_t* kind;
    uint64_t n;
    VSrc v;  // the batch's values
};

NXG_DEV uint32_t slot_of(const NxgPubTable& tb, uint64_t x) {
    return x < tb.n_ids ? tb.slot_of_id[x] : NONE;
}

}  // namespace

// flags[0]: some slot occurs twice among the non-directed rows; flags[1]: UpdateChanged rows
// exist; flags[2]: a value nested deeper than MAX_DEPTH, or a container without child columns;
// flags[3]: some UpdateChanged row compares a Decimal, container or Abstract (nxg_pub_deep_kernel)
__global__ __launch_bounds__(TPB) void nxg_pub_count_kernel(NxgPubTable tb, PubIn in,
                                                            uint32_t* __restrict__ bm,
                                                            uint32_t* __restrict__ flags) {
    // a slot seen twice: its bit in the slot bitmap `bm` (zeroed) already set. 64 rows at a
    // time: when their slots fall in a few runs of equal bitmap words (Ids in order: 2-3 words
    // per 64 rows) each run's bits go in with one atomic from its first lane, otherwise one per
    // lane. A bounded grid strides over the rows, so the two flag words are touched once per
    // wave, not once per 64 rows (every wave of a one-row-per-thread grid reading one flag word
    // made that word's L2 channel the kernel's bound: 147 us at 10^7 rows).
    const uint32_t lane = threadIdx.x & 63;
    bool dup = false, chg = false;
#pragma unroll 1
    for (uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x; i - lane < in.n;
         i += (uint64_t)gridDim.x * TPB) {
        uint32_t s = NONE;
        if (i < in.n && in.kind[i] != NXG_PUB_UPDATE_CLIENT) {
            chg |= in.kind[i] == NXG_PUB_UPDATE_CHANGED;
            s = slot_of(tb, in.id[i]);
        }
        const bool v = s != NONE;
        const uint32_t wd = v ? s >> 5 : NONE, bit = v ? 1u << (s & 31u) : 0u;
        const uint32_t pw = (uint32_t)__shfl_up((int)wd, 1, 64);
        const uint64_t heads = __ballot(v && (lane == 0 || pw != wd));
        if (__popcll(heads) <= 4) {
#pragma unroll 1
            for (uint64_t hm = heads; hm; hm &= hm - 1) {
                const uint32_t h = (uint32_t)__builtin_ctzll(hm);
                const uint32_t w0 = (uint32_t)__builtin_amdgcn_readlane((int)wd, (int)h);
                const uint64_t after = hm & (hm - 1);  // the next run starts at the next head
                const uint32_t hn = after ? (uint32_t)__builtin_ctzll(after) : 64u;
                const bool in_run = lane >= h && lane < hn && wd == w0;
                const uint64_t rm = __ballot(in_run);
                const uint32_t orv = wave_or_u32(in_run ? bit : 0u);
                uint32_t old = 0;
                if (lane == h) old = atomicOr(&bm[w0], orv);
                old = (uint32_t)__builtin_amdgcn_readlane((int)old, (int)h);
                // a slot twice in the run, or already set
                if ((uint32_t)__popcll(rm) != (uint32_t)__popc(orv) || (old & orv)) dup = true;
            }
        } else if (v) {
            dup |= (atomicOr(&bm[wd], bit) & bit) != 0;
        }
    }
    if (__any(dup) && lane == 0 && !ld_agent32(&flags[0])) atomicOr(&flags[0], 1u);
    if (__any(chg) && lane == 0 && !ld_agent32(&flags[1])) atomicOr(&flags[1], 1u);
}

// radix keys: the slot of every non-directed row with one, else NONE (sorted last, ignored)
__global__ __launch_bounds__(TPB) void nxg_pub_keys_kernel(NxgPubTable tb, PubIn in,
                                                           uint32_t* __restrict__ key,
                                                           uint32_t* __restrict__ val) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= in.n) return;
    key[i] = in.kind[i] != NXG_PUB_UPDATE_CLIENT ? slot_of(tb, in.id[i]) : NONE;
    val[i] = (uint32_t)i;
}

// one stable counting-sort pass on bits [shift, shift+8) of key: per 1024-item segment (one
// wave) the digit counts, hist[bin * n_seg + seg]
__global__ __launch_bounds__(TPB) void nxg_radix_count_kernel(const uint32_t* __restrict__ key,
                                                              uint64_t n, uint32_t shift,
                                                              uint64_t n_seg,
                                                              uint32_t* __restrict__ hist) {
    __shared__ uint32_t cnt_lds[WAVES][BINS];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t* cnt = cnt_lds[w];
    for (uint64_t seg = (uint64_t)blockIdx.x * WAVES + w; seg < n_seg;
         seg += (uint64_t)gridDim.x * WAVES) {
        for (uint32_t c = lane; c < BINS; c += 64) cnt[c] = 0;
        wave_lds_order();
        const uint64_t r0 = seg * SEG, r1 = r0 + SEG < n ? r0 + SEG : n;
        for (uint64_t i = r0 + lane; i < r1; i += 64) atomicAdd(&cnt[(key[i] >> shift) & 255u], 1u);
        wave_lds_order();
        for (uint32_t c = lane; c < BINS; c += 64) hist[(uint64_t)c * n_seg + seg] = cnt[c];
        wave_lds_order();
    }
}

// the pass's scatter: an item's rank within its 64-item step is the number of lower lanes with
// the same digit (an LDS lane mask per digit), so equal digits keep their order (stable)
__global__ __launch_bounds__(TPB) void nxg_radix_scatter_kernel(
    const uint32_t* __restrict__ key, const uint32_t* __restrict__ val, uint64_t n, uint32_t shift,
    uint64_t n_seg, const uint64_t* __restrict__ off, uint32_t* __restrict__ key_out,
    uint32_t* __restrict__ val_out) {
    __shared__ uint64_t cur_lds[WAVES][BINS];
    __shared__ uint64_t mask_lds[WAVES][BINS];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t* cur = cur_lds[w];
    uint64_t* mask = mask_lds[w];
    const uint64_t lt = (1ull << lane) - 1;
    for (uint64_t seg = (uint64_t)blockIdx.x * WAVES + w; seg < n_seg;
         seg += (uint64_t)gridDim.x * WAVES) {
        for (uint32_t c = lane; c < BINS; c += 64) {
            cur[c] = off[(uint64_t)c * n_seg + seg];
            mask[c] = 0;
        }
        wave_lds_order();
        const uint64_t r0 = seg * SEG, r1 = r0 + SEG < n ? r0 + SEG : n;
        for (uint64_t b = r0; b < r1; b += 64) {
            const uint64_t i = b + lane;
            const bool in = i < r1;
            const uint32_t k = in ? key[i] : 0u, v = in ? val[i] : 0u;
            const uint32_t d = (k >> shift) & 255u;
            if (in) atomicOr((unsigned long long*)&mask[d], 1ull << lane);
            wave_lds_order();
            const uint64_t m = in ? mask[d] : 0ull;
            if (in) {
                const uint64_t e = cur[d] + __popcll(m & lt);
                key_out[e] = k;
                val_out[e] = v;
            }
            wave_lds_order();
            if (in && 63u - (uint32_t)__builtin_clzll(m) == lane) {
                cur[d] += __popcll(m);
                mask[d] = 0;
            }
            wave_lds_order();
        }
    }
}

// prev(row) from the sorted (slot, row) pairs: the preceding pair of the same slot
__global__ __launch_bounds__(TPB) void nxg_pub_prev_kernel(const uint32_t* __restrict__ key,
                                                           const uint32_t* __restrict__ val,
                                                           uint64_t n, uint32_t* __restrict__ prev) {
    const uint64_t k = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (k >= n || key[k] == NONE) return;
    prev[val[k]] = (k > 0 && key[k - 1] == key[k]) ? val[k - 1] : NONE;
}

// routing of every row (nxg_dispatch.hip Route): 0 through the slot, 1 not pushed, 2 one client
// the comparison of UpdateChanged row i: 1 equal, 0 different, -1 too deep; 2 (DEEP) when a
// side is a Decimal, container or Abstract and `deep` is false (left to nxg_pub_deep_kernel, so
// that this kernel needs no stack)
constexpr int DEEP = 2;
template <bool ALLOW_DEEP>
NXG_DEV int changed_eq(const NxgPubTable& tb, const PubIn& in, const uint32_t* prev, uint64_t i,
                       uint32_t s) {
    const uint32_t j = prev ? prev[i] : NONE;
    const VSrc cur{tb.cur_tag, tb.cur_fixed, tb.cur_aux, tb.cur_ctag, tb.cur_cfixed, tb.cur_caux,
                   tb.cur_heap};
    const VSrc& A = j != NONE ? in.v : cur;
    const uint64_t ia = j != NONE ? j : s;
    const uint32_t ta = A.tag ? A.tag[ia] : 9u, tb_ = in.v.tag ? in.v.tag[i] : 9u;
    if (heavy(ta) || heavy(tb_)) {
        if (!ALLOW_DEEP) return DEEP;
        // one level in registers; a nested container retries with the wave's LDS stack
        __shared__ uint64_t stks[WAVES][3 * (MAX_DEPTH + 1)];
        int r = deep_eq(A, ia, in.v, i, nullptr);
        one_lane_at_a_time(r == DEEP_MORE,
                           [&] { r = deep_eq(A, ia, in.v, i, stks[threadIdx.x >> 6]); });
        return r;
    }
    return scalar_eq(ta, A.fixed[ia], A.aux ? A.aux[ia] : 0u, A.heap, tb_, in.v.fixed[i],
                     in.v.aux ? in.v.aux[i] : 0u, in.v.heap);
}

// routing of every row (nxg_dispatch.hip Route): 0 through the slot, 1 not pushed, 2 one client;
// 3: an UpdateChanged whose comparison needs the stack walk (flags[3] set)
__global__ __launch_bounds__(TPB) void nxg_pub_mode_kernel(NxgPubTable tb, PubIn in,
                                                           const uint32_t* __restrict__ prev,
                                                           uint8_t* __restrict__ mode,
                                                           uint32_t* __restrict__ flags) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    bool deep = false;
    if (i < in.n) {
        const uint32_t kd = in.kind[i];
        uint32_t m = kd == NXG_PUB_UPDATE_CLIENT ? 2u : 0u;
        if (kd == NXG_PUB_UPDATE_CHANGED) {
            const uint32_t s = slot_of(tb, in.id[i]);
            if (s != NONE) {  // unpublished Ids stay 0: no slot, counted as unmatched
                const int eq = changed_eq<false>(tb, in, prev, i, s);
                deep = eq == DEEP;
                m = deep ? 3u : eq > 0 ? 1u : 0u;
            }
        }
        mode[i] = (uint8_t)m;
    }
    if (__any(deep) && (threadIdx.x & 63) == 0 && !ld_agent32(&flags[3])) atomicOr(&flags[3], 1u);
}

// the rows left at mode 3: Value::eq with the stack walk (containers, Decimal, Abstract)
__global__ __launch_bounds__(TPB) void nxg_pub_deep_kernel(NxgPubTable tb, PubIn in,
                                                           const uint32_t* __restrict__ prev,
                                                           uint8_t* __restrict__ mode,
                                                           uint32_t* __restrict__ flags) {
    for (uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x; i < in.n;
         i += (uint64_t)gridDim.x * TPB) {
        if (mode[i] != 3u) continue;
        const int eq = changed_eq<true>(tb, in, prev, i, slot_of(tb, in.id[i]));
        if (eq < 0 && !ld_agent32(&flags[2])) atomicOr(&flags[2], 1u);
        mode[i] = eq > 0 ? 1u : 0u;
    }
}

// ---- launch (host) ------------------------------------------------------------------------------
// kernels shared with the dispatch's scan (nxg_dispatch.hip)
__global__ void nxg_disp_scan_block_kernel(const uint32_t* __restrict__ hist, uint64_t M,
                                           uint64_t* __restrict__ off, uint64_t* __restrict__ bsum);
__global__ void nxg_disp_scan_top_kernel(uint64_t* __restrict__ bsum, uint64_t nb);

namespace {
constexpr uint32_t SCAN_B = 256 * 16;  // = nxg_dispatch.hip's scan block

__global__ __launch_bounds__(TPB) void add_block_kernel(uint64_t* __restrict__ off, uint64_t M,
                                                        const uint64_t* __restrict__ bsum) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i < M) off[i] += bsum[i / SCAN_B];
}
}  // namespace

// exclusive sums of M u32 counts into u64 offsets; bsum holds M / 4096 + 2 words
hipError_t nxg_scan_u32(const uint32_t* hist, uint64_t M, uint64_t* off, uint64_t* bsum,
                        hipStream_t s) {
    if (M == 0) return hipSuccess;
    const uint64_t nb = (M + SCAN_B - 1) / SCAN_B;
    hipLaunchKernelGGL(nxg_disp_scan_block_kernel, dim3((uint32_t)nb), dim3(256), 0, s, hist, M, off,
                       bsum);
    hipLaunchKernelGGL(nxg_disp_scan_top_kernel, dim3(1), dim3(1024), 0, s, bsum, nb);
    hipLaunchKernelGGL(add_block_kernel, dim3((uint32_t)((M + TPB - 1) / TPB)), dim3(TPB), 0, s, off,
                       M, bsum);
    return hipGetLastError();
}

uint64_t nxg_pub_scratch_bytes(uint64_t n, uint64_t n_slots) {
    const uint64_t n_seg = (n + SEG - 1) / SEG;
    const uint64_t M = n_seg * BINS;
    const uint64_t nb = (M + SCAN_B - 1) / SCAN_B;
    // flags, cnt[n_slots], keys/vals x2, prev, mode, hist, off, bsum
    return 64 + 4 * n_slots + 16 * n + 4 * n + n + 4 * M + 8 * M + 8 * (nb + 1) + 64;
}

// Stage 1 (flags); the host then decides which of stage 2 runs. Returns the scratch layout.
struct PubScratch {
    uint32_t* flags;
    uint32_t* cnt;
    uint32_t *k0, *v0, *k1, *v1;
    uint32_t* prev;
    uint8_t* mode;
    uint32_t* hist;
    uint64_t* off;
    uint64_t* bsum;
};
static PubScratch pub_layout(uint8_t* p, uint64_t n, uint64_t n_slots) {
    PubScratch sc;
    const uint64_t n_seg = (n + SEG - 1) / SEG;
    const uint64_t M = n_seg * BINS;
    sc.flags = reinterpret_cast<uint32_t*>(p);
    p += 64;
    sc.cnt = reinterpret_cast<uint32_t*>(p);
    p += 4 * n_slots;
    sc.k0 = reinterpret_cast<uint32_t*>(p);
    p += 4 * n;
    sc.v0 = reinterpret_cast<uint32_t*>(p);
    p += 4 * n;
    sc.k1 = reinterpret_cast<uint32_t*>(p);
    p += 4 * n;
    sc.v1 = reinterpret_cast<uint32_t*>(p);
    p += 4 * n;
    sc.prev = reinterpret_cast<uint32_t*>(p);
    p += 4 * n;
    sc.hist = reinterpret_cast<uint32_t*>(p);
    p += 4 * M;
    p = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(p) + 7) & ~uintptr_t(7));
    sc.off = reinterpret_cast<uint64_t*>(p);
    p += 8 * M;
    sc.bsum = reinterpret_cast<uint64_t*>(p);
    p += 8 * ((M + SCAN_B - 1) / SCAN_B + 1);
    sc.mode = p;
    return sc;
}

#ifndef NXG_PUB_GCAP
#define NXG_PUB_GCAP 8  // the repeated-Id check's workgroups per CU (a bounded grid striding over rows;
// A/B of the commit at 10^7: 4 0.550-0.556, 8 0.508-0.515, 16 0.504-0.514 ms)
#endif
hipError_t nxg_launch_pub_stage1(const NxgPubTable& tb, const NxgPubBatch& b, uint8_t* scratch,
                                 int ncu, hipStream_t s) {
    PubScratch sc = pub_layout(scratch, b.n_rows, tb.n_slots);
    const PubIn in{b.id, b.kind, b.n_rows, {b.tag, b.fixed, b.aux, b.ctag, b.cfixed, b.caux, b.heap}};
    hipError_t e;
    if ((e = hipMemsetAsync(sc.flags, 0, 64, s)) != hipSuccess) return e;
    if (tb.n_slots && (e = hipMemsetAsync(sc.cnt, 0, 4 * ((tb.n_slots + 31) / 32), s)) != hipSuccess)
        return e;  // (the slot bitmap)
    if (b.n_rows)
        hipLaunchKernelGGL(nxg_pub_count_kernel,
                           dim3((uint32_t)std::min<uint64_t>((b.n_rows + TPB - 1) / TPB,
                                                             (uint64_t)ncu * NXG_PUB_GCAP)),
                           dim3(TPB), 0, s, tb, in, sc.cnt, sc.flags);
    return hipGetLastError();
}

const uint32_t* nxg_pub_flags(uint8_t* scratch) { return reinterpret_cast<uint32_t*>(scratch); }

// Stage 2: the UpdateChanged routing (prev() by radix sort when `dup`), then returns the mode
// array (null: no UpdateChanged rows, the kinds route as they are).
hipError_t nxg_launch_pub_stage2(const NxgPubTable& tb, const NxgPubBatch& b, uint8_t* scratch,
                                 bool dup, bool changed, int ncu, hipStream_t s,
                                 const uint8_t** mode_out) {
    PubScratch sc = pub_layout(scratch, b.n_rows, tb.n_slots);
    const PubIn in{b.id, b.kind, b.n_rows, {b.tag, b.fixed, b.aux, b.ctag, b.cfixed, b.caux, b.heap}};
    const uint64_t n = b.n_rows;
    const uint32_t gi = (uint32_t)((n + TPB - 1) / TPB);
    *mode_out = nullptr;
    if (!changed || n == 0) return hipSuccess;
    const uint32_t* prev = nullptr;
    if (dup) {
        hipLaunchKernelGGL(nxg_pub_keys_kernel, dim3(gi), dim3(TPB), 0, s, tb, in, sc.k0, sc.v0);
        hipError_t e = hipMemsetAsync(sc.prev, 0xff, 4 * n, s);
        if (e != hipSuccess) return e;
        const uint64_t n_seg = (n + SEG - 1) / SEG;
        const uint64_t M = n_seg * BINS;
        const uint64_t want = (n_seg + WAVES - 1) / WAVES;
        const uint32_t g = (uint32_t)(want < (uint64_t)ncu * 8 ? want : (uint64_t)ncu * 8);
        // keys are < n_slots or NONE: sorting the low `bits` bits (2^bits > n_slots) groups the
        // slots and puts NONE (all ones) after every slot
        uint32_t bits = 1;
        while (bits < 32 && (1ull << bits) <= tb.n_slots) bits++;
        uint32_t *ka = sc.k0, *va = sc.v0, *kb = sc.k1, *vb = sc.v1;
        for (uint32_t shift = 0; shift < bits; shift += 8) {
            hipLaunchKernelGGL(nxg_radix_count_kernel, dim3(g), dim3(TPB), 0, s, ka, n, shift,
                               n_seg, sc.hist);
            if ((e = nxg_scan_u32(sc.hist, M, sc.off, sc.bsum, s)) != hipSuccess) return e;
            hipLaunchKernelGGL(nxg_radix_scatter_kernel, dim3(g), dim3(TPB), 0, s, ka, va, n, shift,
                               n_seg, sc.off, kb, vb);
            uint32_t* t = ka; ka = kb; kb = t;
            t = va; va = vb; vb = t;
        }
        hipLaunchKernelGGL(nxg_pub_prev_kernel, dim3(gi), dim3(TPB), 0, s, ka, va, n, sc.prev);
        prev = sc.prev;
    }
    hipLaunchKernelGGL(nxg_pub_mode_kernel, dim3(gi), dim3(TPB), 0, s, tb, in, prev, sc.mode,
                       sc.flags);
    *mode_out = sc.mode;
    return hipGetLastError();
}

// Stage 3 (after the host read flags[3]): the comparisons that need the stack walk
hipError_t nxg_launch_pub_deep(const NxgPubTable& tb, const NxgPubBatch& b, uint8_t* scratch,
                               const uint32_t* prev_used, int ncu, hipStream_t s) {
    PubScratch sc = pub_layout(scratch, b.n_rows, tb.n_slots);
    const PubIn in{b.id, b.kind, b.n_rows, {b.tag, b.fixed, b.aux, b.ctag, b.cfixed, b.caux, b.heap}};
    const uint64_t want = (b.n_rows + TPB - 1) / TPB;
    const uint32_t g = (uint32_t)(want < (uint64_t)ncu * 16 ? want : (uint64_t)ncu * 16);
    if (g)
        hipLaunchKernelGGL(nxg_pub_deep_kernel, dim3(g), dim3(TPB), 0, s, tb, in, prev_used,
                           sc.mode, sc.flags);
    return hipGetLastError();
}

const uint32_t* nxg_pub_prev(uint8_t* scratch, uint64_t n, uint64_t n_slots) {
    return pub_layout(scratch, n, n_slots).prev;
}
