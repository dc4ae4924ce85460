// nxg_encode_general.hip -- encode arbitrary columns (rows + children + control spans) to wire.
//
// Replaces handle_updates -> queue_send (netidx/src/publisher/server.rs:610-612,
// netidx/src/channel.rs:177-202). Each row becomes
//     varint(L) 04 varint(id) Value            L = lw(1 + vl(id) + |Value|)
// with Value::encode (netidx-value/src/lib.rs:361-468), ValArray (array.rs:583-593), Map
// (pack.rs:1212-1223) and Abstract (abstract_type.rs:272-278). Control messages (ctl) are
// copied verbatim from the heap and placed before row ctl_row[k], in order.
//
// Three launches:
// 1. ctl_scan: prefix of the control spans' lengths. One workgroup; skipped when there are no
//    control messages.
// 2. rows: each thread encodes GRPT consecutive rows. The launch does a block scan plus a
//    decoupled look-back over byte counts. Without control messages the tile's rows are
//    serialised into LDS at the output's 16-byte phase and leave as aligned nontemporal 16-byte
//    stores (plus byte stores for the two edge blocks), as nxg_encode_f64.hip. With control
//    messages, or when a tile's bytes exceed the staging, each row's position is its
//    rows-prefix plus the ctl bytes that precede it (binary search over ctl_row) and the row is
//    written straight to the output. Scalars, text and arrays of non-container elements are
//    sized and written without the explicit stack; Map, Error and nested containers take the
//    general walk.
// 3. ctl_write: copies each control span to its position.
//
// Archive mode (arch_base > 0, nxg_encode_archive_batch): the rows of an archive batch
// (<Vec<BatchItem> as Pack>::encode, pack.rs:941-952; BatchItem logfile/mod.rs:188-205): each row
// is varint(Id as u32) and its Event -- the byte 0x40 for Unsubscribed (tag 0x40), else the bare
// Value -- after the count varint the host writes at [0, arch_base). No length prefix, no variant.
#include "nxg_device.h"

#ifndef NXG_ENC_SKIP
#define NXG_ENC_SKIP 0  // timing experiments only
#endif
#ifndef NXG_ENC_EB
#define NXG_ENC_EB 4  // array elements loaded together (sizing and writing flat arrays)
#endif
#ifndef NXG_ENC_PF
#define NXG_ENC_PF 1  // the sizing and staging loops load their next entry's columns ahead
#endif
#ifndef NXG_ENC_KEEP
#define NXG_ENC_KEEP 1  // the thread's entries' columns loaded once, all together, and kept in
#endif                  // registers from the sizing pass to the staging pass (config 3 at 10^7:
                        // 0.2265 vs 0.2428 ms with the one-ahead loads of NXG_ENC_PF)
#ifndef NXG_ENC_CLS2
#define NXG_ENC_CLS2 1  // class buckets from per-wave ballot counts (no LDS atomics)
#endif
#ifndef NXG_ENC_LBU
#define NXG_ENC_LBU 1  // look-back window, 64 * NXG_ENC_LBU tiles per round trip (1, 4 and 8 measured equal)
#endif

#ifndef NXG_ENC_PROF
#define NXG_ENC_PROF 0
#endif
#if NXG_ENC_PROF
// diagnostic build only: per tile (the first 16384) s_memrealtime at the rows kernel's phase edges
// (start, classified, sized, scanned, staged, look-back done, stored)
__device__ unsigned long long nxg_enc_st[7][16384];
#define ESTAMP(k)                                                                                \
    do {                                                                                         \
        if (threadIdx.x == 0 && tile < 16384)                                                    \
            nxg_enc_st[k][tile] = __builtin_amdgcn_s_memrealtime();                              \
    } while (0)
#else
#define ESTAMP(k) \
    do {          \
    } while (0)
#endif

namespace {

constexpr int TPB = 256;
#ifndef NXG_ENC_GRPT
#define NXG_ENC_GRPT 4
#endif
#ifndef NXG_ENC_OCC
#define NXG_ENC_OCC 1  // waves per SIMD asked of the register allocator (launch bounds)
#endif
#ifndef NXG_ENC_BPR
#define NXG_ENC_BPR 28  // staging bytes per row
#endif
constexpr int GRPT = NXG_ENC_GRPT;       // rows per thread
constexpr int GTILE = TPB * GRPT;        // rows per tile
constexpr int GSTG = GTILE * NXG_ENC_BPR + 32;  // staging (config 3 averages 21.5 bytes per row)
constexpr uint64_t kMaxVec = 2ull * 1024 * 1024 * 1024;

struct Slot {
    uint32_t tag;
    uint64_t fixed;
    uint32_t aux;
};

NXG_DEV Slot get_slot(const ColsDesc& c, bool row, uint64_t i) {
    if (row) return Slot{c.tag[i], c.fixed[i], c.aux[i]};
    return Slot{c.ctag[i], c.cfixed[i], c.caux[i]};
}

NXG_DEV bool is_container(uint32_t tag) { return tag == 19 || tag == 21 || tag == 22; }

// |Value| of a non-container value (tags other than 19, 21, 22); 0 => unknown tag
NXG_DEV uint64_t scalar_len(const Slot& s) {
    switch (s.tag) {
    case 0: case 2: case 8: return 5;
    case 1: return 1 + vl64((uint32_t)s.fixed);
    case 3: return 1 + vl64(zz32((int32_t)(uint32_t)s.fixed));
    case 4: case 6: case 9: return 9;
    case 5: return 1 + vl64(s.fixed);
    case 7: return 1 + vl64(zz64((int64_t)s.fixed));
    case 10: case 11: return 13;
    case 12: case 13: case 18: return 1 + vl64(s.aux) + s.aux;
    case 14: case 15: case 16: return 1;
    case 20: return 17;
    case 23: case 24: return 2;
    case 25: case 26: return 3;
    case 27: return 1 + lwlen(s.aux);
    default: return 0;
    }
}

#ifndef NXG_ENC_AFAST
#define NXG_ENC_AFAST 1  // arrays of 1..8 fixed-size elements sized from one load of their tags (the same on the write side: no gain)
#endif
// |Value| of a value of fixed size by its tag (tag byte included; Decimal 17), 0 for the others:
// nibble tables, tag 20's 15 standing for 17
NXG_DEV uint32_t fixed_len(uint32_t t) {
    if (t < 16) return (uint32_t)(0x1100dd9509090505ull >> (4 * t)) & 15u;
    const uint32_t v = t < 28 ? (uint32_t)(0x332200f0001ull >> (4 * (t - 16))) & 15u : 0u;
    return v == 15u ? 17u : v;
}
// the tags of an array's 1..8 elements, ctag[p .. p + n), from the covering aligned dwords (a
// dword-aligned read never leaves the page of the bytes it covers); bytes past n zero
NXG_DEV uint64_t tags8(const uint8_t* p, uint32_t n) {
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3u);
    const uint32_t* w = reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3);
    const uint32_t nw = (sh + n + 3) >> 2;
    const uint32_t w0 = w[0], w1 = nw > 1 ? w[1] : 0u, w2 = nw > 2 ? w[2] : 0u;
    const uint64_t v = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) |
                       ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    return n >= 8 ? v : v & ((1ull << (8 * n)) - 1ull);
}

// The general walk's stack: kStk levels of (children left, next child slot), in LDS, one stack
// per wave (the walk runs one lane at a time: one_lane_at_a_time). Kept out of registers and
// scratch: a dynamically indexed private array would be scratch memory in every wave.
constexpr int kStk = NXG_MAX_DEPTH + 2;
struct WalkStack {
    uint64_t rem[kStk];
    uint64_t slot[kStk];
};

// |Value| for the value in (row?, slot), children included; 0 => error (*err set)
NXG_DEV uint64_t value_len(const ColsDesc& c, bool row, uint64_t slot, uint32_t* err,
                           WalkStack* stk) {
    uint64_t* frem = stk->rem;
    uint64_t* fslot = stk->slot;
    int top = -1, depth = 0;
    bool is_row = row;
    uint64_t cur = slot, total = 0;
    for (;;) {
        if (depth > NXG_MAX_DEPTH) {
            *err = 6;
            return 0;
        }
        const Slot s = get_slot(c, is_row, cur);
        uint64_t kids = 0;
        switch (s.tag) {
        case 0: case 2: case 8: total += 5; break;
        case 1: total += 1 + vl64((uint32_t)s.fixed); break;
        case 3: total += 1 + vl64(zz32((int32_t)(uint32_t)s.fixed)); break;
        case 4: case 6: case 9: total += 9; break;
        case 5: total += 1 + vl64(s.fixed); break;
        case 7: total += 1 + vl64(zz64((int64_t)s.fixed)); break;
        case 10: case 11: total += 13; break;
        case 12: case 13: case 18: total += 1 + vl64(s.aux) + s.aux; break;
        case 14: case 15: case 16: total += 1; break;
        case 19:
        case 21:
            if ((uint64_t)s.aux * (s.tag == 19 ? 16 : 32) > kMaxVec) {  // encode guard
                *err = 2;
                return 0;
            }
            total += 1 + vl64(s.aux);
            kids = s.tag == 19 ? s.aux : 2ull * s.aux;
            break;
        case 20: total += 17; break;
        case 22: total += 1; kids = 1; break;
        case 23: case 24: total += 2; break;
        case 25: case 26: total += 3; break;
        case 27: total += 1 + lwlen(s.aux); break;
        default:
            *err = 1;
            return 0;
        }
        if (kids) {
            ++top;
            frem[top] = kids;
            fslot[top] = s.fixed;
        }
        while (top >= 0 && frem[top] == 0) top--;
        if (top < 0) return total;
        frem[top]--;
        cur = fslot[top]++;
        is_row = false;
        depth = top + 1;
    }
}

struct Out {
    uint8_t* o;
    uint64_t p;
    NXG_DEV void b(uint32_t x) { o[p++] = (uint8_t)x; }
    NXG_DEV void be(uint64_t v, int n) {
        for (int i = n - 1; i >= 0; i--) o[p++] = (uint8_t)(v >> (8 * i));
    }
    NXG_DEV void var(uint64_t v) {
        while (v >= 0x80) {
            o[p++] = (uint8_t)((v & 0x7f) | 0x80);
            v >>= 7;
        }
        o[p++] = (uint8_t)v;
    }
    // Heap bytes (text, Decimal, Abstract payloads). Up to 44 bytes: the covering aligned dwords
    // are loaded together (no memory round trip per byte; a dword-aligned read never leaves the
    // page of the bytes it covers), realigned with alignbyte, then written byte by byte.
    NXG_DEV void copy(const uint8_t* src, uint64_t n) {
        constexpr int NW = 12;  // dwords loaded: covers 44 bytes at any alignment
        if (n <= 4 * NW - 4) {
            const uint32_t sh = (uint32_t)((uintptr_t)src & 3u);
            const uint32_t* w = reinterpret_cast<const uint32_t*>((uintptr_t)src & ~(uintptr_t)3);
            const uint32_t nw = (uint32_t)((sh + n + 3) >> 2);
            uint32_t d[NW + 1];
#pragma unroll
            for (int i = 0; i < NW; i++) d[i] = (uint32_t)i < nw ? w[i] : 0u;
            d[NW] = 0u;
#pragma unroll
            for (int i = 0; i < NW - 1; i++) {
                const uint32_t e = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
#pragma unroll
                for (int b = 0; b < 4; b++)
                    if ((uint64_t)(4 * i + b) < n) o[p + 4 * i + b] = (uint8_t)(e >> (8 * b));
            }
            p += n;
            return;
        }
        for (uint64_t i = 0; i < n; i++) o[p++] = src[i];
    }
};

template <typename W>
NXG_DEV void value_write(const ColsDesc& c, const uint8_t* heap, bool row, uint64_t slot, W& w,
                         WalkStack* stk) {
    uint64_t* frem = stk->rem;
    uint64_t* fslot = stk->slot;
    int top = -1;
    bool is_row = row;
    uint64_t cur = slot;
    for (;;) {
        const Slot s = get_slot(c, is_row, cur);
        uint64_t kids = 0;
        w.b(s.tag);
        switch (s.tag) {
        case 0: case 2: case 8: w.be(s.fixed, 4); break;
        case 1: w.var((uint32_t)s.fixed); break;
        case 3: w.var(zz32((int32_t)(uint32_t)s.fixed)); break;
        case 4: case 6: case 9: w.be(s.fixed, 8); break;
        case 5: w.var(s.fixed); break;
        case 7: w.var(zz64((int64_t)s.fixed)); break;
        case 10: case 11: w.be(s.fixed, 8); w.be(s.aux, 4); break;
        case 12: case 13: case 18: w.var(s.aux); w.copy(heap + s.fixed, s.aux); break;
        case 19: case 21:
            w.var(s.aux);
            kids = s.tag == 19 ? s.aux : 2ull * s.aux;
            break;
        case 20: w.copy(heap + s.fixed, 16); break;
        case 22: kids = 1; break;
        case 23: case 24: w.be(s.fixed, 1); break;
        case 25: case 26: w.be(s.fixed, 2); break;
        case 27: w.var(lwlen(s.aux)); w.copy(heap + s.fixed, s.aux); break;
        default: break;
        }
        if (kids) {
            ++top;
            frem[top] = kids;
            fslot[top] = s.fixed;
        }
        while (top >= 0 && frem[top] == 0) top--;
        if (top < 0) return;
        frem[top]--;
        cur = fslot[top]++;
        is_row = false;
    }
}

// Writes a non-container value (tag byte included).
template <typename W>
NXG_DEV void scalar_write(const Slot& s, const uint8_t* heap, W& w) {
    w.b(s.tag);
    switch (s.tag) {
    case 0: case 2: case 8: w.be(s.fixed, 4); break;
    case 1: w.var((uint32_t)s.fixed); break;
    case 3: w.var(zz32((int32_t)(uint32_t)s.fixed)); break;
    case 4: case 6: case 9: w.be(s.fixed, 8); break;
    case 5: w.var(s.fixed); break;
    case 7: w.var(zz64((int64_t)s.fixed)); break;
    case 10: case 11: w.be(s.fixed, 8); w.be(s.aux, 4); break;
    case 12: case 13: case 18: w.var(s.aux); w.copy(heap + s.fixed, s.aux); break;
    case 20: w.copy(heap + s.fixed, 16); break;
    case 23: case 24: w.be(s.fixed, 1); break;
    case 25: case 26: w.be(s.fixed, 2); break;
    case 27: w.var(lwlen(s.aux)); w.copy(heap + s.fixed, s.aux); break;
    default: break;
    }
}

// Row r's |Value| without the stack when the value is a scalar, text, or an array whose
// elements are not containers; `flat` false (and 0) otherwise, or on an unknown tag.
NXG_DEV uint64_t row_len_flat(const ColsDesc& c, const Slot& s, bool& flat) {
    flat = true;
    if (!is_container(s.tag)) {
        const uint64_t l = scalar_len(s);
        flat = l != 0;
        return l;
    }
    if (s.tag != 19 || (uint64_t)s.aux * 16 > kMaxVec) {
        flat = false;
        return 0;
    }
    if ((NXG_ENC_AFAST & 1) && s.aux - 1u < 8u) {  // 1..8 elements: their tags in one load
        const uint64_t tg = tags8(c.ctag + s.fixed, s.aux);
        uint32_t sum = 0;
        bool ok = true;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if ((uint32_t)j < s.aux) {
                const uint32_t f = fixed_len((uint32_t)(tg >> (8 * j)) & 0xffu);
                ok = ok && f != 0;
                sum += f;
            }
        }
        if (ok) return 2 + sum;  // tag 19, the count (one byte), the elements
    }
    uint64_t total = 1 + vl64(s.aux);
    // the elements NXG_ENC_EB at a time: their loads in flight together (one memory round trip
    // per group, not per element)
#pragma unroll 1
    for (uint64_t k0 = 0; k0 < s.aux; k0 += NXG_ENC_EB) {
        Slot e[NXG_ENC_EB];
#pragma unroll
        for (int j = 0; j < NXG_ENC_EB; j++)
            if (k0 + j < s.aux) e[j] = get_slot(c, false, s.fixed + k0 + j);
        bool ok = true;
#pragma unroll
        for (int j = 0; j < NXG_ENC_EB; j++) {
            if (k0 + j < s.aux) {
                const uint64_t l = is_container(e[j].tag) ? 0 : scalar_len(e[j]);
                ok = ok && l != 0;
                total += l;
            }
        }
        if (!ok) {
            flat = false;
            return 0;
        }
    }
    return total;
}
template <typename W>
NXG_DEV void row_write_flat(const ColsDesc& c, const uint8_t* heap, const Slot& s, W& w) {
    if (s.tag != 19) {
        scalar_write(s, heap, w);
        return;
    }
    w.b(19);
    w.var(s.aux);
#pragma unroll 1
    for (uint64_t k0 = 0; k0 < s.aux; k0 += NXG_ENC_EB) {
        Slot e[NXG_ENC_EB];
#pragma unroll
        for (int j = 0; j < NXG_ENC_EB; j++)
            if (k0 + j < s.aux) e[j] = get_slot(c, false, s.fixed + k0 + j);
#pragma unroll
        for (int j = 0; j < NXG_ENC_EB; j++)
            if (k0 + j < s.aux) scalar_write(e[j], heap, w);
    }
}

// Value classes by tag (CLS_GEN: Map, Error, nested containers and unknown tags, which take
// the stack walk), each sized and written by its own code so that a wave runs one class at a
// time.
enum : uint32_t { CLS_FIX8, CLS_TEXT, CLS_TIME, CLS_ARR, CLS_SCAL, CLS_GEN, NCLS };
NXG_DEV uint32_t value_class(uint32_t tag) {
    switch (tag) {
    case 4: case 6: case 9: return CLS_FIX8;
    case 12: case 13: case 18: return CLS_TEXT;
    case 10: case 11: return CLS_TIME;
    case 19: return CLS_ARR;  // CLS_GEN once sizing finds a container element
    case 21: case 22: return CLS_GEN;
    default: return tag < 28 ? CLS_SCAL : CLS_GEN;  // unknown tags: the walk reports them
    }
}

// number of ctl entries with ctl_row <= r (ctl_row is non-decreasing)
NXG_DEV uint64_t ctl_upto(const uint64_t* ctl_row, uint64_t n_ctl, uint64_t r) {
    uint64_t lo = 0, hi = n_ctl;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (ctl_row[mid] <= r) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Row r's message length exactly as the rows kernel sizes it (0 for a row whose value errs:
// that tile reports the error itself).
NXG_DEV uint64_t row_msg_len(const ColsDesc& c, uint64_t r, bool arch, WalkStack* stk) {
    const Slot v = get_slot(c, true, r);
    uint64_t vlen = 0;
    uint32_t err = 0;
    const uint32_t cl = arch && v.tag == 0x40u ? (uint32_t)CLS_SCAL : value_class(v.tag);
    bool gen = false;
    switch (cl) {
    case CLS_FIX8: vlen = 9; break;
    case CLS_TEXT: vlen = 1 + vl64(v.aux) + v.aux; break;
    case CLS_TIME: vlen = 13; break;
    case CLS_SCAL:
        vlen = arch && v.tag == 0x40u ? 1 : scalar_len(v);
        gen = !vlen;
        break;
    case CLS_ARR: {
        bool flat;
        vlen = row_len_flat(c, v, flat);
        gen = !flat;
        break;
    }
    default: gen = true; break;
    }
    one_lane_at_a_time(gen, [&] { vlen = value_len(c, true, r, &err, stk); });
    const uint64_t ml = err ? 0ull : arch ? vl64((uint32_t)c.id[r]) + vlen : lwlen(1 + vl64(c.id[r]) + vlen);
    if (!err && ml > (arch ? 0xFFFFFFFFull : 0x3FFFFFFFull)) return 0;
    return ml;
}

}  // namespace

// exclusive prefix of ctl_len into ctl_pre[0..n_ctl] (one workgroup)
__global__ __launch_bounds__(TPB) void nxg_enc_ctl_scan_kernel(ColsDesc c, uint64_t* ctl_pre) {
    __shared__ uint64_t tmp[4];
    uint64_t carry = 0;
    for (uint64_t b = 0; b < c.n_ctl; b += TPB) {
        const uint64_t i = b + threadIdx.x;
        const uint64_t v = i < c.n_ctl ? c.ctl_len[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan<uint64_t, TPB>(v, tmp, &tot);
        if (i < c.n_ctl) ctl_pre[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) ctl_pre[c.n_ctl] = carry;
}

__global__ __launch_bounds__(TPB, NXG_ENC_OCC) void nxg_enc_rows_kernel(
    ColsDesc c, const uint8_t* __restrict__ heap, uint8_t* __restrict__ out, uint64_t cap,
    const uint64_t* __restrict__ ctl_pre, uint64_t* __restrict__ row_off,
    uint64_t* __restrict__ tstat, uint32_t ntiles, uint32_t epoch, DevStatus* __restrict__ st,
    DevStatus* zst, uint64_t arch_base, uint32_t patience) {
    const bool arch = arch_base != 0;
    zero_status(zst);
    __shared__ uint64_t tmp[4];
    __shared__ uint64_t sh_base;
    __shared__ __attribute__((aligned(16))) uint8_t stg[GSTG];
    __shared__ uint32_t cls_n[NCLS], cls_b[NCLS + 1];
    __shared__ uint32_t cls_w[TPB / 64][NCLS];  // per wave: class counts, then first entries
    __shared__ uint16_t lst_row[GTILE];  // the tile's rows sorted by value class
    __shared__ uint16_t off_lds[GTILE];  // staging offset per row (tile-local index)
    __shared__ uint32_t len_lds[GTILE];  // message length per row (0: absent or erroring)
    __shared__ uint8_t cls_lds[GTILE];   // value class per row (CLS_GEN: the general walk)
    __shared__ WalkStack wstk[TPB / 64];  // the general walk's stack, one per wave
    static_assert(GSTG < 65536, "staging offsets fit 16 bits");
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    WalkStack* const stk = &wstk[tid >> 6];
    const uint64_t n = c.n_rows;
    // the tags of the thread's rows in its next tile, loaded during this tile's look-back
    uint32_t ntg[GRPT];
#pragma unroll
    for (int k = 0; k < GRPT; k++) {
        const uint64_t r = (uint64_t)blockIdx.x * GTILE + (uint64_t)tid * GRPT + k;
        ntg[k] = r < n ? c.tag[r] : 0u;
    }
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t rt = (uint64_t)tile * GTILE;
        const uint64_t r0 = rt + (uint64_t)tid * GRPT;
        ESTAMP(0);
        // 1. classify by tag and bucket the rows (wave-ballot counting sort in LDS); a wave then
        //    writes and sizes one class at a time
        uint32_t cls[GRPT], pos[GRPT];
#if NXG_ENC_CLS2
        // per wave: class counts and ranks from ballots alone (uniform counters, no LDS atomics),
        // then one table of the waves' offsets per class
        {
            uint32_t cnt[NCLS];
#pragma unroll
            for (int q = 0; q < NCLS; q++) cnt[q] = 0;
#pragma unroll
            for (int k = 0; k < GRPT; k++) {
                const uint64_t r = r0 + k;
                const uint32_t tg = NXG_ENC_PF ? ntg[k] : r < n ? c.tag[r] : 0u;
                cls[k] = r < n ? (arch && tg == 0x40u ? (uint32_t)CLS_SCAL : value_class(tg)) : NCLS;
                pos[k] = 0;
#pragma unroll
                for (uint32_t q = 0; q < NCLS; q++) {
                    const uint64_t m = __ballot(cls[k] == q);
                    if (cls[k] == q) pos[k] = cnt[q] + (uint32_t)__popcll(m & ((1ull << lane) - 1));
                    cnt[q] += (uint32_t)__popcll(m);
                }
            }
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < NCLS; q++) cls_w[tid >> 6][q] = cnt[q];
            }
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t acc = 0;
            for (int q = 0; q < NCLS; q++) {
                cls_b[q] = acc;
                for (int v = 0; v < TPB / 64; v++) {
                    const uint32_t x = cls_w[v][q];
                    cls_w[v][q] = acc;  // the wave's first entry of class q
                    acc += x;
                }
            }
            cls_b[NCLS] = acc;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < GRPT; k++) {
            const uint32_t rl = tid * GRPT + k;
            len_lds[rl] = 0;
            cls_lds[rl] = (uint8_t)cls[k];
            if (cls[k] < NCLS) lst_row[cls_w[tid >> 6][cls[k]] + pos[k]] = (uint16_t)rl;
        }
#else
        if (tid < NCLS) cls_n[tid] = 0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < GRPT; k++) {
            const uint64_t r = r0 + k;
            const uint32_t tg = NXG_ENC_PF ? ntg[k] : r < n ? c.tag[r] : 0u;
            cls[k] = r < n ? (arch && tg == 0x40u ? (uint32_t)CLS_SCAL : value_class(tg)) : NCLS;
            pos[k] = 0;
#pragma unroll
            for (uint32_t q = 0; q < NCLS; q++) {
                const uint64_t m = __ballot(cls[k] == q);
                if (!m) continue;
                const uint32_t lead = (uint32_t)__builtin_ctzll(m);
                uint32_t b0 = 0;
                if (lane == lead) b0 = atomicAdd(&cls_n[q], (uint32_t)__popcll(m));
                b0 = __shfl(b0, (int)lead);
                if (cls[k] == q) pos[k] = b0 + (uint32_t)__popcll(m & ((1ull << lane) - 1));
            }
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t acc = 0;
            for (int q = 0; q < NCLS; q++) {
                cls_b[q] = acc;
                acc += cls_n[q];
            }
            cls_b[NCLS] = acc;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < GRPT; k++) {
            const uint32_t rl = tid * GRPT + k;
            len_lds[rl] = 0;
            cls_lds[rl] = (uint8_t)cls[k];
            if (cls[k] < NCLS) lst_row[cls_b[cls[k]] + pos[k]] = (uint16_t)rl;
        }
#endif
        __syncthreads();
        ESTAMP(1);
        const uint32_t ne = cls_b[NCLS];
        // 2. message lengths, class by class. Each thread's next entry's slot and id are loaded
        //    while it sizes the current one (NXG_ENC_PF: two memory round trips in flight)
        auto size_one = [&](uint32_t rl, Slot v, uint64_t idv) {
            const uint64_t r = rt + rl;
            uint64_t vlen = 0;
            uint32_t err = 0;
            bool gen = false;
            switch (cls_lds[rl]) {
            case CLS_FIX8: vlen = 9; break;
            case CLS_TEXT: vlen = 1 + vl64(v.aux) + v.aux; break;
            case CLS_TIME: vlen = 13; break;
            case CLS_SCAL:
                vlen = arch && v.tag == 0x40u ? 1 : scalar_len(v);
                if (!vlen) {  // a tag the encoder does not write (17): the walk reports it
                    cls_lds[rl] = CLS_GEN;
                    gen = true;
                }
                break;
            case CLS_ARR: {
                bool flat;
                vlen = row_len_flat(c, v, flat);
                if (!flat) {
                    cls_lds[rl] = CLS_GEN;
                    gen = true;
                }
                break;
            }
            default: gen = true; break;
            }
            // Map, Error, nested containers: the general walk, one lane of the wave at a time
            one_lane_at_a_time(gen, [&] { vlen = value_len(c, true, r, &err, stk); });
            // queue_send refuses a message longer than MAX_BATCH (channel.rs:178-181); that bound
            // also keeps the 32-bit staged lengths exact
            const uint64_t ml = err    ? 0ull
                                : arch ? vl64((uint32_t)idv) + vlen
                                       : lwlen(1 + vl64(idv) + vlen);
            if (!err && ml > (arch ? 0xFFFFFFFFull : 0x3FFFFFFFull)) err = NXG_TOO_BIG;
            if (err) atomicMax(&st->err_kind, err);
            len_lds[rl] = err ? 0u : (uint32_t)ml;
        };
#if NXG_ENC_KEEP
        uint32_t k_rl[4];
        Slot k_v[4];
        uint64_t k_id[4];
#pragma unroll
        for (int j = 0; j < GRPT; j++) {
            const uint32_t e = tid + (uint32_t)j * TPB;
            k_rl[j] = e < ne ? lst_row[e] : 0u;
            k_v[j] = e < ne ? get_slot(c, true, rt + k_rl[j]) : Slot{0, 0, 0};
            k_id[j] = e < ne ? c.id[rt + k_rl[j]] : 0ull;
        }
        // (spelled out: a loop the compiler leaves rolled would index the arrays dynamically,
        // i.e. put them in scratch memory)
        static_assert(GRPT <= 4, "NXG_ENC_KEEP keeps at most 4 rows per thread");
#define NXG_KEEP_CALL(F, j) \
    if ((j) < GRPT && tid + (uint32_t)(j) * TPB < ne) F(k_rl[j], k_v[j], k_id[j])
        NXG_KEEP_CALL(size_one, 0);
        NXG_KEEP_CALL(size_one, 1);
        NXG_KEEP_CALL(size_one, 2);
        NXG_KEEP_CALL(size_one, 3);
#else
        {
            uint32_t p_rl = 0;
            Slot p_v{0, 0, 0};
            uint64_t p_id = 0;
            if (NXG_ENC_PF && tid < ne) {
                p_rl = lst_row[tid];
                p_v = get_slot(c, true, rt + p_rl);
                p_id = c.id[rt + p_rl];
            }
            for (uint32_t e = tid; e < ne; e += TPB) {
                const uint32_t rl = NXG_ENC_PF ? p_rl : lst_row[e];
                const Slot v = NXG_ENC_PF ? p_v : get_slot(c, true, rt + rl);
                const uint64_t idv = NXG_ENC_PF ? p_id : c.id[rt + rl];
                if (NXG_ENC_PF && e + TPB < ne) {
                    p_rl = lst_row[e + TPB];
                    p_v = get_slot(c, true, rt + p_rl);
                    p_id = c.id[rt + p_rl];
                }
                size_one(rl, v, idv);
            }
        }
#endif
        __syncthreads();
        ESTAMP(2);
        // 3. the tile's byte offsets: block scan, then look-back over the tiles' byte counts
        uint64_t L[GRPT];
        uint64_t mine = 0;
#pragma unroll
        for (int k = 0; k < GRPT; k++) {
            L[k] = len_lds[tid * GRPT + k];
            mine += L[k];
        }
        uint64_t tot;
        const uint64_t off = block_excl_scan<uint64_t, TPB>(mine, tmp, &tot);
        if (tid == 0) st_agent(&tstat[tile], lb_word(tile == 0 ? kFlagInc : kFlagAgg, epoch, tot));
        ESTAMP(3);
        // 4a. without control messages: the rows into the staging at their tile-local offsets
        //     first, so that the look-back below finds its predecessors mostly done
        // the tile's base (wave 0)
        auto lookback = [&]() {
            uint64_t base = 0;
            if (tile != 0) {
                bool give_up;
#if NXG_ENC_SKIP & 1
                give_up = false;  // timing experiments only: no look-back (wrong offsets)
#else
                // no wait on a workgroup that may not be running: an unpublished predecessor's
                // byte count is computed here from its rows (self-help)
                give_up = false;
                base = lookback_selfhelp_fn(
                    tstat, tile, epoch, patience, [&](uint64_t t) -> uint64_t {
                        const uint64_t q0 = t * GTILE;
                        uint64_t b = 0;
                        for (uint64_t r = q0 + lane; r < q0 + GTILE && r < n; r += 64)
                            b += row_msg_len(c, r, arch, &wstk[0]);
                        return wave_sum<uint64_t>(b);
                    });
#endif
                if (give_up && lane == 0) atomicOr(&st->timeout, 1u);
                if (lane == 0) st_agent(&tstat[tile], lb_word(kFlagInc, epoch, base + tot));
            }
            if (lane == 0) sh_base = base;
        };
        const bool stage = out && c.n_ctl == 0 && tot <= (uint64_t)(GSTG - 32);
        if (stage) {
            {
                uint32_t o = (uint32_t)off;
#pragma unroll
                for (int k = 0; k < GRPT; k++) {
                    off_lds[tid * GRPT + k] = (uint16_t)o;
                    o += (uint32_t)L[k];
                }
            }
            __syncthreads();
            auto stage_one = [&](uint32_t rl, Slot v, uint64_t idv) {
                const uint64_t r = rt + rl;
                const uint32_t len = len_lds[rl];
                if (!len) return;
                Out w{stg, off_lds[rl]};
                if (arch) {
                    w.var((uint32_t)idv);
                } else {
                    w.var(len);
                    w.b(4);
                    w.var(idv);
                }
                switch (cls_lds[rl]) {
                case CLS_FIX8:
                    w.b(v.tag);
                    w.be(v.fixed, 8);
                    break;
                case CLS_TEXT:
                    w.b(v.tag);
                    w.var(v.aux);
                    w.copy(heap + v.fixed, v.aux);
                    break;
                case CLS_TIME:
                    w.b(v.tag);
                    w.be(v.fixed, 8);
                    w.be(v.aux, 4);
                    break;
                case CLS_ARR: row_write_flat(c, heap, v, w); break;
                case CLS_SCAL: scalar_write(v, heap, w); break;
                default: break;
                }
                one_lane_at_a_time(cls_lds[rl] == CLS_GEN,
                                   [&] { value_write(c, heap, true, r, w, stk); });
            };
#if NXG_ENC_KEEP
            NXG_KEEP_CALL(stage_one, 0);
            NXG_KEEP_CALL(stage_one, 1);
            NXG_KEEP_CALL(stage_one, 2);
            NXG_KEEP_CALL(stage_one, 3);
#else
            const uint32_t e0 = tid, es = TPB;
            uint32_t q_rl = 0;
            Slot q_v{0, 0, 0};
            uint64_t q_id = 0;
            if (NXG_ENC_PF && e0 < ne) {
                q_rl = lst_row[e0];
                q_v = get_slot(c, true, rt + q_rl);
                q_id = c.id[rt + q_rl];
            }
            for (uint32_t e = e0; e < ne; e += es) {
                const uint32_t rl = NXG_ENC_PF ? q_rl : lst_row[e];
                const Slot v = NXG_ENC_PF ? q_v : get_slot(c, true, rt + rl);
                const uint64_t idv = NXG_ENC_PF ? q_id : c.id[rt + rl];
                if (NXG_ENC_PF && e + es < ne) {
                    q_rl = lst_row[e + es];
                    q_v = get_slot(c, true, rt + q_rl);
                    q_id = c.id[rt + q_rl];
                }
                stage_one(rl, v, idv);
            }
#endif
        }
        if (NXG_ENC_PF) {  // the next tile's tags: their round trip overlaps the look-back
            const uint64_t rn = (uint64_t)(tile + gridDim.x) * GTILE + (uint64_t)tid * GRPT;
#pragma unroll
            for (int k = 0; k < GRPT; k++) ntg[k] = rn + k < n ? c.tag[rn + k] : 0u;
        }
        // 3b. the tile's base: look-back over the tiles' byte counts (wave 0; running it while
        //     the other waves stage measured slower, 0.281 vs 0.245 ms)
        ESTAMP(4);
        if (tid < 64) lookback();
        __syncthreads();
        ESTAMP(5);
        const uint64_t tbase = sh_base + arch_base;
        if (stage && tbase + tot <= cap) {
            // 4b. the staging out as aligned nontemporal 16-byte stores: global block g holds the
            //     staged bytes from g - tbase; the two edge blocks (shared with the neighbours)
            //     by bytes
            if (!arch && tbase <= kMaxBatch && kMaxBatch < tbase + tot) {
                uint64_t o = tbase + off;
#pragma unroll
                for (int k = 0; k < GRPT; k++) {
                    const uint32_t lk = len_lds[tid * GRPT + k];
                    note_split(st, o, lk);
                    o += lk;
                }
            }
            const uint64_t end = tbase + tot;
            if (tot) {
                const uint64_t gb0 = tbase & ~15ull;
                const uint32_t phase = (uint32_t)(tbase & 15u);
                const uint32_t nblk = (uint32_t)((end - gb0 + 15) >> 4);
                typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
                for (uint32_t b = tid; b < nblk; b += TPB) {
                    const uint64_t g = gb0 + 16ull * b;
                    if (g >= tbase && g + 16 <= end) {
                        // local bytes [16 b - phase, + 16): five aligned dwords from LDS, realigned
                        const uint32_t ls = 16u * b - phase, a = ls >> 2, sb = ls & 3u;
                        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(stg);
                        const uint32_t e0 = s32[a], e1 = s32[a + 1], e2 = s32[a + 2], e3 = s32[a + 3],
                                       e4 = s32[a + 4];
                        u32x4v v;
                        v[0] = __builtin_amdgcn_alignbyte(e1, e0, sb);
                        v[1] = __builtin_amdgcn_alignbyte(e2, e1, sb);
                        v[2] = __builtin_amdgcn_alignbyte(e3, e2, sb);
                        v[3] = __builtin_amdgcn_alignbyte(e4, e3, sb);
                        __builtin_nontemporal_store(v, reinterpret_cast<u32x4v*>(out + g));
                    } else {
                        for (int k = 0; k < 16; k++)
                            if (g + k >= tbase && g + k < end) out[g + k] = stg[g + k - tbase];
                    }
                }
            }
        } else {
            // control messages interleaved, or more bytes than the staging: straight to the
            // frame, each thread its own rows
            uint64_t rpos = tbase + off;  // rows-only prefix
#pragma unroll 1  // (a large body with a lane-serial walk: not worth unrolling)
            for (int k = 0; k < GRPT; k++) {
                const uint64_t r = r0 + k;
                const uint64_t Lk = len_lds[tid * GRPT + k];
                if (r < n && row_off) row_off[r] = rpos;  // ctl placement needs every row's base
                if (r < n && Lk && out) {
                    uint64_t pos = rpos;
                    if (c.n_ctl) pos += ctl_pre[ctl_upto(c.ctl_row, c.n_ctl, r)];
                    if (!arch) note_split(st, pos, Lk);
                    if (pos + Lk > cap) {
                        atomicOr(&st->capacity, 1u);
                    } else {
                        Out w{out, pos};
                        if (arch) {
                            w.var((uint32_t)c.id[r]);
                        } else {
                            w.var(Lk);
                            w.b(4);
                            w.var(c.id[r]);
                        }
                        if (cls_lds[tid * GRPT + k] != CLS_GEN) row_write_flat(c, heap, get_slot(c, true, r), w);
                        one_lane_at_a_time(cls_lds[tid * GRPT + k] == CLS_GEN,
                                           [&] { value_write(c, heap, true, r, w, stk); });
                    }
                }
                rpos += Lk;
            }
        }
        if (tile == ntiles - 1 && tid == 0) {
            st->total_bytes = sh_base + tot + arch_base;  // rows (+ archive header); ctl: host
            st->n_rows = n;
        }
        ESTAMP(6);
        __syncthreads();
    }
}

__global__ __launch_bounds__(TPB) void nxg_enc_ctl_write_kernel(
    ColsDesc c, const uint8_t* __restrict__ heap, uint8_t* __restrict__ out, uint64_t cap,
    const uint64_t* __restrict__ ctl_pre, const uint64_t* __restrict__ row_off,
    const DevStatus* __restrict__ st, DevStatus* stw) {
    const uint64_t rows_total = st->total_bytes;
    for (uint64_t k = (uint64_t)blockIdx.x * TPB + threadIdx.x; k < c.n_ctl;
         k += (uint64_t)gridDim.x * TPB) {
        const uint64_t r = c.ctl_row[k];
        const uint64_t rb = r < c.n_rows ? row_off[r] : rows_total;
        const uint64_t pos = rb + ctl_pre[k];
        const uint64_t len = c.ctl_len[k];
        note_split(stw, pos, len);
        if (pos + len > cap) {
            atomicOr(&stw->capacity, 1u);
            continue;
        }
        const uint8_t* src = heap + c.ctl_off[k];
        for (uint64_t i = 0; i < len; i++) out[pos + i] = src[i];
    }
}

uint64_t nxg_enc_general_tiles(uint64_t n) { return (n + GTILE - 1) / GTILE; }

#if NXG_ENC_PROF
// diagnostic build only (not ABI): the stamps of the last general encode, 7 x 16384 u64
extern "C" int nxg_debug_enc_stamps(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(nxg_enc_st), sizeof(nxg_enc_st), 0,
                                    hipMemcpyDeviceToHost);
}
#endif

hipError_t nxg_launch_enc_general(const ColsDesc& cd, const uint8_t* heap, uint8_t* out,
                                  uint64_t cap, uint64_t* scratch, uint64_t* tstat,
                                  uint32_t epoch, DevStatus* st, int grid, hipStream_t s,
                                  uint64_t arch_base) {
    // scratch layout: ctl_pre[n_ctl + 1] | row_off[n_rows]  (only when n_ctl > 0)
    uint64_t* ctl_pre = scratch;
    uint64_t* row_off = cd.n_ctl ? scratch + cd.n_ctl + 1 : nullptr;
    if (cd.n_ctl) hipLaunchKernelGGL(nxg_enc_ctl_scan_kernel, dim3(1), dim3(TPB), 0, s, cd, ctl_pre);
    const uint64_t nt = nxg_enc_general_tiles(cd.n_rows);
    if (nt) {
        const uint64_t g = grid <= 0 ? nt : (nt < (uint64_t)grid ? nt : (uint64_t)grid);
        hipLaunchKernelGGL(nxg_enc_rows_kernel, dim3(g), dim3(TPB), 0, s, cd, heap, out, cap,
                           cd.n_ctl ? ctl_pre : nullptr, row_off, tstat, (uint32_t)nt, epoch, st, nxg_take_zero_slot(),
                           arch_base, nxg_patience);
    }
    if (cd.n_ctl && out) {
        const uint64_t nb = (cd.n_ctl + TPB - 1) / TPB;
        hipLaunchKernelGGL(nxg_enc_ctl_write_kernel, dim3((unsigned)(nb < 1024 ? nb : 1024)),
                           dim3(TPB), 0, s, cd, heap, out, cap, ctl_pre, row_off, st, st);
    }
    return hipGetLastError();
}

int nxg_occupancy_enc_general() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, nxg_enc_rows_kernel, TPB, 0) !=
        hipSuccess)
        return 1;
    return n;
}
