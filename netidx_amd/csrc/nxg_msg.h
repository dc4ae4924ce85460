// nxg_msg.h -- device-side decoder of one publisher::From message (general path).
//
// A per-lane restatement of:
//   len_wrapped_decode         netidx-core/src/pack.rs:537-555
//   derived enum decode        netidx-derive/src/lib.rs:482-601 (From, publisher.rs:73-96;
//                              #[pack(default)] WriteId per lib.rs:392-401)
//   Value::decode              netidx-value/src/lib.rs:470-506
//   ValArray / Map / PBytes / ArcStr / DateTime / Duration / Decimal / Abstract decoders
//                              array.rs:595-612, pack.rs:1225-1239, pbuf.rs:139-147,
//                              pack.rs:457-469, 1567-1575, 1591-1595, 614-622,
//                              abstract_type.rs:280-298
// A value is decoded without a stack when it is nested at most one level deep (dvalue_flat, the
// common case); deeper values are walked iteratively with an explicit stack (dvalue_deep).
// Children are allocated depth-first, the same order as the recursive reference decoder, which
// produces them as it goes.
//
// Modes:
//   M_SPEC    plausibility only (no UTF-8 scan), small work budget: used to GUESS a start
//   M_BOUNDED full validation with a work budget (E_BUDGET when exceeded): speculative walks,
//             which may start from a wrong position and must not wander through megabytes
//   M_EXACT   full validation, unbounded: walks from positions known to be message starts
#pragma once
#include "nxg_device.h"

namespace nxgmsg {

constexpr uint32_t E_OK = 0, E_UNKNOWN_TAG = 1, E_TOO_BIG = 2, E_INVALID = 3, E_SHORT = 4,
                   E_DEPTH = 6, E_BUDGET = 100;  // E_BUDGET: gave up, not a decode error
constexpr uint64_t kMaxVec = 2ull * 1024 * 1024 * 1024;  // pack.rs:917
enum Mode { M_SPEC = 0, M_BOUNDED = 1, M_EXACT = 2 };
constexpr uint32_t kSpecBudget = 256;     // value headers per speculative decode
constexpr uint32_t kWalkBudget = 2048;    // work units per bounded walk (headers + 16 B of text)

// Bytes of the frame: [t0, t0+nlds) come from LDS, everything else from global memory.
struct Src {
    const uint8_t* lds;
    uint64_t t0;
    uint32_t nlds;
    const uint8_t* __restrict__ g;
    uint64_t W;
    NXG_DEV uint32_t byte(uint64_t p) const {
        const uint64_t r = p - t0;
        return r < nlds ? (uint32_t)lds[r] : (uint32_t)g[p];
    }
};

// std::str::from_utf8 (pack.rs:462) over a Src: four ASCII bytes per step while the text lies
// in the LDS image, the byte-wise state machine (nxg_device.h utf8_valid) otherwise.
NXG_DEV bool utf8_valid_src(const Src& s, uint64_t p, uint64_t n) {
    uint64_t i = 0;
    const uint64_t r0 = p - s.t0;
#pragma unroll 1
    while (i < n) {
        const uint64_t r = r0 + i;
        if (i + 4 <= n && r + 8 <= s.nlds) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(s.lds + (r & ~3ull));
            const uint32_t x = alignbyte(w[1], w[0], (uint32_t)(r & 3));
            if (!(x & 0x80808080u)) {
                i += 4;
                continue;
            }
        }
        const uint32_t c = s.byte(p + i);
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
        const uint32_t c1 = s.byte(p + i + 1);
        if (c1 < lo || c1 > hi) return false;
        for (uint32_t k = 2; k <= need; k++)
            if ((s.byte(p + i + k) & 0xC0) != 0x80) return false;
        i += need + 1;
    }
    return true;
}

// Where a decoded value goes. EMIT=false only counts children.
struct Sink {
    ColsDesc c;
    uint32_t* cap_flag;
    uint32_t* nonf64;  // F64-only columns (tag == nullptr) met a value they cannot hold
};

NXG_DEV uint32_t dvar(const Src& s, uint64_t& p, uint64_t lim, uint64_t& v) {
    uint64_t val = 0;
#pragma unroll 1
    for (uint32_t i = 0; i < 10; i++) {
        if (p + i >= lim) return E_SHORT;
        const uint32_t b = s.byte(p + i);
        val |= (uint64_t)(b & 0x7fu) << (7 * i);
        if (b < 0x80u) {
            p += i + 1;
            v = val;
            return E_OK;
        }
    }
    return E_INVALID;
}

NXG_DEV uint32_t dfix(const Src& s, uint64_t& p, uint64_t lim, uint32_t n, uint64_t& v) {
    if (lim - p < n) return E_SHORT;
    uint64_t x = 0;
    for (uint32_t i = 0; i < n; i++) x = (x << 8) | s.byte(p + i);
    p += n;
    v = x;
    return E_OK;
}

template <bool EMIT>
NXG_DEV void put(const Sink* k, bool row, uint64_t slot, uint32_t tag, uint64_t fixed, uint32_t aux) {
    if (!EMIT) return;
    if (row) {
        if (!k->c.tag) {  // F64-only columns
            if (tag != 9) atomicOr(k->nonf64, 1u);
            else if (slot < k->c.cap_rows) k->c.fixed[slot] = fixed;
        } else if (slot < k->c.cap_rows) {
            k->c.tag[slot] = (uint8_t)tag;
            k->c.fixed[slot] = fixed;
            k->c.aux[slot] = aux;
        }
    } else {
        if (!k->c.ctag) {
            atomicOr(k->nonf64, 1u);
        } else if (slot < k->c.cap_children) {
            k->c.ctag[slot] = (uint8_t)tag;
            k->c.cfixed[slot] = fixed;
            k->c.caux[slot] = aux;
        } else {
            atomicOr(k->cap_flag, 1u);
        }
    }
}

// string/bytes payload: varint len; TooBig if len > remaining; UTF-8 for strings (not in
// M_SPEC). In M_BOUNDED a long text spends work, one unit per 16 bytes.
template <int MODE>
NXG_DEV uint32_t dstr(const Src& s, uint64_t& p, uint64_t lim, bool utf8, uint64_t& off,
                      uint64_t& len, uint32_t& work) {
    uint64_t n;
    uint32_t e = dvar(s, p, lim, n);
    if (e) return e;
    if (n > lim - p) return E_TOO_BIG;
    if (utf8 && MODE != M_SPEC) {
        if (MODE == M_BOUNDED) {
            work += (uint32_t)min<uint64_t>(n >> 4, kWalkBudget);
            if (work > kWalkBudget) return E_BUDGET;
        }
        if (!utf8_valid_src(s, p, n)) return E_INVALID;
    }
    off = p;
    len = n;
    p += n;
    return E_OK;
}

// Payload of one non-container value with wire tag t (the tag byte already consumed) into
// (row?, slot). Containers (19 Array, 21 Map, 22 Error(Value) whose inner is not a String) are
// handled by the callers. Tag 22 reaches here only as Error(String).
template <bool EMIT, int MODE>
NXG_DEV uint32_t dleaf(const Src& s, uint32_t t, uint64_t& p, uint64_t lim, const Sink* k,
                       bool is_row, uint64_t cur, uint32_t& work) {
    uint64_t v, v2, off, len;
    uint32_t e = E_OK;
    switch (t) {
    case 0:
        if (!(e = dfix(s, p, lim, 4, v))) put<EMIT>(k, is_row, cur, 0, v, 0);
        break;
    case 1:
        if (!(e = dvar(s, p, lim, v))) put<EMIT>(k, is_row, cur, 1, (uint32_t)v, 0);
        break;
    case 2:
        if (!(e = dfix(s, p, lim, 4, v)))
            put<EMIT>(k, is_row, cur, 2, (uint64_t)(int64_t)(int32_t)(uint32_t)v, 0);
        break;
    case 3:
        if (!(e = dvar(s, p, lim, v))) {
            const uint32_t n = (uint32_t)v;
            const int32_t r = (int32_t)(n >> 1) ^ (int32_t)(0u - (n & 1u));
            put<EMIT>(k, is_row, cur, 3, (uint64_t)(int64_t)r, 0);
        }
        break;
    case 4:
    case 6:
    case 9:
        if (!(e = dfix(s, p, lim, 8, v))) put<EMIT>(k, is_row, cur, t, v, 0);
        break;
    case 5:
        if (!(e = dvar(s, p, lim, v))) put<EMIT>(k, is_row, cur, 5, v, 0);
        break;
    case 7:
        if (!(e = dvar(s, p, lim, v)))
            put<EMIT>(k, is_row, cur, 7, (v >> 1) ^ (0ull - (v & 1ull)), 0);
        break;
    case 8:
        if (!(e = dfix(s, p, lim, 4, v))) put<EMIT>(k, is_row, cur, 8, v, 0);
        break;
    case 10:
        if ((e = dfix(s, p, lim, 8, v))) break;
        if ((e = dfix(s, p, lim, 4, v2))) break;
        if (!datetime_valid((int64_t)v, (uint32_t)v2)) {
            e = E_INVALID;
            break;
        }
        put<EMIT>(k, is_row, cur, 10, v, (uint32_t)v2);
        break;
    case 11: {
        if ((e = dfix(s, p, lim, 8, v))) break;
        if ((e = dfix(s, p, lim, 4, v2))) break;
        uint64_t secs = v;
        uint32_t ns = (uint32_t)v2;
        if (ns >= 1000000000u) {
            const uint64_t add = ns / 1000000000u;
            if (secs + add < secs) {
                e = E_INVALID;  // Duration::new overflow panics in the reference
                break;
            }
            secs += add;
            ns %= 1000000000u;
        }
        put<EMIT>(k, is_row, cur, 11, secs, ns);
        break;
    }
    case 12:
    case 18:
        if (!(e = dstr<MODE>(s, p, lim, true, off, len, work)))
            put<EMIT>(k, is_row, cur, t, off, (uint32_t)len);
        break;
    case 13:
        if (!(e = dstr<MODE>(s, p, lim, false, off, len, work)))
            put<EMIT>(k, is_row, cur, 13, off, (uint32_t)len);
        break;
    case 14:
        put<EMIT>(k, is_row, cur, 14, 1, 0);
        break;
    case 15:
        put<EMIT>(k, is_row, cur, 15, 0, 0);
        break;
    case 16:
    case 17:
        put<EMIT>(k, is_row, cur, 16, 0, 0);
        break;
    case 20:
        if (lim - p < 16) {
            e = E_SHORT;
            break;
        }
        put<EMIT>(k, is_row, cur, 20, p, 16);
        p += 16;
        break;
    case 22:  // Error(Value) whose inner value is a String: wire tag 18 in the columns
        p++;  // the inner String tag (12), checked by the caller
        if (!(e = dstr<MODE>(s, p, lim, true, off, len, work)))
            put<EMIT>(k, is_row, cur, 18, off, (uint32_t)len);
        break;
    case 23:
        if (!(e = dfix(s, p, lim, 1, v))) put<EMIT>(k, is_row, cur, 23, v, 0);
        break;
    case 24:
        if (!(e = dfix(s, p, lim, 1, v)))
            put<EMIT>(k, is_row, cur, 24, (uint64_t)(int64_t)(int8_t)(uint8_t)v, 0);
        break;
    case 25:
        if (!(e = dfix(s, p, lim, 2, v))) put<EMIT>(k, is_row, cur, 25, v, 0);
        break;
    case 26:
        if (!(e = dfix(s, p, lim, 2, v)))
            put<EMIT>(k, is_row, cur, 26, (uint64_t)(int64_t)(int16_t)(uint16_t)v, 0);
        break;
    case 27: {
        if ((e = dvar(s, p, lim, v))) break;
        if (v < 1) {
            e = E_SHORT;
            break;
        }
        const uint64_t take = v - vl64(v);
        const uint64_t l2 = take < lim - p ? p + take : lim;
        if (l2 - p < 16) {
            e = E_SHORT;
            break;
        }
        put<EMIT>(k, is_row, cur, 27, p, (uint32_t)(l2 - p));
        p = l2;
        break;
    }
    default:
        e = E_UNKNOWN_TAG;
    }
    return e;
}

// Does the value whose tag t was just consumed (next byte at p) contain other values?
NXG_DEV bool is_container(const Src& s, uint32_t t, uint64_t p, uint64_t lim) {
    return t == 19 || t == 21 || (t == 22 && !(p < lim && s.byte(p) == 12u));
}

// Container header at p (tag t consumed): element count -> kids, and the container's own row.
template <bool EMIT>
NXG_DEV uint32_t dcontainer(const Src& s, uint32_t t, uint64_t& p, uint64_t lim, const Sink* k,
                            bool is_row, uint64_t cur, uint64_t child_next, uint64_t& kids) {
    if (t == 22) {
        kids = 1;
        put<EMIT>(k, is_row, cur, 22, child_next, 1);
        return E_OK;
    }
    uint64_t v;
    const uint32_t e = dvar(s, p, lim, v);
    if (e) return e;
    // ValArray / Map guards: array.rs:600-603 (16 B per element), pack.rs:1228-1231 (32 B)
    const uint64_t maxe = t == 19 ? (kMaxVec / 16) : (kMaxVec / 32);
    const uint64_t unit = t == 19 ? 16 : 32;
    if (v > maxe || v * unit > ((lim - p) << 8)) return E_TOO_BIG;
    kids = t == 19 ? v : 2 * v;
    put<EMIT>(k, is_row, cur, t, child_next, (uint32_t)v);
    return E_OK;
}

constexpr uint32_t E_NESTED = 101;  // internal: flat decoder met a nested container

// One Value at p, for values nested at most one level deep (a container of leaves): no stack,
// so nothing spills to scratch. A deeper value returns E_NESTED (after the same checks the
// general decoder would have made up to that point), and the caller re-decodes it with dvalue.
template <bool EMIT, int MODE>
NXG_DEV uint32_t dvalue_flat(const Src& s, uint64_t& p, uint64_t lim, const Sink* k, bool row,
                             uint64_t slot, uint64_t& child_next, uint32_t& work) {
    if (MODE == M_SPEC && ++work > kSpecBudget) return E_BUDGET;
    if (MODE == M_BOUNDED && ++work > kWalkBudget) return E_BUDGET;
    if (p >= lim) return E_SHORT;
    const uint32_t t = s.byte(p++);
    if (!is_container(s, t, p, lim)) return dleaf<EMIT, MODE>(s, t, p, lim, k, row, slot, work);
    uint64_t kids;
    uint32_t e = dcontainer<EMIT>(s, t, p, lim, k, row, slot, child_next, kids);
    if (e) return e;
    const uint64_t base = child_next;
    child_next += kids;
#pragma unroll 1
    for (uint64_t i = 0; i < kids; i++) {
        if (MODE == M_SPEC && ++work > kSpecBudget) return E_BUDGET;
        if (MODE == M_BOUNDED && ++work > kWalkBudget) return E_BUDGET;
        if (p >= lim) return E_SHORT;
        const uint32_t t2 = s.byte(p++);
        if (is_container(s, t2, p, lim)) return E_NESTED;
        if ((e = dleaf<EMIT, MODE>(s, t2, p, lim, k, false, base + i, work))) return e;
    }
    return E_OK;
}

// Any Value at p: iterative depth-first walk with an explicit stack (scratch memory), used only
// for values nested deeper than dvalue_flat handles. Children are allocated depth-first, the
// order in which the recursive reference decoder produces them.
template <bool EMIT, int MODE>
__device__ __attribute__((noinline)) uint32_t dvalue_deep(const Src& s, uint64_t& p, uint64_t lim,
                                                          const Sink* k, bool row, uint64_t slot,
                                                          uint64_t& child_next, uint32_t& work) {
    uint64_t frem[NXG_MAX_DEPTH + 2];
    uint64_t fslot[NXG_MAX_DEPTH + 2];
    int top = -1;
    int depth = 0;
    bool is_row = row;
    uint64_t cur = slot;
#pragma unroll 1
    for (;;) {
        if (depth > NXG_MAX_DEPTH) return E_DEPTH;
        if (MODE == M_SPEC && ++work > kSpecBudget) return E_BUDGET;
        if (MODE == M_BOUNDED && ++work > kWalkBudget) return E_BUDGET;
        if (p >= lim) return E_SHORT;
        const uint32_t t = s.byte(p++);
        uint32_t e;
        uint64_t kids = 0;
        if (is_container(s, t, p, lim)) e = dcontainer<EMIT>(s, t, p, lim, k, is_row, cur, child_next, kids);
        else e = dleaf<EMIT, MODE>(s, t, p, lim, k, is_row, cur, work);
        if (e) return e;
        if (kids) {
            const uint64_t base = child_next;
            child_next += kids;
            ++top;
            frem[top] = kids;
            fslot[top] = base;
        }
        while (top >= 0 && frem[top] == 0) top--;
        if (top < 0) return E_OK;
        frem[top]--;
        cur = fslot[top]++;
        is_row = false;
        depth = top + 1;
    }
}

// Decode one Value at p (limit lim) into (row?, slot), children from `child_next`.
template <bool EMIT, int MODE>
NXG_DEV uint32_t dvalue(const Src& s, uint64_t& p, uint64_t lim, const Sink* k, bool row,
                        uint64_t slot, uint64_t& child_next, uint32_t& work) {
    const uint64_t p0 = p, c0 = child_next;
    const uint32_t w0 = work;
    const uint32_t e = dvalue_flat<EMIT, MODE>(s, p, lim, k, row, slot, child_next, work);
    if (e != E_NESTED) return e;
    p = p0;
    child_next = c0;
    work = w0;
    return dvalue_deep<EMIT, MODE>(s, p, lim, k, row, slot, child_next, work);
}

struct MsgInfo {
    uint64_t next;
    uint32_t variant;
    uint64_t id;
};

// Decode the message starting at `pos`. On success, info.next is the position after the
// length-wrapped region (trailing bytes skipped, pack.rs:551-553). Update values are written
// to row `row` (EMIT); children are allocated from child_next.
template <bool EMIT, int MODE>
NXG_DEV uint32_t decode_msg(const Src& s, uint64_t pos, MsgInfo& info, const Sink* k,
                            uint64_t row, uint64_t& child_next, uint32_t& work) {
    uint64_t p = pos, L;
    uint32_t e = dvar(s, p, s.W, L);
    if (e) return e;
    if (L < 1) return E_SHORT;
    // a guess must look like encoder output: minimal length varint (and, below, content that
    // fills the length-wrapped region exactly). Otherwise a payload byte >= 0x80 just before a
    // true start makes a "shadow" message with a huge length and skipped trailing bytes.
    if (MODE == M_SPEC && p - pos != vl64(L)) return E_INVALID;
    const uint64_t take = L - vl64(L);
    const uint64_t lim = take < s.W - p ? p + take : s.W;
    info.next = lim;
    if (p >= lim) return E_SHORT;
    const uint32_t variant = s.byte(p++);
    info.variant = variant;
    uint64_t v, off, len, dummy = 0;
    switch (variant) {
    case 0:
    case 1:
        return dstr<MODE>(s, p, lim, true, off, len, work);
    case 2:
        return dvar(s, p, lim, v);
    case 3:
        if ((e = dstr<MODE>(s, p, lim, true, off, len, work))) return e;
        if ((e = dvar(s, p, lim, v))) return e;
        return dvalue<false, MODE>(s, p, lim, k, false, 0, dummy, work);
    case 4:
        if ((e = dvar(s, p, lim, v))) return e;
        info.id = v;
        e = dvalue<EMIT, MODE>(s, p, lim, k, true, row, child_next, work);
        if (MODE == M_SPEC && !e && p != lim) return E_INVALID;  // exact fit (see above)
        return e;
    case 5:
        return E_OK;
    case 6:
        if ((e = dvar(s, p, lim, v))) return e;
        if ((e = dvalue<false, MODE>(s, p, lim, k, false, 0, dummy, work))) return e;
        e = dvar(s, p, lim, v);
        return e == E_SHORT ? E_OK : e;  // #[pack(default)] WriteId
    default:
        return E_UNKNOWN_TAG;
    }
}

}  // namespace nxgmsg
