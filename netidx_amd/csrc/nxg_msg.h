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
// Values are walked iteratively; the top level and the first container level live in registers.
// A value nested deeper than that is decoded again with an explicit stack that lives in LDS, one
// per wave (DMode.stk, kStk levels), by one lane of the wave at a time: no lane keeps a private
// stack, so no kernel needs scratch memory for it. Children are allocated depth-first, the same
// order as the recursive reference decoder, which produces them as it goes.
//
// Byte sources. A message whose bytes all lie in the wave's LDS image is decoded from LDS with
// unchecked reads, multi-byte fields read a word at a time (LdsSrc); any other message is
// decoded from global memory (GlbSrc). The choice is made once per message, after its length
// prefix, so the common path never waits on global memory and never branches per byte.
//
// Modes (DMode, a runtime value so that each kernel inlines ONE copy of the decoder per source):
//   kSpec     plausibility only (no UTF-8 scan), small work budget, minimal length varint and a
//             value that fills the message exactly: used to GUESS a start
//   kBounded  full validation with a work budget (E_BUDGET when exceeded): speculative walks,
//             which may start from a wrong position and must not wander through megabytes
//   kExact    full validation, unbounded: walks from positions known to be message starts
#pragma once
#include "nxg_device.h"

namespace nxgmsg {

constexpr uint32_t E_OK = 0, E_UNKNOWN_TAG = 1, E_TOO_BIG = 2, E_INVALID = 3, E_SHORT = 4,
                   E_DEPTH = 6, E_BUDGET = 100;  // E_BUDGET: gave up, not a decode error
constexpr uint64_t kMaxVec = 2ull * 1024 * 1024 * 1024;  // pack.rs:917
constexpr uint32_t kSpecBudget = 256;     // value headers per speculative decode
constexpr uint32_t kWalkBudget = 2048;    // work units per bounded walk (headers + 16 B of text)
struct DMode {
    uint32_t budget;  // work units before E_BUDGET (~0u: unbounded)
    uint32_t spec;    // plausibility mode (see above)
    uint32_t write;   // with EMIT: write the decoded values to the sink
};
constexpr DMode kSpec{kSpecBudget, 1, 0}, kBounded{kWalkBudget, 0, 0}, kExact{0xffffffffu, 0, 0};

// The explicit stack of a value nested two or more levels deep: kStk levels of (values left,
// next slot), in LDS, one per wave of the workgroup (a translation unit whose kernels run more
// than NXG_DV_WAVES waves per workgroup defines it before including this header). Only kernels
// that decode values allocate it.
constexpr int kStk = NXG_MAX_DEPTH + 2;
#ifndef NXG_DV_WAVES
#define NXG_DV_WAVES 4
#endif
typedef __attribute__((address_space(3))) uint64_t* lds_stk;
static __shared__ uint64_t nxg_dv_stk[NXG_DV_WAVES * 2 * kStk];
NXG_DEV lds_stk dv_stack() { return (lds_stk)(nxg_dv_stk + (threadIdx.x >> 6) * 2 * kStk); }
constexpr uint32_t E_DEEP = 101;  // (internal) the value needs the stack

typedef const __attribute__((address_space(3))) uint8_t* lds_bytes;
typedef const __attribute__((address_space(3))) uint32_t* lds_words;
typedef const __attribute__((address_space(1))) uint8_t* gbl_bytes;

// The frame as a wave sees it: bytes [t0, t0+nlds) are in the LDS image `lds` (which has at
// least 16 readable bytes past nlds), the whole frame [0, W) is at `g` in global memory.
struct Src {
    lds_bytes lds;
    uint64_t t0;
    uint32_t nlds;
    gbl_bytes g;
    uint64_t W;
    // a byte known to be inside the image
    NXG_DEV uint32_t img_byte(uint64_t p) const { return lds[(uint32_t)(p - t0)]; }
    // any byte of the frame (p < W)
    NXG_DEV uint32_t any_byte(uint64_t p) const {
        const uint64_t r = p - t0;
        if (r < nlds) return lds[(uint32_t)r];
        return g[p];
    }
};

// unchecked reads from the LDS image; word() reads up to 7 bytes past p
struct LdsSrc {
    lds_bytes lds;
    uint64_t t0;
    NXG_DEV uint32_t byte(uint64_t p) const { return lds[(uint32_t)(p - t0)]; }
    // bytes p..p+3, little-endian, any alignment
    NXG_DEV uint32_t word(uint64_t p) const {
        const uint32_t r = (uint32_t)(p - t0);
        lds_words w = (lds_words)(lds + (r & ~3u));
        return alignbyte(w[1], w[0], r & 3u);
    }
};
// reads from global memory (callers stay inside the frame)
struct GlbSrc {
    gbl_bytes g;
    NXG_DEV uint32_t byte(uint64_t p) const { return g[p]; }
    NXG_DEV uint32_t word(uint64_t p) const {
        return g[p] | ((uint32_t)g[p + 1] << 8) | ((uint32_t)g[p + 2] << 16) |
               ((uint32_t)g[p + 3] << 24);
    }
};

// 1 + payload size of the fixed-size value tags (pack.rs / value lib.rs:361-468), 4 bits per
// tag; 0 = variable size (varints, text, containers), not checked (Decimal) or unknown (>= 28)
constexpr uint64_t kFixLo = 0x1100DD9509090505ull;  // tags 0..15
constexpr uint64_t kFixHi = 0x0000033220000011ull;  // tags 16..27
NXG_DEV uint32_t fixed_size1(uint32_t t) {
    if (t >= 28u) return 0u;
    return (uint32_t)(((t < 16 ? kFixLo >> (4 * t) : kFixHi >> (4 * (t - 16)))) & 0xfu);
}

// Where a decoded value goes.
struct Sink {
    ColsDesc c;
    uint32_t* cap_flag;
    uint32_t* nonf64;  // F64-only columns (tag == nullptr) met a value they cannot hold
};

// LEB128 (pack.rs:504-520): at most 10 bytes, bits past 64 dropped, no minimality check.
// With 8 bytes available, one pair of word reads finds the terminator (ends in 1..8 bytes).
// A terminator in the first 4 bytes (almost every varint on this path) is decoded with 32-bit
// operations; 5..8 bytes with a 3-step 64-bit compress of the 7-bit groups.
template <class S>
NXG_DEV uint32_t dvar(const S& s, uint64_t& p, uint64_t lim, uint64_t& v) {
    if (lim > p && lim - p >= 4) {
        const uint32_t lo = s.word(p);
        const uint32_t st4 = ~lo & 0x80808080u;
        if (st4) {
            const uint32_t nb = ((uint32_t)__builtin_ctz(st4) >> 3) + 1;  // 1..4
            const uint32_t y = lo & (0xffffffffu >> (32u - 8u * nb));
            v = (y & 0x7fu) | ((y >> 1) & 0x3f80u) | ((y >> 2) & 0x1fc000u) | ((y >> 3) & 0xfe00000u);
            p += nb;
            return E_OK;
        }
        if (lim - p >= 8) {
            const uint64_t x = (uint64_t)lo | ((uint64_t)s.word(p + 4) << 32);
            const uint64_t stop = ~x & 0x8080808080808080ull;
            if (stop) {
                const uint32_t nb = ((uint32_t)__builtin_ctzll(stop) >> 3) + 1;  // 5..8
                const uint64_t y = nb == 8 ? x : (x & ((1ull << (8 * nb)) - 1));
                const uint64_t z1 = (y & 0x007f007f007f007full) | ((y >> 1) & 0x3f803f803f803f80ull);
                const uint64_t z2 = (z1 & 0x00003fff00003fffull) | ((z1 >> 2) & 0x0fffc0000fffc000ull);
                v = (z2 & 0x0fffffffull) | ((z2 >> 4) & 0x00fffffff0000000ull);
                p += nb;
                return E_OK;
            }
        }
    }
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

// big-endian fixed-width field of n = 1, 2, 4 or 8 bytes (bytes::Buf::get_*)
template <class S>
NXG_DEV uint32_t dfix(const S& s, uint64_t& p, uint64_t lim, uint32_t n, uint64_t& v) {
    if (lim - p < n) return E_SHORT;
    uint64_t x;
    if (n == 8) x = ((uint64_t)bswap32(s.word(p)) << 32) | bswap32(s.word(p + 4));
    else if (n == 4) x = bswap32(s.word(p));
    else if (n == 2) x = (s.byte(p) << 8) | s.byte(p + 1);
    else x = s.byte(p);
    p += n;
    v = x;
    return E_OK;
}

// std::str::from_utf8 (pack.rs:462): four ASCII bytes per step, the state machine otherwise
template <class S>
NXG_DEV bool utf8_ok(const S& s, uint64_t p, uint64_t n) {
    uint64_t i = 0;
#pragma unroll 1
    while (i < n) {
        if (i + 4 <= n && !(s.word(p + i) & 0x80808080u)) {
            i += 4;
            continue;
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

// wr == false: nothing is written (counting, or the values of control messages)
template <bool EMIT>
NXG_DEV void put(const Sink* k, bool wr, bool row, uint64_t slot, uint32_t tag, uint64_t fixed,
                 uint32_t aux) {
    if (!EMIT || !wr) return;
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
// kSpec). A bounded walk spends one work unit per 16 bytes of text.
template <class S>
NXG_DEV uint32_t dstr(const S& s, uint64_t& p, uint64_t lim, bool utf8, uint64_t& off,
                      uint64_t& len, uint32_t& work, const DMode& md) {
    uint64_t n;
    uint32_t e = dvar(s, p, lim, n);
    if (e) return e;
    if (n > lim - p) return E_TOO_BIG;
    if (utf8 && !md.spec) {
        if (md.budget != 0xffffffffu) {
            work += (uint32_t)min<uint64_t>(n >> 4, kWalkBudget);
            if (work > md.budget) return E_BUDGET;
        }
        if (!utf8_ok(s, p, n)) return E_INVALID;
    }
    off = p;
    len = n;
    p += n;
    return E_OK;
}

// Payload of one non-container value with wire tag t (the tag byte already consumed) into
// (row?, slot). Containers (19 Array, 21 Map, 22 Error(Value) whose inner is not a String) are
// handled by the caller. Tag 22 reaches here only as Error(String).
template <bool EMIT, class S>
NXG_DEV uint32_t dleaf(const S& s, uint32_t t, uint64_t& p, uint64_t lim, const Sink* k,
                       bool is_row, uint64_t cur, uint32_t& work, const DMode& md) {
    uint64_t v, v2, off, len;
    uint32_t e = E_OK;
    switch (t) {
    case 0:
        if (!(e = dfix(s, p, lim, 4, v))) put<EMIT>(k, md.write, is_row, cur, 0, v, 0);
        break;
    case 1:
        if (!(e = dvar(s, p, lim, v))) put<EMIT>(k, md.write, is_row, cur, 1, (uint32_t)v, 0);
        break;
    case 2:
        if (!(e = dfix(s, p, lim, 4, v)))
            put<EMIT>(k, md.write, is_row, cur, 2, (uint64_t)(int64_t)(int32_t)(uint32_t)v, 0);
        break;
    case 3:
        if (!(e = dvar(s, p, lim, v))) {
            const uint32_t n = (uint32_t)v;
            const int32_t r = (int32_t)(n >> 1) ^ (int32_t)(0u - (n & 1u));
            put<EMIT>(k, md.write, is_row, cur, 3, (uint64_t)(int64_t)r, 0);
        }
        break;
    case 4:
    case 6:
    case 9:
        if (!(e = dfix(s, p, lim, 8, v))) put<EMIT>(k, md.write, is_row, cur, t, v, 0);
        break;
    case 5:
        if (!(e = dvar(s, p, lim, v))) put<EMIT>(k, md.write, is_row, cur, 5, v, 0);
        break;
    case 7:
        if (!(e = dvar(s, p, lim, v)))
            put<EMIT>(k, md.write, is_row, cur, 7, (v >> 1) ^ (0ull - (v & 1ull)), 0);
        break;
    case 8:
        if (!(e = dfix(s, p, lim, 4, v))) put<EMIT>(k, md.write, is_row, cur, 8, v, 0);
        break;
    case 10:
        if ((e = dfix(s, p, lim, 8, v))) break;
        if ((e = dfix(s, p, lim, 4, v2))) break;
        if (!datetime_valid((int64_t)v, (uint32_t)v2)) {
            e = E_INVALID;
            break;
        }
        put<EMIT>(k, md.write, is_row, cur, 10, v, (uint32_t)v2);
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
        put<EMIT>(k, md.write, is_row, cur, 11, secs, ns);
        break;
    }
    case 12:
    case 18:
        if (!(e = dstr(s, p, lim, true, off, len, work, md)))
            put<EMIT>(k, md.write, is_row, cur, t, off, (uint32_t)len);
        break;
    case 13:
        if (!(e = dstr(s, p, lim, false, off, len, work, md)))
            put<EMIT>(k, md.write, is_row, cur, 13, off, (uint32_t)len);
        break;
    case 14:
        put<EMIT>(k, md.write, is_row, cur, 14, 1, 0);
        break;
    case 15:
        put<EMIT>(k, md.write, is_row, cur, 15, 0, 0);
        break;
    case 16:
    case 17:
        put<EMIT>(k, md.write, is_row, cur, 16, 0, 0);
        break;
    case 20:
        if (lim - p < 16) {
            e = E_SHORT;
            break;
        }
        put<EMIT>(k, md.write, is_row, cur, 20, p, 16);
        p += 16;
        break;
    case 22:  // Error(Value) whose inner value is a String: wire tag 18 in the columns
        p++;  // the inner String tag (12), checked by the caller
        if (!(e = dstr(s, p, lim, true, off, len, work, md)))
            put<EMIT>(k, md.write, is_row, cur, 18, off, (uint32_t)len);
        break;
    case 23:
        if (!(e = dfix(s, p, lim, 1, v))) put<EMIT>(k, md.write, is_row, cur, 23, v, 0);
        break;
    case 24:
        if (!(e = dfix(s, p, lim, 1, v)))
            put<EMIT>(k, md.write, is_row, cur, 24, (uint64_t)(int64_t)(int8_t)(uint8_t)v, 0);
        break;
    case 25:
        if (!(e = dfix(s, p, lim, 2, v))) put<EMIT>(k, md.write, is_row, cur, 25, v, 0);
        break;
    case 26:
        if (!(e = dfix(s, p, lim, 2, v)))
            put<EMIT>(k, md.write, is_row, cur, 26, (uint64_t)(int64_t)(int16_t)(uint16_t)v, 0);
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
        put<EMIT>(k, md.write, is_row, cur, 27, p, (uint32_t)(l2 - p));
        p = l2;
        break;
    }
    default:
        e = E_UNKNOWN_TAG;
    }
    return e;
}

// Does the value whose tag t was just consumed (next byte at p) contain other values?
template <class S>
NXG_DEV bool is_container(const S& s, uint32_t t, uint64_t p, uint64_t lim) {
    return t == 19 || t == 21 || (t == 22 && !(p < lim && s.byte(p) == 12u));
}

// Container header at p (tag t consumed): element count -> kids, and the container's own row.
template <bool EMIT, class S>
NXG_DEV uint32_t dcontainer(const S& s, uint32_t t, uint64_t& p, uint64_t lim, const Sink* k,
                            const DMode& md, bool is_row, uint64_t cur, uint64_t child_next,
                            uint64_t& kids) {
    if (t == 22) {
        kids = 1;
        put<EMIT>(k, md.write, is_row, cur, 22, child_next, 1);
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
    put<EMIT>(k, md.write, is_row, cur, t, child_next, (uint32_t)v);
    return E_OK;
}

// Decode one Value at p (limit lim) into (row?, slot); children are allocated from child_next,
// depth-first, the order in which the recursive reference decoder produces them. One leaf
// decoder serves every level. The top level and the first container level live in registers;
// only values nested two or more levels deep touch the stack arrays (scratch memory).
// STK false: a value that needs level 2 returns E_DEEP (dvalue then decodes it again with STK).
template <bool EMIT, bool STK, class S>
NXG_DEV uint32_t dvalue_impl(const S& s, uint64_t& p, uint64_t lim, const Sink* k, bool row,
                             uint64_t slot, uint64_t& child_next, uint32_t& work,
                             const DMode& md) {
    const lds_stk frem = STK ? dv_stack() : nullptr;  // levels >= 2: values left,
    const lds_stk fslot = frem + kStk;                 // next slot
    int top = -1;
    uint64_t left = 1, cur = slot;     // current level
    uint64_t sv_left = 0, sv_cur = 0;  // level 0 while level 1 is decoded
    int depth = 0;
    bool is_row = row;
#pragma unroll 1
    for (;;) {
        while (left == 0) {  // level finished: pop
            if (depth == 0) return E_OK;
            if (depth == 1) {
                left = sv_left;
                cur = sv_cur;
            } else {
                left = frem[top];
                cur = fslot[top];
                top--;
            }
            depth--;
        }
        if (depth > NXG_MAX_DEPTH) return E_DEPTH;
        if (++work > md.budget) return E_BUDGET;
        if (p >= lim) return E_SHORT;
        const uint32_t t = s.byte(p++);
        uint32_t e;
        if (is_container(s, t, p, lim)) {
            uint64_t kids;
            e = dcontainer<EMIT>(s, t, p, lim, k, md, is_row, cur, child_next, kids);
            if (e) return e;
            left--;
            cur++;
            is_row = false;
            if (kids) {
                if (depth == 0) {
                    sv_left = left;
                    sv_cur = cur;
                } else {
                    if (!STK) return E_DEEP;
                    ++top;
                    frem[top] = left;
                    fslot[top] = cur;
                }
                depth++;
                left = kids;
                cur = child_next;
                child_next += kids;
            }
            continue;
        }
        if ((e = dleaf<EMIT>(s, t, p, lim, k, is_row, cur, work, md))) return e;
        left--;
        cur++;
        is_row = false;
    }
}

// Decode one Value (see dvalue_impl): in registers when it nests at most one level, else again
// with the wave's LDS stack, one lane at a time (any lanes of the wave may be inactive here).
template <bool EMIT, class S>
NXG_DEV uint32_t dvalue(const S& s, uint64_t& p, uint64_t lim, const Sink* k, bool row,
                        uint64_t slot, uint64_t& child_next, uint32_t& work, const DMode& md) {
    const uint64_t p_in = p, cn_in = child_next;
    const uint32_t w_in = work;
    uint32_t e = dvalue_impl<EMIT, false>(s, p, lim, k, row, slot, child_next, work, md);
    one_lane_at_a_time(e == E_DEEP, [&] {
        p = p_in;
        child_next = cn_in;
        work = w_in;
        e = dvalue_impl<EMIT, true>(s, p, lim, k, row, slot, child_next, work, md);
    });
    return e;
}

struct MsgInfo {
    uint64_t next;
    uint32_t variant;
    uint64_t id;
};

// The message body after its length prefix: variant byte and fields, from source s.
template <bool EMIT, class S>
NXG_DEV uint32_t decode_body(const S& s, uint64_t p, uint64_t lim, MsgInfo& info, const Sink* k,
                             uint64_t row, uint64_t& child_next, uint32_t& work,
                             const DMode& md) {
    if (p >= lim) return E_SHORT;
    const uint32_t variant = s.byte(p++);
    info.variant = variant;
    uint64_t v, off, len;
    uint32_t e;
    bool upd = false, tail = false;
    switch (variant) {
    case 0:  // NoSuchValue(Path)
    case 1:  // Denied(Path)
        return dstr(s, p, lim, true, off, len, work, md);
    case 2:  // Unsubscribed(Id)
        return dvar(s, p, lim, v);
    case 3:  // Subscribed(Path, Id, Value)
        if ((e = dstr(s, p, lim, true, off, len, work, md))) return e;
        if ((e = dvar(s, p, lim, v))) return e;
        break;
    case 4:  // Update(Id, Value)
        if ((e = dvar(s, p, lim, v))) return e;
        info.id = v;
        upd = true;
        break;
    case 5:  // Heartbeat
        return E_OK;
    case 6:  // WriteResult(Id, Value, #[pack(default)] WriteId)
        if ((e = dvar(s, p, lim, v))) return e;
        tail = true;
        break;
    default:
        return E_UNKNOWN_TAG;
    }
    uint64_t cn = upd ? child_next : 0;
    const DMode mv{md.budget, md.spec, md.write && upd};
    e = dvalue<EMIT>(s, p, lim, k, upd, row, cn, work, mv);
    if (upd) child_next = cn;
    if (e) return e;
    if (upd && md.spec && p != lim) return E_INVALID;  // exact fit (see decode_msg)
    if (tail) {
        e = dvar(s, p, lim, v);
        return e == E_SHORT ? E_OK : e;  // #[pack(default)] WriteId (derive lib.rs:392-401)
    }
    return E_OK;
}

// Decode the message starting at `pos`. On success, info.next is the position after the
// length-wrapped region (trailing bytes skipped, pack.rs:551-553). Update values are written
// to row `row` (EMIT with md.write); their children are allocated from child_next. The values
// inside control messages (Subscribed, WriteResult) are validated, not written.
template <bool EMIT>
NXG_DEV uint32_t decode_msg(const Src& s, uint64_t pos, MsgInfo& info, const Sink* k,
                            uint64_t row, uint64_t& child_next, uint32_t& work, const DMode& md) {
    const LdsSrc ls{s.lds, s.t0};
    const GlbSrc gs{s.g};
    uint64_t p = pos, L;
    // the length prefix (<= 10 bytes) from the image when it lies there
    const bool img = pos >= s.t0 && pos - s.t0 + 10 <= s.nlds;
    uint32_t e = img ? dvar(ls, p, s.W, L) : dvar(gs, p, s.W, L);
    if (e) return e;
    if (L < 1) return E_SHORT;
    // a guess must look like encoder output: minimal length varint (and, below, content that
    // fills the length-wrapped region exactly). Otherwise a payload byte >= 0x80 just before a
    // true start makes a "shadow" message with a huge length and skipped trailing bytes.
    if (md.spec && p - pos != vl64(L)) return E_INVALID;
    const uint64_t take = L - vl64(L);
    const uint64_t lim = take < s.W - p ? p + take : s.W;
    info.next = lim;
    if (img && lim - s.t0 <= s.nlds)
        return decode_body<EMIT>(ls, p, lim, info, k, row, child_next, work, md);
    return decode_body<EMIT>(gs, p, lim, info, k, row, child_next, work, md);
}

// ---- structure only (the general decoder's count pass) ---------------------------------------
// Message boundaries depend only on the length prefixes (len_wrapped_decode, pack.rs:537-555),
// so the count pass reads just the prefix, the variant and, for an Update whose value is a
// container, the container structure (to count the child slots the emit pass will allocate).
// Content is not validated here: the emit pass decodes every message on the chain and reports
// the first content error. Only errors in the length prefix, which break the chain, are
// returned (and E_BUDGET from a bounded container walk).
template <class S>
NXG_DEV uint32_t skim_body(const S& s, uint64_t p, uint64_t lim, MsgInfo& info,
                           uint64_t& children, uint32_t& work, uint32_t budget) {
    const uint32_t variant = s.byte(p++);
    info.variant = variant;
    if (variant != 4) return E_OK;
    uint64_t v;
    if (dvar(s, p, lim, v) || p >= lim) return E_OK;  // content error: reported by emit
    const uint32_t t = s.byte(p);
    if (!is_container(s, t, p + 1, lim)) return E_OK;
    if (t == 19) {  // an array of fixed-size scalars: one child slot per element (as dvalue)
        uint64_t q = p + 1, cnt;
        if (!dvar(s, q, lim, cnt) && cnt <= kMaxVec / 16 && cnt * 16 <= ((lim - q) << 8)) {
            bool flat = true;
#pragma unroll 1
            for (uint64_t i = 0; flat && i < cnt; i++) {
                const uint32_t f1 = q < lim ? fixed_size1(s.byte(q)) : 0u;  // 1 + payload bytes
                flat = f1 != 0 && q + f1 <= lim;
                q += f1;
            }
            if (flat) {
                children = cnt;
                return E_OK;
            }
        }
    }
    uint64_t cn = 0;
    const DMode md{budget, 1, 0};  // structure: no UTF-8 scan, no writes
    const uint32_t e = dvalue<false>(s, p, lim, nullptr, true, 0, cn, work, md);
    children = cn;
    return e == E_BUDGET ? E_BUDGET : E_OK;
}

NXG_DEV uint32_t skim_msg(const Src& s, uint64_t pos, MsgInfo& info, uint64_t& children,
                          uint32_t& work, uint32_t budget) {
    const LdsSrc ls{s.lds, s.t0};
    const GlbSrc gs{s.g};
    uint64_t p = pos, L;
    const bool img = pos >= s.t0 && pos - s.t0 + 10 <= s.nlds;
    const uint32_t e = img ? dvar(ls, p, s.W, L) : dvar(gs, p, s.W, L);
    if (e) return e;
    if (L < 1) return E_SHORT;
    const uint64_t take = L - vl64(L);
    const uint64_t lim = take < s.W - p ? p + take : s.W;
    info.next = lim;
    info.variant = 0xff;  // no variant byte: a content error (BufferShort), reported by emit
    children = 0;
    if (p >= lim) return E_OK;
    if (img && lim - s.t0 <= s.nlds) return skim_body(ls, p, lim, info, children, work, budget);
    return skim_body(gs, p, lim, info, children, work, budget);
}

// the first-error key: the larger key is the earlier (offset, kind); 0 = no error
NXG_DEV uint64_t err_key(uint64_t off, uint32_t kind) { return ~((off << 8) | (kind & 0xffu)); }

}  // namespace nxgmsg
