// nxg_wire.h -- host-side builders and readers of netidx's packed wire format, for the control
// messages the library speaks on the host (sessions, the resolver): varints (pack.rs:472-520),
// length wrapping (pack.rs:522-555), big-endian fixed-width fields, and the derived enum/struct
// layout (netidx-derive/src/lib.rs:143-601: a length-wrapped body, enums led by a u8 variant).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace nxgwire {

inline uint32_t vlen(uint64_t v) {
    uint32_t n = 1;
    while (v >= 0x80) {
        v >>= 7;
        n++;
    }
    return n;
}
inline uint64_t lwlen(uint64_t n) { return n + vlen(n + vlen(n)); }  // pack.rs:522-525

struct Out {
    std::vector<uint8_t> b;
    void u8(uint32_t x) { b.push_back((uint8_t)x); }
    void be(uint64_t v, int n) {
        for (int i = n - 1; i >= 0; i--) b.push_back((uint8_t)(v >> (8 * i)));
    }
    void var(uint64_t v) {
        while (v >= 0x80) {
            b.push_back((uint8_t)((v & 0x7f) | 0x80));
            v >>= 7;
        }
        b.push_back((uint8_t)v);
    }
    void bytes(const void* p, size_t n) {
        const uint8_t* q = static_cast<const uint8_t*>(p);
        b.insert(b.end(), q, q + n);
    }
};

// a derived enum message: varint(lw(1 + fields)) variant fields (netidx-derive lib.rs:289-381)
inline std::vector<uint8_t> wrap(uint32_t variant, const std::vector<uint8_t>& fields) {
    Out o;
    o.var(lwlen(1 + fields.size()));
    o.u8(variant);
    o.bytes(fields.data(), fields.size());
    return o.b;
}

// a derived struct (length-wrapped fields, derive lib.rs:228-257)
inline std::vector<uint8_t> wrap_struct(const std::vector<uint8_t>& fields) {
    Out o;
    o.var(lwlen(fields.size()));
    o.bytes(fields.data(), fields.size());
    return o.b;
}

// A bounds-checked reader over one message; every get fails (returns false) past the end, as
// Buf::remaining checks do (PackError::BufferShort).
struct In {
    const uint8_t* p;
    size_t n, i = 0;
    In(const uint8_t* p_, size_t n_) : p(p_), n(n_) {}
    size_t left() const { return n - i; }
    bool u8(uint32_t& x) {
        if (i >= n) return false;
        x = p[i++];
        return true;
    }
    bool be(uint64_t& v, int k) {
        if (left() < (size_t)k) return false;
        v = 0;
        for (int j = 0; j < k; j++) v = (v << 8) | p[i++];
        return true;
    }
    bool var(uint64_t& v) {  // decode_varint (pack.rs:504-520)
        v = 0;
        for (int k = 0; k < 10; k++) {
            if (i >= n) return false;
            const uint8_t b = p[i++];
            if (k < 10) v |= (uint64_t)(b & 0x7f) << (7 * k);
            if (b < 0x80) return true;
        }
        return false;
    }
    bool str(std::string& s) {
        uint64_t L;
        if (!var(L) || L > left()) return false;
        s.assign(reinterpret_cast<const char*>(p + i), (size_t)L);
        i += (size_t)L;
        return true;
    }
    // a length-wrapped region: [i, end) after the prefix (len_wrapped_decode, pack.rs:537-555)
    bool wrapped(size_t& end) {
        uint64_t L;
        if (!var(L) || L < 1) return false;
        const uint64_t take = L - vlen(L);
        if (take > left()) return false;
        end = i + (size_t)take;
        return true;
    }
};

}  // namespace nxgwire
