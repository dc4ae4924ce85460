// nxg_zstd.hip -- zstd decompression of compressed archive batch records on gfx950.
//
// A compressed archive record, after its RecordHeader, is u32 BE uncompressed length | the
// index (indexed files) | one zstd frame of the batch, compressed with the archive's trained
// dictionary (netidx-archive/src/logfile/reader.rs:453-477, 737-801). The reference decompresses
// one record at a time on a host core (zstd::bulk::Decompressor::decompress_to_buffer); here a
// wave decompresses one record and the grid takes many records at once, straight into device
// memory, where nxg_decode_archive_batch decodes each batch.
//
// One wave per frame (a persistent grid over the records). Per block (RFC 8878 3.1.1):
//   raw / RLE blocks: a wave-parallel byte copy;
//   compressed blocks: the literals section -- raw, RLE, or Huffman-coded in 1 or 4 streams,
//     lanes 0..3 decoding one stream each into the wave's literal buffer -- then the sequences
//     section, decoded uniformly by the wave (FSE states, extra bits, repeat offsets) and executed
//     sequence by sequence with wave-parallel copies: literals through a 1 KiB LDS stage, matches
//     from a 16 KiB LDS ring of the latest output (the global output for older bytes, the
//     dictionary's content before the frame).
// Output bytes go to the global output and to the ring. Global output is read back only more
// than RING bytes behind the write position, and the wave drains its stores every RING / 4
// bytes, so every byte read back was stored and drained before any load of its line. Literal
// buffers are rewritten every block and read with nontemporal loads (which bypass the CU's L1,
// MI355X_MICROARCH.md load flavours), so no stale line is ever read.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "nxg_device.h"
#include "nxg_zstd.h"

using namespace nxz;

// device-resident entropy state a frame starts from: a dictionary's tables, or (has_tables 0)
// none; and the predefined distributions' tables
struct NxzDictDev {
    uint32_t id, content_len, has_tables, huf_bits;
    uint32_t rep[3];
    uint32_t ll_log, ml_log, of_log;
    const uint8_t* content;
    HufCell huf[1u << kHufMaxBits];
    FseCell ll[1u << kLLLog], ml[1u << kMLLog], of[1u << kOFLog];
};
struct NxzDefaults {
    FseCell ll[64], ml[64], of[32];
};
// one record: its frame in the staged source, its output slot; the result
struct NxzRec {
    uint64_t frame_off, frame_len, out_off, out_cap;
};
struct NxzRes {
    uint64_t out_len;
    uint32_t err, pad;
};

namespace {

constexpr uint32_t RING = 16384, RMASK = RING - 1, DRAIN = RING / 4;
constexpr uint32_t LSTAGE = 1024;
constexpr uint32_t LITBUF = kBlockMax;  // literal buffer per wave (global)

struct ZLds {
    FseCell ll[1u << kLLLog], ml[1u << kMLLog], of[1u << kOFLog];
    HufCell huf[1u << kHufMaxBits];
    uint8_t ring[RING];
    uint8_t stage[LSTAGE];
    int16_t norm[64];
    uint16_t nxt[64];
    uint8_t wts[256];
    FseCell wfse[64];
};

NXG_DEV uint32_t bcast(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
NXG_DEV uint8_t ldnt(const uint8_t* p) { return __builtin_nontemporal_load(p); }

// backward bitstream (RFC 8878 4.1: read from the last byte's marker bit down to bit 0); bits
// below the start read as 0, as libzstd's containers do
struct Bwd {
    const uint8_t* p;
    uint32_t n;
    int32_t bp;   // unread bits: [0, bp)
    int32_t wlo;  // the cached window: bytes [wlo, wlo + 8)
    uint64_t win;
    NXG_DEV bool init(const uint8_t* p_, uint32_t n_) {
        p = p_;
        n = n_;
        wlo = -64;
        win = 0;
        if (n == 0) return false;
        const uint32_t last = p[n - 1];
        if (!last) return false;
        bp = (int32_t)(n * 8 - 8 + highbit(last));
        return true;
    }
    NXG_DEV void load() {
        const int32_t top = (bp + 7) >> 3;
        const int32_t lo = top - 8 < 0 ? 0 : top - 8;
        uint64_t v = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t q = (uint32_t)lo + i;
            if (q < n) v |= (uint64_t)p[q] << (8 * i);
        }
        win = v;
        wlo = lo;
    }
    NXG_DEV uint32_t peek(uint32_t k) {  // k <= 32
        if (k == 0) return 0;
        const uint64_t mask = (1ull << k) - 1ull;
        const int32_t lo = bp - (int32_t)k;
        if (bp <= 0) return 0;
        if ((lo < 0 ? 0 : lo) < wlo * 8 || bp > wlo * 8 + 64) load();
        if (lo >= 0) return (uint32_t)((win >> (lo - wlo * 8)) & mask);
        return (uint32_t)(((win & ((1ull << bp) - 1ull)) << (-lo)) & mask);
    }
    NXG_DEV uint32_t read(uint32_t k) {
        const uint32_t v = peek(k);
        bp -= (int32_t)k;
        return v;
    }
};

// the decoding state of one frame, uniform in the wave
struct Frame {
    const uint8_t* src;
    uint8_t* out;
    uint64_t cap;
    uint64_t op;         // bytes written
    uint64_t drained;    // every byte below was stored and drained
    const NxzDictDev* dict;
    uint32_t rep[3];
    bool huf_ok, ll_ok, ml_ok, of_ok;
    uint32_t huf_bits, ll_log, ml_log, of_log;
};

NXG_DEV void drain_if(Frame& f) {
    if (f.op >= f.drained + DRAIN) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        f.drained = f.op;
    }
}

// byte at frame position q (< f.op): the ring, the global output, or the dictionary's content
NXG_DEV uint32_t hist_byte(const ZLds& L, const Frame& f, int64_t q, uint64_t b0) {
    if (q < 0) return f.dict->content[(int64_t)f.dict->content_len + q];
    if (b0 - (uint64_t)q <= RING) return L.ring[(uint64_t)q & RMASK];
    return f.out[q];
}

// a wave-parallel copy of `len` bytes into the output: byte i = get(i) (uniform len)
template <typename Get>
NXG_DEV void emit_bytes(ZLds& L, Frame& f, uint32_t len, uint32_t lane, Get get) {
    const uint64_t o0 = f.op;
    for (uint32_t k = 0; k < len; k += 64) {
        const uint32_t i = k + lane;
        uint32_t b = 0;
        if (i < len) b = get(i, o0 + k);
        wave_lds_order();
        if (i < len) {
            const uint64_t p = o0 + i;
            L.ring[p & RMASK] = (uint8_t)b;
            f.out[p] = (uint8_t)b;
        }
        wave_lds_order();
        f.op = o0 + min(len, k + 64);
        drain_if(f);  // (inside the copy too: a long match reads what it wrote RING bytes ago)
    }
}

// a match: `len` bytes from `off` back (off <= op + dictionary content, checked by the caller)
NXG_DEV void emit_match(ZLds& L, Frame& f, uint32_t len, uint64_t off, uint32_t lane) {
    const uint64_t o0 = f.op;
    emit_bytes(L, f, len, lane, [&](uint32_t i, uint64_t b0) -> uint32_t {
        const uint64_t p = o0 + i;
        // the source lies before this round's first byte (a short offset repeats its period)
        const int64_t q = off >= 64 ? (int64_t)p - (int64_t)off
                                    : (int64_t)b0 - (int64_t)off + (int64_t)((p - b0) % off);
        return hist_byte(L, f, q, b0);
    });
}

// the literal stage: bytes [sb, sb + LSTAGE) of the block's literals
struct Lits {
    const uint8_t* p;  // raw: the frame bytes; Huffman: the wave's literal buffer (nontemporal)
    bool nt, rle;
    uint32_t rle_byte, total, pos, sb, se;
};
NXG_DEV void stage_fill(ZLds& L, Lits& l, uint32_t at, uint32_t lane) {
    wave_lds_order();
#pragma unroll
    for (uint32_t j = 0; j < LSTAGE / 64; j++) {
        const uint32_t q = at + j * 64 + lane;
        uint32_t b = 0;
        if (q < l.total) b = l.rle ? l.rle_byte : (l.nt ? ldnt(l.p + q) : l.p[q]);
        L.stage[j * 64 + lane] = (uint8_t)b;
    }
    wave_lds_order();
    l.sb = at;
    l.se = at + LSTAGE;
}
NXG_DEV void emit_lits(ZLds& L, Frame& f, Lits& l, uint32_t len, uint32_t lane) {
    while (len) {
        if (l.pos < l.sb || l.pos + 64 > l.se) stage_fill(L, l, l.pos, lane);
        const uint32_t c = min(len, min(64u, l.se - l.pos));
        const uint32_t s0 = l.pos - l.sb;
        emit_bytes(L, f, c, lane, [&](uint32_t i, uint64_t) -> uint32_t { return L.stage[s0 + i]; });
        l.pos += c;
        len -= c;
    }
}

// an FSE table for the sequences: mode 0 predefined, 1 RLE, 2 described, 3 repeat. Returns the
// bytes consumed, or -1. Uniform; lane 0 builds, the wave waits.
NXG_DEV int seq_table(ZLds& L, FseCell* tab, const FseCell* def, uint32_t def_log, uint32_t mode,
                      const uint8_t* p, uint32_t n, uint32_t max_sym, uint32_t max_log,
                      uint32_t& log, bool& ok, uint32_t lane) {
    int used = 0;
    if (mode == 0) {
        for (uint32_t i = lane; i < (1u << def_log); i += 64) tab[i] = def[i];
        log = def_log;
        ok = true;
    } else if (mode == 1) {
        if (n < 1 || p[0] > max_sym) return -1;
        if (lane == 0) build_rle(tab, p[0]);
        log = 0;
        ok = true;
        used = 1;
    } else if (mode == 2) {
        uint32_t r = 0, al = 0, ms = 0;
        if (lane == 0) {
            r = read_ncount(p, n, L.norm, max_sym, max_log, &al, &ms);
            if (r && !build_fse(tab, L.norm, ms, al, L.nxt)) r = 0;
        }
        r = bcast(r);
        al = bcast(al);
        if (!r) return -1;
        log = al;
        ok = true;
        used = (int)r;
    } else {
        if (!ok) return -1;
    }
    wave_lds_order();
    return used;
}

// Huffman tree description at p (n bytes) into L.huf; bytes used or 0
NXG_DEV uint32_t huf_table(ZLds& L, const uint8_t* p, uint32_t n, uint32_t& bits, uint32_t lane) {
    uint32_t used = 0, ns = 0, mb = 0;
    if (lane == 0) used = read_huf_weights(p, n, L.wts, &ns, &mb, L.wfse, L.norm, L.nxt);
    used = bcast(used);
    ns = bcast(ns);
    mb = bcast(mb);
    wave_lds_order();
    if (!used) return 0;
    // symbols of weight w take 2^(w-1) cells from their weight's start (build_huf, in parallel:
    // lane s fills symbol s's cells; its start = cells of lower weights + earlier same-weight
    // symbols)
    uint32_t cnt[kHufMaxBits + 2];
#pragma unroll
    for (int k = 0; k < kHufMaxBits + 2; k++) cnt[k] = 0;
    for (uint32_t s = 0; s < ns; s++) cnt[L.wts[s]]++;
    uint32_t start[kHufMaxBits + 2];
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t k = 0; k < kHufMaxBits + 2; k++) {
        start[k] = acc;
        if (k >= 1 && k <= mb) acc += cnt[k] << (k - 1);
    }
    for (uint32_t s0 = 0; s0 < ns; s0 += 64) {
        const uint32_t s = s0 + lane;
        const uint32_t w = s < ns ? L.wts[s] : 0u;
        // cells before s among symbols of the same weight (s0 .. s-1 of this round by a scan per
        // weight would need 12 scans; the rounds are few: count serially per lane)
        uint32_t st = 0;
        if (w) {
            st = start[w];
            for (uint32_t t = 0; t < s; t++)
                if (L.wts[t] == w) st += 1u << (w - 1);
            const uint32_t len = 1u << (w - 1);
            const uint8_t nb = (uint8_t)(mb + 1 - w);
            for (uint32_t i = 0; i < len; i++) L.huf[st + i] = HufCell{(uint8_t)s, nb};
        }
    }
    wave_lds_order();
    bits = mb;
    return used;
}

// one stream of Huffman-coded literals into dst[0, cnt): true when the stream is consumed
// exactly (HUF_decompress1X: BIT_endOfDStream)
NXG_DEV bool huf_stream(const ZLds& L, const uint8_t* s, uint32_t n, uint8_t* dst, uint32_t cnt,
                        uint32_t bits) {
    Bwd b;
    if (!b.init(s, n)) return false;
    for (uint32_t k = 0; k < cnt; k++) {
        const HufCell c = L.huf[b.peek(bits)];
        dst[k] = c.sym;
        b.bp -= c.nbits;
    }
    return b.bp == 0;
}

NXG_DEV uint64_t rd_le(const uint8_t* p, uint32_t k) {
    uint64_t v = 0;
    for (uint32_t i = 0; i < k; i++) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

// XXH64 (seed 0) of the output; lane 0 only, after a drain
NXG_DEV uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
NXG_DEV uint64_t xxh64(const uint8_t* p, uint64_t len) {
    constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull,
                       P3 = 1609587929392839161ull, P4 = 9650029242287828579ull,
                       P5 = 2870177450012600261ull;
    auto rd8 = [&](uint64_t i) {
        uint64_t v = 0;
        for (int k = 0; k < 8; k++) v |= (uint64_t)ldnt(p + i + k) << (8 * k);
        return v;
    };
    auto round = [&](uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; };
    uint64_t i = 0, h;
    if (len >= 32) {
        uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
        for (; i + 32 <= len; i += 32) {
            v1 = round(v1, rd8(i));
            v2 = round(v2, rd8(i + 8));
            v3 = round(v3, rd8(i + 16));
            v4 = round(v4, rd8(i + 24));
        }
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        h = (h ^ round(0, v1)) * P1 + P4;
        h = (h ^ round(0, v2)) * P1 + P4;
        h = (h ^ round(0, v3)) * P1 + P4;
        h = (h ^ round(0, v4)) * P1 + P4;
    } else {
        h = P5;
    }
    h += len;
    for (; i + 8 <= len; i += 8) {
        h ^= round(0, rd8(i));
        h = rotl(h, 27) * P1 + P4;
    }
    if (i + 4 <= len) {
        uint64_t v = 0;
        for (int k = 0; k < 4; k++) v |= (uint64_t)ldnt(p + i + k) << (8 * k);
        h ^= v * P1;
        h = rotl(h, 23) * P2 + P3;
        i += 4;
    }
    for (; i < len; i++) {
        h ^= (uint64_t)ldnt(p + i) * P5;
        h = rotl(h, 11) * P1;
    }
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

// One compressed block [ip, ip + bs). Returns Z_OK or an error.
NXG_DEV uint32_t block_compressed(ZLds& L, Frame& f, const uint8_t* ip, uint32_t bs,
                                  uint8_t* litbuf, const NxzDefaults* defs, uint32_t lane) {
    if (bs < 1) return Z_CORRUPT;
    const uint8_t* bend = ip + bs;
    // ---- literals section (RFC 8878 3.1.1.3.1)
    const uint32_t b0 = ip[0];
    const uint32_t lt = b0 & 3, sf = (b0 >> 2) & 3;
    Lits l{};
    uint32_t sect;
    if (lt <= 1) {
        uint32_t lhs, rs;
        if ((sf & 1) == 0) {
            lhs = 1;
            rs = b0 >> 3;
        } else if (sf == 1) {
            if (bs < 2) return Z_CORRUPT;
            lhs = 2;
            rs = (b0 >> 4) + ((uint32_t)ip[1] << 4);
        } else {
            if (bs < 3) return Z_CORRUPT;
            lhs = 3;
            rs = (b0 >> 4) + ((uint32_t)ip[1] << 4) + ((uint32_t)ip[2] << 12);
        }
        if (rs > kBlockMax) return Z_CORRUPT;
        l.total = rs;
        if (lt == 0) {
            if (lhs + rs > bs) return Z_CORRUPT;
            l.p = ip + lhs;
            sect = lhs + rs;
        } else {
            if (lhs + 1 > bs) return Z_CORRUPT;
            l.rle = true;
            l.rle_byte = ip[lhs];
            sect = lhs + 1;
        }
    } else {
        const uint32_t lhs = sf <= 1 ? 3 : (sf == 2 ? 4 : 5);
        const uint32_t nb = sf <= 1 ? 10 : (sf == 2 ? 14 : 18);
        if (lhs > bs) return Z_CORRUPT;
        const uint64_t h = rd_le(ip, lhs);
        const uint32_t rs = (uint32_t)(h >> 4) & ((1u << nb) - 1);
        const uint32_t cs = (uint32_t)(h >> (4 + nb)) & ((1u << nb) - 1);
        if (rs > kBlockMax || lhs + cs > bs) return Z_CORRUPT;
        const uint8_t* d = ip + lhs;
        uint32_t dn = cs;
        if (lt == 2) {
            const uint32_t u = huf_table(L, d, dn, f.huf_bits, lane);
            if (!u) return Z_CORRUPT;
            f.huf_ok = true;
            d += u;
            dn -= u;
        } else if (!f.huf_ok) {
            return Z_CORRUPT;  // treeless literals with no previous table
        }
        bool ok = true;
        if (sf == 0) {  // one stream
            if (lane == 0) ok = huf_stream(L, d, dn, litbuf, rs, f.huf_bits);
        } else {  // four streams behind a jump table
            // libzstd: fewer than MIN_LITERALS_FOR_4_STREAMS (6) literals cannot be 4 streams
            if (dn < 10 || rs < 6) return Z_CORRUPT;
            const uint32_t s1 = (uint32_t)rd_le(d, 2), s2 = (uint32_t)rd_le(d + 2, 2),
                           s3 = (uint32_t)rd_le(d + 4, 2);
            if (6u + s1 + s2 + s3 >= dn) return Z_CORRUPT;
            const uint32_t s4 = dn - 6 - s1 - s2 - s3;
            const uint32_t seg = (rs + 3) / 4;
            if (3 * seg > rs) return Z_CORRUPT;
            if (lane < 4) {
                const uint32_t so = lane == 0 ? 0 : (lane == 1 ? s1 : (lane == 2 ? s1 + s2 : s1 + s2 + s3));
                const uint32_t sn = lane == 0 ? s1 : (lane == 1 ? s2 : (lane == 2 ? s3 : s4));
                const uint32_t c = lane < 3 ? seg : rs - 3 * seg;
                ok = huf_stream(L, d + 6 + so, sn, litbuf + lane * seg, c, f.huf_bits);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (__any(!ok)) return Z_CORRUPT;
        l.p = litbuf;
        l.nt = true;
        l.total = rs;
        sect = lhs + cs;
    }
    l.sb = 1;
    l.se = 0;  // empty stage
    // ---- sequences section (RFC 8878 3.1.1.3.2)
    const uint8_t* sp = ip + sect;
    if (sp >= bend) return Z_CORRUPT;
    uint32_t nseq = sp[0];
    if (nseq == 0) {
        if (sp + 1 != bend) return Z_CORRUPT;
        if (f.op + l.total > f.cap) return Z_DST_SMALL;
        emit_lits(L, f, l, l.total, lane);
        return Z_OK;
    }
    if (nseq < 128) {
        sp += 1;
    } else if (nseq < 255) {
        if (sp + 2 > bend) return Z_CORRUPT;
        nseq = ((nseq - 128) << 8) + sp[1];
        sp += 2;
    } else {
        if (sp + 3 > bend) return Z_CORRUPT;
        nseq = sp[1] + ((uint32_t)sp[2] << 8) + 0x7F00;
        sp += 3;
    }
    if (sp >= bend) return Z_CORRUPT;
    const uint32_t modes = sp[0];
    sp += 1;
    if (modes & 3) return Z_CORRUPT;
    int u = seq_table(L, L.ll, defs->ll, 6, modes >> 6, sp, (uint32_t)(bend - sp), kLLMax, kLLLog,
                      f.ll_log, f.ll_ok, lane);
    if (u < 0) return Z_CORRUPT;
    sp += u;
    u = seq_table(L, L.of, defs->of, 5, (modes >> 4) & 3, sp, (uint32_t)(bend - sp), kOFMax,
                  kOFLog, f.of_log, f.of_ok, lane);
    if (u < 0) return Z_CORRUPT;
    sp += u;
    u = seq_table(L, L.ml, defs->ml, 6, (modes >> 2) & 3, sp, (uint32_t)(bend - sp), kMLMax,
                  kMLLog, f.ml_log, f.ml_ok, lane);
    if (u < 0) return Z_CORRUPT;
    sp += u;
    Bwd b;
    if (sp >= bend || !b.init(sp, (uint32_t)(bend - sp))) return Z_CORRUPT;
    uint32_t sll = b.read(f.ll_log), sof = b.read(f.of_log), sml = b.read(f.ml_log);
    const uint64_t hist = f.dict ? f.dict->content_len : 0;
    for (uint32_t i = 0; i < nseq; i++) {
        const FseCell cl = L.ll[sll], cm = L.ml[sml], co = L.of[sof];
        const uint32_t ofc = co.sym;
        if (ofc > 31) return Z_CORRUPT;
        const uint64_t ofv = (1ull << ofc) + b.read(ofc);
        const uint32_t mlc = cm.sym, llc = cl.sym;
        const uint32_t ml = ml_base(mlc) + b.read(ml_bits(mlc));
        const uint32_t ll = ll_base(llc) + b.read(ll_bits(llc));
        if (i + 1 < nseq) {  // states: literals length, match length, offset
            sll = cl.base + b.read(cl.nbits);
            sml = cm.base + b.read(cm.nbits);
            sof = co.base + b.read(co.nbits);
        }
        // repeat offsets (RFC 8878 3.1.1.5)
        uint64_t off;
        if (ofv > 3) {
            off = ofv - 3;
            f.rep[2] = f.rep[1];
            f.rep[1] = f.rep[0];
            f.rep[0] = (uint32_t)off;
        } else {
            const uint32_t idx = (uint32_t)ofv - 1 + (ll == 0 ? 1u : 0u);
            if (idx == 0) {
                off = f.rep[0];
            } else if (idx == 3) {
                off = (uint64_t)f.rep[0] - 1;
                f.rep[2] = f.rep[1];
                f.rep[1] = f.rep[0];
                f.rep[0] = (uint32_t)off;
            } else {
                off = idx == 1 ? f.rep[1] : f.rep[2];  // (no dynamic index: registers)
                if (idx == 2) f.rep[2] = f.rep[1];
                f.rep[1] = f.rep[0];
                f.rep[0] = (uint32_t)off;
            }
        }
        if (l.pos + ll > l.total) return Z_CORRUPT;
        if (f.op + ll + ml > f.cap) return Z_DST_SMALL;
        emit_lits(L, f, l, ll, lane);
        if (off == 0 || off > f.op + hist) return Z_CORRUPT;
        emit_match(L, f, ml, off, lane);
    }
    if (b.bp > 0) return Z_CORRUPT;  // bits left over (libzstd: < BIT_DStream_completed)
    const uint32_t rest = l.total - l.pos;
    if (f.op + rest > f.cap) return Z_DST_SMALL;
    emit_lits(L, f, l, rest, lane);
    return Z_OK;
}

// one frame [p, p + n) into out[0, cap)
NXG_DEV uint32_t frame_decode(ZLds& L, Frame& f, const uint8_t* p, uint64_t n, uint8_t* litbuf,
                              const NxzDefaults* defs, uint32_t lane) {
    if (n < 6 || (uint32_t)rd_le(p, 4) != kFrameMagic) return Z_PREFIX;
    const uint32_t fhd = p[4];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, cksum = (fhd >> 2) & 1;
    const uint32_t did_flag = fhd & 3;
    if (fhd & 8) return Z_PREFIX;  // reserved bit
    uint64_t ip = 5;
    if (!single) ip += 1;  // window descriptor
    const uint32_t did_len = did_flag == 3 ? 4 : did_flag;
    const uint32_t fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : (1u << fcs_flag);
    if (ip + did_len + fcs_len > n) return Z_SRC;
    const uint32_t did = (uint32_t)rd_le(p + ip, did_len);
    ip += did_len;
    int64_t fcs = -1;
    if (fcs_len) {
        fcs = (int64_t)rd_le(p + ip, fcs_len) + (fcs_len == 2 ? 256 : 0);
        ip += fcs_len;
    }
    if (did && (!f.dict || f.dict->id != did)) return Z_DICT;
    if (fcs >= 0 && (uint64_t)fcs > f.cap) return Z_DST_SMALL;
    // the entropy state a frame starts from (a dictionary's, else none) and the repeat offsets
    if (f.dict && f.dict->has_tables) {
        for (uint32_t i = lane; i < (1u << kHufMaxBits); i += 64) L.huf[i] = f.dict->huf[i];
        for (uint32_t i = lane; i < (1u << kLLLog); i += 64) L.ll[i] = f.dict->ll[i];
        for (uint32_t i = lane; i < (1u << kMLLog); i += 64) L.ml[i] = f.dict->ml[i];
        for (uint32_t i = lane; i < (1u << kOFLog); i += 64) L.of[i] = f.dict->of[i];
        f.huf_ok = f.ll_ok = f.ml_ok = f.of_ok = true;
        f.huf_bits = f.dict->huf_bits;
        f.ll_log = f.dict->ll_log;
        f.ml_log = f.dict->ml_log;
        f.of_log = f.dict->of_log;
        for (int k = 0; k < 3; k++) f.rep[k] = f.dict->rep[k];
    } else {
        f.huf_ok = f.ll_ok = f.ml_ok = f.of_ok = false;
        f.rep[0] = 1;
        f.rep[1] = 4;
        f.rep[2] = 8;
    }
    wave_lds_order();
    for (;;) {
        if (ip + 3 > n) return Z_SRC;
        const uint32_t bh = (uint32_t)rd_le(p + ip, 3);
        ip += 3;
        const uint32_t last = bh & 1, type = (bh >> 1) & 3, bs = bh >> 3;
        uint32_t r = Z_OK;
        if (type == 0) {  // raw
            if (bs > kBlockMax || ip + bs > n) return Z_CORRUPT;
            if (f.op + bs > f.cap) return Z_DST_SMALL;
            const uint8_t* q = p + ip;
            emit_bytes(L, f, bs, lane, [&](uint32_t i, uint64_t) -> uint32_t { return q[i]; });
            ip += bs;
        } else if (type == 1) {  // RLE: one byte, bs times
            if (bs > kBlockMax || ip + 1 > n) return Z_CORRUPT;
            if (f.op + bs > f.cap) return Z_DST_SMALL;
            const uint32_t v = p[ip];
            emit_bytes(L, f, bs, lane, [&](uint32_t, uint64_t) -> uint32_t { return v; });
            ip += 1;
        } else if (type == 2) {
            if (bs > kBlockMax || ip + bs > n) return Z_CORRUPT;
            const uint64_t o0 = f.op;
            r = block_compressed(L, f, p + ip, bs, litbuf, defs, lane);
            if (r == Z_OK && f.op - o0 > kBlockMax) r = Z_CORRUPT;
            ip += bs;
        } else {
            return Z_CORRUPT;  // reserved block type
        }
        if (r != Z_OK) return r;
        if (last) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (cksum) {
        if (ip + 4 > n) return Z_SRC;
        const uint32_t want = (uint32_t)rd_le(p + ip, 4);
        ip += 4;
        uint32_t got = 0;
        if (lane == 0) got = (uint32_t)xxh64(f.out, f.op);
        got = bcast(got);
        if (got != want) return Z_CHECKSUM;
    }
    if (ip != n) return Z_PREFIX;  // a second frame or trailing bytes: not one record's frame
    if (fcs >= 0 && (uint64_t)fcs != f.op) return Z_FRAME_SIZE;
    return Z_OK;
}

__global__ __launch_bounds__(64) void nxg_zstd_kernel(const uint8_t* __restrict__ src,
                                                      const NxzRec* __restrict__ recs, uint32_t n,
                                                      const NxzDictDev* dict,
                                                      const NxzDefaults* defs, uint8_t* out,
                                                      uint8_t* lit, NxzRes* res) {
    __shared__ __attribute__((aligned(16))) ZLds L;
    const uint32_t lane = threadIdx.x;
    uint8_t* litbuf = lit + (uint64_t)blockIdx.x * LITBUF;
    for (uint32_t r = blockIdx.x; r < n; r += gridDim.x) {
        const NxzRec rc = recs[r];
        Frame f{};
        f.src = src;
        f.out = out + rc.out_off;
        f.cap = rc.out_cap;
        f.op = 0;
        f.drained = 0;
        f.dict = dict;
        const uint32_t e = frame_decode(L, f, src + rc.frame_off, rc.frame_len, litbuf, defs, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) res[r] = NxzRes{f.op, e, 0};
        wave_lds_order();
    }
}

}  // namespace

// ---- host ---------------------------------------------------------------------------------
// the host builds tables with the same code (nxg_zstd.h) the device runs per block
bool nxg_zstd_build_dict(const uint8_t* d, uint64_t n, NxzDictDev* out, uint64_t* content_off) {
    memset(out, 0, sizeof *out);
    if (n < 8 || (uint32_t)(d[0] | d[1] << 8 | d[2] << 16 | (uint32_t)d[3] << 24) != kDictMagic) {
        // a raw-content dictionary (no magic): history only, no tables, default offsets
        out->rep[0] = 1;
        out->rep[1] = 4;
        out->rep[2] = 8;
        out->content_len = (uint32_t)n;
        *content_off = 0;
        return true;
    }
    out->id = (uint32_t)(d[4] | d[5] << 8 | d[6] << 16 | (uint32_t)d[7] << 24);
    uint64_t p = 8;
    uint8_t w[256];
    FseCell fse[64];
    int16_t norm[64];
    uint16_t next[64];
    uint32_t ns, mb;
    const uint32_t hu = read_huf_weights(d + p, (uint32_t)(n - p), w, &ns, &mb, fse, norm, next);
    if (!hu) return false;
    build_huf(out->huf, w, ns, mb);
    out->huf_bits = mb;
    p += hu;
    uint32_t al, ms, u;
    u = read_ncount(d + p, (uint32_t)(n - p), norm, kOFMax, kOFLog, &al, &ms);
    if (!u || !build_fse(out->of, norm, ms, al, next)) return false;
    out->of_log = al;
    p += u;
    u = read_ncount(d + p, (uint32_t)(n - p), norm, kMLMax, kMLLog, &al, &ms);
    if (!u || !build_fse(out->ml, norm, ms, al, next)) return false;
    out->ml_log = al;
    p += u;
    u = read_ncount(d + p, (uint32_t)(n - p), norm, kLLMax, kLLLog, &al, &ms);
    if (!u || !build_fse(out->ll, norm, ms, al, next)) return false;
    out->ll_log = al;
    p += u;
    if (p + 12 > n) return false;
    for (int k = 0; k < 3; k++) {
        const uint8_t* q = d + p + 4 * k;
        out->rep[k] = (uint32_t)(q[0] | q[1] << 8 | q[2] << 16 | (uint32_t)q[3] << 24);
    }
    p += 12;
    out->content_len = (uint32_t)(n - p);
    for (int k = 0; k < 3; k++)
        if (out->rep[k] == 0 || out->rep[k] > out->content_len) return false;
    out->has_tables = 1;
    *content_off = p;
    return true;
}

bool nxg_zstd_build_defaults(NxzDefaults* o) {
    int16_t norm[64];
    uint16_t next[64];
    for (int s = 0; s < 36; s++) norm[s] = kLLDefault[s];
    if (!build_fse(o->ll, norm, 35, 6, next)) return false;
    for (int s = 0; s < 53; s++) norm[s] = kMLDefault[s];
    if (!build_fse(o->ml, norm, 52, 6, next)) return false;
    for (int s = 0; s < 29; s++) norm[s] = kOFDefault[s];
    return build_fse(o->of, norm, 28, 5, next);
}

void nxg_zstd_set_content(NxzDictDev* d, const uint8_t* dcontent) { d->content = dcontent; }

// Not part of the ABI (tests, host only, no GPU): the Huffman tree description reader and the
// dictionary parser on arbitrary bytes. Returns the bytes the tree used (0: rejected) / whether
// the dictionary parses.
extern "C" uint32_t nxg_debug_huf_weights(const uint8_t* p, uint32_t n, uint32_t* n_sym) {
    uint8_t w[256];
    FseCell fse[64];
    int16_t norm[64];
    uint16_t next[64];
    uint32_t ns = 0, mb = 0;
    const uint32_t u = read_huf_weights(p, n, w, &ns, &mb, fse, norm, next);
    if (n_sym) *n_sym = ns;
    return u;
}
extern "C" bool nxg_debug_zstd_dict_ok(const uint8_t* d, uint64_t n) {
    NxzDictDev* o = new NxzDictDev();
    uint64_t coff = 0;
    const bool ok = nxg_zstd_build_dict(d, n, o, &coff);
    delete o;
    return ok;
}
uint64_t nxg_zstd_dict_dev_bytes() { return sizeof(NxzDictDev); }
uint64_t nxg_zstd_defaults_bytes() { return sizeof(NxzDefaults); }
uint64_t nxg_zstd_rec_bytes() { return sizeof(NxzRec); }
uint64_t nxg_zstd_res_bytes() { return sizeof(NxzRes); }
uint64_t nxg_zstd_litbuf_bytes() { return LITBUF; }
int nxg_zstd_grid(int ncu) {
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, nxg_zstd_kernel, 64, 0) != hipSuccess)
        occ = 1;
    return std::max(1, occ) * ncu;
}

hipError_t nxg_launch_zstd(const uint8_t* dsrc, const void* drecs, uint32_t n, const void* ddict,
                           const void* ddefs, uint8_t* dout, uint8_t* dlit, void* dres, int grid,
                           hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t g = (uint32_t)std::min<uint64_t>((uint64_t)grid, n);
    hipLaunchKernelGGL(nxg_zstd_kernel, dim3(g), dim3(64), 0, s, dsrc,
                       reinterpret_cast<const NxzRec*>(drecs), n,
                       reinterpret_cast<const NxzDictDev*>(ddict),
                       reinterpret_cast<const NxzDefaults*>(ddefs), dout, dlit,
                       reinterpret_cast<NxzRes*>(dres));
    return hipGetLastError();
}
