// nxg_archive_fast.hip -- the fast path of archive batch decode for gfx950:
// <GPooled<Vec<BatchItem>> as Pack>::decode (netidx-core/src/pack.rs:934-973) with
// BatchItem(Id, Event) (netidx-archive/src/logfile/mod.rs:150-205) and Event::decode
// (netidx/src/subscriber/mod.rs:154-177):
//     varint count | count x ( varint Id (as u32) | 0x40 = Unsubscribed, or a bare Value )
// No item carries a length: where one ends follows from its value's tags. The batch is cut into
// 4 KiB tiles held in LDS, one wave each, 64-byte chunks one lane each, as the fast mixed decoder
// does (nxg_decode_mixed.hip), with the item structure walk in place of the length prefixes:
//
//   count   per tile: each lane walks its chunk from the chunk's first byte, one byte on after a
//           failed parse (a guess that synchronises within an item or two), then exactly from
//           its predecessor's guess; one uniform loop follows the true chain through the
//           chunks from the tile's entry (a chunk entered off its guess is walked again). The
//           tile's entry is the first item its first lane's guess found (tile 0: after the
//           count); its exit, items, child slots and item starts (bits per chunk) go out. A
//           chain that fails to parse stops there (BROKEN): bytes after the batch (the rest of an
//           mmap'd file, logfile/reader.rs:449) need not parse.
//   resolve one launch: a tile entered off its predecessor's exit is recounted from that exit;
//           block scans of (items, child slots) give every tile its first row and child slot.
//   emit    per tile whose first row is < count: the chain check (entry = predecessor's exit,
//           tile 0 at the count's end; a BROKEN tile, or the window's last, must hold the
//           batch's last item), then items 64 at a time per lane -- the Id varint, 0x40 or the
//           value by val_decode (the same restatement of Value::decode as the publisher stream's
//           fast path), text checked for UTF-8 once per tile (in LDS) or per lane from global
//           memory (text leaving the tile's image), Array elements by round_elements. Rows past
//           count are not written. The lane of row count - 1 writes the batch's end (consumed)
//           and child slots.
//
// Anything else -- an Id wider than 5 bytes, Maps, Error(Value) of a non-String, nested or
// 128+-element Arrays, Arrays leaving the tile's image, more than 1024 items in a tile, a decode
// error, too small columns -- sets fast_fail, and the host reruns the batch on the exact decoder
// (nxg_archive.hip), which reports errors exactly. The host runs this path over a window of the
// buffer that grows geometrically until the batch fits, so the cost follows the batch, not the
// bytes after it.
#include <algorithm>

#include "nxg_fmx_common.h"

#ifndef NXG_FF_CHECK
#define NXG_FF_CHECK 1  // emit waves skip a batch already declined
#endif

namespace fa {
constexpr uint32_t UNSUB = 0x40;         // Event::Unsubscribed (subscriber/mod.rs:168)
constexpr uint32_t BROKEN = 0x80000000u;  // FaDesc.items: the chain stops at `exit`
constexpr uint32_t IMGL = fmx::IMG - 24;  // emit image: items end before this (text aside)
#ifndef NXG_FA_PRE
#define NXG_FA_PRE 128
#endif
constexpr uint32_t PRE = NXG_FA_PRE;      // count image: bytes before the tile (walked for the entry)
#ifndef NXG_FA_WIN
#define NXG_FA_WIN 1  // text / varint lengths from the item's own window in the item walks
#endif
#ifndef NXG_FA_SKIP
#define NXG_FA_SKIP 1  // the chain loop jumps over chunks whose own walks continue the chain
#endif
#ifndef NXG_FA_RK
#define NXG_FA_RK 1  // an entry inside the spec walk's last run takes that run's tail, arrays included
#endif
#ifndef NXG_FA_STRIDE
#define NXG_FA_STRIDE 1  // array elements by stride speculation in the item walks
#endif
constexpr uint32_t CIMG = PRE + fmx::IMG;  // count image bytes
constexpr uint32_t CIMGL = CIMG - 24;      // count image: items end before this (text aside)
}  // namespace fa

// device results of one call (zeroed by the host)
struct FaHead {
    uint32_t fast_fail;
    uint32_t arrived;        // resolve: blocks done
    uint64_t end;            // 1 + the end of item count - 1 (0: not seen)
    uint64_t end_children;   // child slots of items 0 .. count - 1
    uint64_t items;          // total on the chains (diagnostics)
    uint64_t ticket;         // resolve: blocks by ticket (next_tile)
    uint64_t recounts;       // tiles recounted by the resolve pass (diagnostics)
    uint64_t why;            // emit: reasons of a decline, bits (diagnostics, nxg_debug_fa)
    uint64_t why_tile;       // emit: the first tile that declined (diagnostics, see below)
};
static_assert(sizeof(FaHead) == 64, "FaHead layout");

#ifndef NXG_FA_PROF
#define NXG_FA_PROF 0  // diagnostic build only: per-section wave clocks of the count pass
#endif
#if NXG_FA_PROF
// [0..4] clocks: image, own chunk's spec walk, walk before the tile, own exact walk, chain;
// [8] waves, [9] lanes that walked their chunk again exactly, [10] waves whose chain left the
// ballot path, [11] chunks walked by the whole wave in the chain loop
__device__ unsigned long long nxg_fa_prof[16];
#define FAP(k)                                                                   \
    do {                                                                         \
        if (prof) {                                                              \
            const uint64_t _t = __builtin_amdgcn_s_memtime();                    \
            prof[k] += _t - prof[15];                                            \
            prof[15] = _t;                                                       \
        }                                                                        \
    } while (0)
#else
#define FAP(k) \
    do {       \
    } while (0)
#endif
namespace {
using namespace fmx;
using namespace fa;

struct FaCountLds {  // the tile and PRE bytes before it: image offset = tile offset + PRE
    uint8_t img[CIMG];
};
struct FaEmitLds {
    uint8_t img[IMG];
    uint16_t msg[MAXM];  // the tile's item starts
    uint32_t el[MAXC];   // text checks / a round's array elements
    uint8_t mark[256];   // utf8_packed, round_elements
};

struct FaDesc {
    uint32_t entry, exit;  // tile offsets: the first item, where the chain leaves (or breaks)
    uint32_t items;        // items on the chain | BROKEN
    uint32_t kids;         // their child slots (Array elements)
};

constexpr uint32_t kTextTags = B(12) | B(13) | B(18);

// The end (image offset) of a non-Array value with tag t at q (structure only, as dleaf sizes
// it), or FAIL; wl: the window's end. Fixed-size, varint and Decimal values must end before
// il (the image's last safe offset); text, Bytes and Abstract payloads may run past the image
// (their bytes are not read here).
NXG_DEV uint32_t leaf_end(lds_bytes img, uint32_t q, uint32_t t, uint32_t wl, uint32_t il) {
    if (t >= 28u) return FAIL;
    const uint32_t bit = 1u << t;
    const uint32_t lim = min(wl, il);
    const uint32_t f1 = fixed_size1(t);
    if (f1) return q + f1 <= lim ? q + f1 : FAIL;
    if (bit & B(20)) return q + 17u <= lim ? q + 17u : FAIL;  // Decimal: 16 bytes
    uint32_t u = q + 1;
    if (bit & B(22)) {  // Error(String) only
        if (img[u] != 12u) return FAIL;
        u++;
    }
    const Win16 v = win16(img, u);
    uint64_t x;
    const uint32_t nb = wvar(v.lo, v.hi, x);
    if (nb == 0) return FAIL;
    const uint32_t s = u + nb;
    if (bit & kVarTags) return s <= lim ? s : FAIL;
    if (s > wl || !(bit & (kTextTags | B(22) | B(27)))) return FAIL;  // Map, Array: the caller
    uint64_t take = x;
    if (bit & B(27)) {  // Abstract: len-wrapped, at least 16 bytes (dleaf case 27)
        if (x < 1) return FAIL;
        take = x - vl64(x);
        if (take < 16) return FAIL;
    }
    return take < (uint64_t)(wl - s) || (take == (uint64_t)(wl - s) && !(bit & B(27)))
               ? s + (uint32_t)take
               : FAIL;
}

// The end of the item at image offset p (p + 20 <= il): Id varint (at most 5 bytes), then 0x40 or
// a value; an Array's elements are walked (fewer than 128, non-containers, ending before il).
// kids: the Array's element count.
NXG_DEV uint32_t item_end(lds_bytes img, uint32_t p, uint32_t wl, uint32_t il, uint32_t& kids) {
    kids = 0;
    const Win16 w = win16(img, p);
    const uint64_t stop = ~w.lo & 0x8080808080808080ull;
    const uint32_t k = stop ? (uint32_t)__builtin_ctzll(stop) >> 3 : 8u;
    if (k >= 5u) return FAIL;
    const uint32_t q = p + k + 1;  // the Event's first byte
    const uint32_t t = (uint32_t)(w.lo >> (8 * (k + 1))) & 0xffu;
    if (t == UNSUB) return q + 1 <= wl ? q + 1 : FAIL;
    if (NXG_FA_WIN && t < 28u && ((1u << t) & (kVarTags | kTextTags))) {
        // a varint scalar or text: its varint from the same window (bytes k + 2 .. k + 11 of it,
        // k <= 4), not a second window read as leaf_end makes
        const uint32_t o = 8 * (k + 2);
        uint64_t x;
        const uint32_t nb = wvar((w.lo >> o) | (w.hi << (64 - o)), w.hi >> o, x);
        if (nb == 0) return FAIL;
        const uint32_t s = q + 1 + nb;
        if ((1u << t) & kVarTags) return s <= min(wl, il) ? s : FAIL;
        return s <= wl && x <= (uint64_t)(wl - s) ? s + (uint32_t)x : FAIL;
    }
    if (t != 19u) return leaf_end(img, q, t, wl, il);
    const uint32_t c = img[q + 1];
    if (c >= 0x80u) return FAIL;
    kids = c;
    uint32_t e = q + 2;
    if (NXG_FA_STRIDE && c) {
        // stride speculation: an array whose first element has a fixed size f is taken to be c
        // elements of that size, each element's tag then read independently (8 at a time, one
        // LDS round trip instead of one per element); any other element falls to the exact walk
        const uint32_t f = fixed_size1(img[e]);
        if (f && e + c * f <= min(wl, il)) {
            bool ok = true;
#pragma unroll 1
            for (uint32_t i0 = 1; i0 < c && ok; i0 += 8) {
                uint32_t tg[8];
#pragma unroll
                for (int j = 0; j < 8; j++) tg[j] = img[i0 + j < c ? e + (i0 + j) * f : e];
#pragma unroll
                for (int j = 0; j < 8; j++) ok = ok && fixed_size1(tg[j]) == f;
            }
            if (ok) return e + c * f;
        }
    }
#pragma unroll 1
    for (uint32_t i = 0; i < c && e != FAIL; i++) {
        if (e >= il) return FAIL;
        const uint32_t et = img[e];
        e = et == 19u ? FAIL : leaf_end(img, e, et, wl, il);
    }
    return e != FAIL && e <= min(wl, il) ? e : FAIL;
}

// The exact walk of chunk [c, end) from x: items, child slots and starts (bit i: byte c + i);
// returns where it leaves the chunk, or FAIL with brk = the start that does not parse (the counts
// then cover the items before it)
NXG_DEV uint32_t chunk_walk(lds_bytes img, uint32_t x, uint32_t c, uint32_t end, uint32_t wl,
                            uint32_t& n, uint32_t& kids, uint64_t& bits, uint32_t& brk) {
    n = 0;
    kids = 0;
    bits = 0;
    brk = FAIL;
#pragma unroll 1
    while (x < end) {
        uint32_t k;
        const uint32_t e = item_end(img, x, wl, CIMGL, k);
        if (e == FAIL) {
            brk = x;
            return FAIL;
        }
        bits |= 1ull << (x - c);
        n++;
        kids += k;
        x = e;
    }
    return x;
}

// Where an item can start among the 64 positions from image offset c (4-aligned; the image holds
// c + 72 bytes): bit i when bytes c+i.. read as an Id varint of 1..5 bytes followed by a byte that
// can begin an Event (0x40, or a Value tag < 28), the first checks item_end makes. A superset of
// the item starts, from SWAR over 18 words, so a spec walk skips the positions between candidates
// instead of trying a parse at every byte (text and f64 bytes mostly fail the tag test).
NXG_DEV uint64_t item_cands(lds_bytes img, uint32_t c) {
    uint64_t T = 0, G = 0;  // T: bytes < 0x80 (varint end), G: possible Event first bytes
    uint32_t th = 0, gh = 0;  // positions 64..71
#pragma unroll
    for (int k = 0; k < 18; k++) {
        const uint32_t a = *reinterpret_cast<const __attribute__((address_space(3))) uint32_t*>(
            img + c + 4 * k);
        const uint32_t t = ~a & 0x80808080u;
        const uint32_t lt28 = ~(((a & 0x7f7f7f7fu) + 0x64646464u) | a) & 0x80808080u;
        const uint32_t g = lt28 | zero_bytes(a ^ 0x40404040u);
        if (k < 16) {
            T |= (uint64_t)nib(t) << (4 * k);
            G |= (uint64_t)nib(g) << (4 * k);
        } else {
            th |= nib(t) << (4 * (k - 16));
            gh |= nib(g) << (4 * (k - 16));
        }
    }
    // x >> s over the 72 positions (s in 1..5)
    auto sh = [](uint64_t lo, uint32_t hi, uint32_t s) { return (lo >> s) | ((uint64_t)hi << (64 - s)); };
    const uint64_t C = ~T;
    const uint64_t T1 = sh(T, th, 1), T2 = sh(T, th, 2), T3 = sh(T, th, 3), T4 = sh(T, th, 4);
    const uint64_t C1 = ~T1, C2 = ~T2, C3 = ~T3;
    const uint64_t G1 = sh(G, gh, 1), G2 = sh(G, gh, 2), G3 = sh(G, gh, 3), G4 = sh(G, gh, 4),
                   G5 = sh(G, gh, 5);
    return (T & G1) | (C & T1 & G2) | (C & C1 & T2 & G3) | (C & C1 & C2 & T3 & G4) |
           (C & C1 & C2 & C3 & T4 & G5);
}

// The guessed exit of [x0, end): the walk from x0, on to the next candidate position
// (item_cands: bit i = position cb + i, which skips only positions where the parse would fail)
// after a failed parse. first: where its last unbroken run of items starts (every item from
// there to the exit parsed in a row); rbits / rkids: that run's item starts (bit i = cb + i) and
// child slots.
NXG_DEV uint32_t spec_walk(lds_bytes img, uint32_t x0, uint32_t cb, uint32_t end, uint32_t wl,
                           uint32_t& first, uint64_t cm, uint64_t& rbits, uint32_t& rkids,
                           uint64_t& rabits) {
    auto next = [&](uint32_t p) -> uint32_t {  // the first candidate at or after p
        const uint32_t d = p - cb;
        const uint64_t rest = d < 64 ? cm & (~0ull << d) : 0ull;
        return rest ? cb + (uint32_t)__builtin_ctzll(rest) : end;
    };
    uint32_t x = next(x0);
    first = x;
    rbits = 0;
    rkids = 0;
    rabits = 0;
#pragma unroll 1
    while (x < end) {
        uint32_t k;
        const uint32_t e = item_end(img, x, wl, CIMGL, k);
        if (e == FAIL) {
            x = next(x + 1);
            first = x;
            rbits = 0;
            rkids = 0;
            rabits = 0;
            continue;
        }
        if (x - cb < 64) {
            rbits |= 1ull << (x - cb);
            if (k) rabits |= 1ull << (x - cb);  // an Array with elements
        }
        rkids += k;
        x = e;
    }
    return x;
}

// the element count of the Array item at image offset p (its Id varint, tag 19, the count byte)
NXG_DEV uint32_t arr_count(lds_bytes img, uint32_t p) {
    const Win16 w = win16(img, p);
    const uint64_t stop = ~w.lo & 0x8080808080808080ull;
    const uint32_t k = (uint32_t)__builtin_ctzll(stop) >> 3;  // (< 5: the walk parsed it)
    return (uint32_t)(w.lo >> (8 * (k + 2))) & 0xffu;
}

// The tile's chain from entry E (uniform; image offsets, chunk j at PRE + 64 j, the tile's end at
// lim): its descriptor (tile offsets), and per lane the starts of its chunk. A / X / n / kids /
// bits / brk: the lane's walk from its guessed entry (a lane whose chunk the chain enters
// elsewhere walks again).
NXG_DEV FaDesc chain_from(lds_bytes img, uint32_t E, uint32_t lim, uint32_t wl, uint32_t lane,
                          uint32_t A, uint32_t X, uint32_t n, uint32_t kids, uint64_t bits,
                          uint32_t brk, uint64_t& obits, uint64_t* prof = nullptr) {
    uint32_t x = E, ce = NONE, bp = FAIL;
    // Every chunk entered where its predecessor's walk left it (the usual case: the guesses
    // synchronised): the chain is the lanes' own walks, from one ballot. Otherwise the uniform
    // loop below takes over from the first chunk that is not.
    uint32_t j0 = 0;
    uint64_t badm;  // chunks not entered at their guess (or whose walk broke)
    bool cov;       // an item covers the lane's whole chunk
    uint32_t jact;  // the last chunk in the tile
    {
        const uint32_t cl = PRE + lane * CH;
        const bool act = cl < lim;
        const uint32_t xp = (uint32_t)__shfl_up((int)X, 1, 64);
        const uint32_t pin = lane == 0 ? E : xp;  // where the chain enters the lane's chunk
        cov = pin >= min(cl + CH, lim);
        const uint64_t bad = __ballot(act && !(pin == A && X != FAIL));
        badm = bad;
        const uint64_t am0 = __ballot(act);
        jact = am0 ? 63u - (uint32_t)__builtin_clzll(am0) : 0u;
        j0 = bad ? (uint32_t)__builtin_ctzll(bad) : TILE / CH;
#if NXG_FA_PROF
        if (prof && bad) prof[10]++;
#endif
        if (lane < j0 && act && !cov) ce = A;
        if (j0 > 0) x = (uint32_t)__builtin_amdgcn_readlane((int)X, (int)(j0 - 1));
        if (j0 == TILE / CH) {
            const uint64_t am = __ballot(act);
            x = (uint32_t)__builtin_amdgcn_readlane((int)X, 63 - (int)__builtin_clzll(am));
        }
    }
#pragma unroll 1
    for (uint32_t j = j0; j < TILE / CH && x < lim; j++) {
        const uint32_t cj = PRE + j * CH;
        const uint32_t endj = min(cj + CH, lim);
        if (x >= endj) continue;  // an item covers the whole chunk
        if (lane == j) ce = x;
        const uint32_t Aj = (uint32_t)__builtin_amdgcn_readlane((int)A, (int)j);
        if (x == Aj) {
            const uint32_t Xj = (uint32_t)__builtin_amdgcn_readlane((int)X, (int)j);
            if (Xj == FAIL) {
                bp = (uint32_t)__builtin_amdgcn_readlane((int)brk, (int)j);
                break;
            }
            x = Xj;
            if (NXG_FA_SKIP) {
                // the chunks up to the next off-guess one continue the chain with their own
                // walks (each entered at its guess, which its predecessor's walk reaches): as on
                // the ballot path
                const uint64_t rest = badm & ~(~0ull >> (63 - j));  // off-guess chunks after j
                const uint32_t jn = min(rest ? (uint32_t)__builtin_ctzll(rest) : 64u, jact + 1);
                if (jn > j + 1) {
                    if (lane > j && lane < jn && !cov) ce = A;
                    x = (uint32_t)__builtin_amdgcn_readlane((int)X, (int)(jn - 1));
                    j = jn - 1;
                }
            }
        } else {  // entered off the guess: every lane walks it (uniform addresses)
#if NXG_FA_PROF
            if (prof) prof[11]++;
#endif
            uint32_t n2, k2, b2;
            uint64_t m2;
            const uint32_t y = chunk_walk(img, x, cj, endj, wl, n2, k2, m2, b2);
            if (lane == j) {
                n = n2;
                kids = k2;
                bits = m2;
            }
            if (y == FAIL) {
                bp = b2;
                break;
            }
            x = y;
        }
    }
    const bool mine = ce != NONE;
    obits = mine ? bits : 0ull;
    const uint32_t items = wave_sum<uint32_t>(mine ? n : 0u);
    const uint32_t ks = wave_sum<uint32_t>(mine ? kids : 0u);
    if (items > MAXM) return FaDesc{FAIL, FAIL, BROKEN, 0};  // the emit pass's list holds 1024
    return bp != FAIL ? FaDesc{E - PRE, bp - PRE, items | BROKEN, ks}
                      : FaDesc{E - PRE, x - PRE, items, ks};
}

// the count image of tile t: frame bytes [t0 - PRE, t0 + IMG) (zeros before 0 and past W)
struct CountRegs {
    uint4 v[5];
};
NXG_DEV void count_load(CountRegs& g, const uint8_t* __restrict__ buf, uint64_t t0, uint64_t W,
                        uint32_t lane) {
#pragma unroll
    for (uint32_t i = 0; i < 5; i++) {
        const uint32_t off = i * 1024 + lane * 16;
        if (off < CIMG) {
            const uint64_t pos = t0 + off - PRE;  // (t0 >= PRE or t0 == 0)
            g.v[i] = t0 == 0 && off < PRE ? make_uint4(0, 0, 0, 0) : ld16(buf, pos, W);
        }
    }
}
NXG_DEV void count_store(uint8_t* img, const CountRegs& g, uint32_t lane) {
    wave_lds_order();
#pragma unroll
    for (uint32_t i = 0; i < 5; i++) {
        const uint32_t off = i * 1024 + lane * 16;
        if (off < CIMG) *reinterpret_cast<uint4*>(img + off) = g.v[i];
    }
    wave_lds_order();
}

// the count for tile t from entry E (a tile offset; NONE: guess it); the count image is in LDS.
// The guess: where the walk over the PRE bytes before the tile leaves them.
NXG_DEV FaDesc count_tile(lds_bytes img, uint64_t t, uint64_t W, uint32_t E, uint32_t lane,
                          uint64_t& obits, uint64_t* prof = nullptr) {
    const uint64_t t0 = t * TILE;
    const uint32_t lim = PRE + (uint32_t)min<uint64_t>(TILE, W - t0);
    const uint32_t wl = PRE + (uint32_t)min<uint64_t>(W - t0, 0xffffffffull - PRE);
    const uint32_t c = PRE + lane * CH, end = min(c + CH, lim);
    uint32_t first, rkids = 0;
    uint64_t rbits = 0, rabits = 0;
    const uint32_t g = c < lim ? spec_walk(img, c, c, end, wl, first, item_cands((lds_bytes)img, c),
                                           rbits, rkids, rabits)
                               : c;
    FAP(1);
    uint32_t ge = 0;
    if (E == NONE) {
        // the walk over the PRE / 64 chunks before the tile: lane q walks chunk q, all at once;
        // then from the first chunk's exit on: an exit that is an item of the next chunk's last
        // unbroken run continues as that run (the exact walk from there is that run), anything
        // else is walked on by lane 0 (rare: the walks merge within an item or two)
        constexpr uint32_t NQ = PRE / CH;
        static_assert(PRE % CH == 0 && NQ >= 1 && NQ <= 8, "whole chunks before the tile");
        uint32_t fq = 0, kq = 0;
        uint64_t bq = 0, aq = 0;
        if (lane < NQ) {
            const uint32_t cb = lane * CH;
            ge = spec_walk(img, cb, cb, cb + CH, wl, fq, item_cands((lds_bytes)img, cb), bq, kq, aq);
        }
        uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)ge, 0);
#pragma unroll 1
        for (uint32_t q = 1; q < NQ; q++) {
            const uint32_t cq = q * CH;
            if (x >= cq + CH) continue;  // an item covers chunk q
            const uint32_t fr = (uint32_t)__builtin_amdgcn_readlane((int)fq, (int)q);
            const uint64_t rb =
                (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bq, (int)q) |
                ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bq >> 32), (int)q)
                 << 32);
            if (x >= fr && ((rb >> (x - cq)) & 1ull)) {
                x = (uint32_t)__builtin_amdgcn_readlane((int)ge, (int)q);
                continue;
            }
            uint32_t f2 = 0, k2 = 0, g2 = 0;
            uint64_t b2 = 0, a2 = 0;
            if (lane == 0)
                g2 = spec_walk(img, x, cq, cq + CH, wl, f2, item_cands((lds_bytes)img, cq), b2, k2, a2);
            x = (uint32_t)__builtin_amdgcn_readlane((int)g2, 0);
        }
        E = x;
    } else {
        E += PRE;
    }
    FAP(2);
    // the lane's guessed entry: its predecessor's guessed exit (lane 0: E)
    const uint32_t gp = (uint32_t)__shfl_up((int)g, 1, 64);
    const uint32_t A = lane == 0 ? E : gp;
    uint32_t n = 0, kids = 0, brk = FAIL;
    uint64_t bits = 0;
    uint32_t X = A;
    if (A < end) {
        // entered at an item of the spec walk's last unbroken run: the exact walk from there is
        // that run (the same parses), so its counts are the run's
        const uint32_t d = A - c;
        if (d < 64 && ((rbits >> d) & 1ull) && (A == first || rkids == 0 || NXG_FA_RK)) {
            bits = rbits & (~0ull << d);
            n = (uint32_t)__popcll(bits);
            kids = rkids;
            if (NXG_FA_RK && A != first && rkids) {
                // the run's tail from A: the element counts of its Arrays at or after A
                kids = 0;
#pragma unroll 1
                for (uint64_t m = rabits & (~0ull << d); m; m &= m - 1)
                    kids += arr_count(img, c + (uint32_t)__builtin_ctzll(m));
            }
            X = g;
        } else {
#if NXG_FA_PROF
            if (prof) prof[9] += __popcll(__ballot(true));
#endif
            X = chunk_walk(img, A, c, end, wl, n, kids, bits, brk);
        }
    }
    FAP(3);
    const FaDesc r = chain_from(img, E, lim, wl, lane, A, X, n, kids, bits, brk, obits, prof);
    FAP(4);
    return r;
}

}  // namespace

// The exit at which the chain leaves tile t - 1 (t >= 1), by the whole wave (uniform), from the
// count pass's descriptors: the last tile before t whose entry is its predecessor's exit keeps
// its exit; each tile after it passes the chain on -- a tile one long item covers entirely (its
// true entry past its end) unchanged, a tile entered at its counted entry by its counted exit,
// and a tile entered elsewhere (the end of a long item that covered the tiles before it) by a
// recount from its true entry, as the wave that owns it does. FAIL: the chain breaks on the way.
// Lets a wave's first tile see past the previous wave's recounts (long text across waves).
NXG_DEV uint32_t exit_before(const uint8_t* __restrict__ buf, uint64_t W, const FaDesc* td,
                             uint64_t t, uint8_t* img, uint32_t lane) {
    uint64_t k = t - 1;
#pragma unroll 1
    for (uint32_t back = 0; k > 0 && back < 64; back++, k--) {
        const FaDesc a = td[k], b = td[k - 1];
        if (b.exit != FAIL && !(b.items & BROKEN) && b.exit - TILE == a.entry) break;
    }
    uint32_t x = td[k].exit;
    if (td[k].items & BROKEN) return FAIL;
#pragma unroll 1
    for (k = k + 1; k < t && x != FAIL; k++) {
        const uint32_t e = x - TILE;  // tile k's true entry
        if (e >= TILE) {
            x = e;  // covered: no item starts in tile k
            continue;
        }
        const FaDesc a = td[k];
        if (e == a.entry && !(a.items & BROKEN)) {
            x = a.exit;
            continue;
        }
        CountRegs g;
        count_load(g, buf, k * TILE, W, lane);
        count_store(img, g, lane);
        uint64_t bits;
        const FaDesc r = count_tile((lds_bytes)img, k, W, e, lane, bits);
        x = (r.items & BROKEN) ? FAIL : r.exit;
    }
    return x;
}

// count pass: one wave per tile
__global__ __launch_bounds__(TPB) void nxg_fa_count_kernel(const uint8_t* __restrict__ buf,
                                                           uint64_t W, uint64_t nt, uint32_t p0,
                                                           FaDesc* __restrict__ td,
                                                           uint64_t* __restrict__ starts) {
    __shared__ __attribute__((aligned(16))) FaCountLds lds[TPB / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t t = (uint64_t)blockIdx.x * (TPB / 64) + w;
    if (t >= nt) return;
    uint8_t* img = lds[w].img;
#if NXG_FA_PROF
    uint64_t pacc[16] = {};
    uint64_t* prof = pacc;
    prof[15] = __builtin_amdgcn_s_memtime();
#else
    uint64_t* prof = nullptr;
#endif
    CountRegs g;
    count_load(g, buf, t * TILE, W, lane);
    count_store(img, g, lane);
    FAP(0);
    uint64_t bits;
    const FaDesc d = count_tile((lds_bytes)img, t, W, t == 0 ? p0 : NONE, lane, bits, prof);
    starts[t * 64 + lane] = bits;
    if (lane == 0) td[t] = d;
#if NXG_FA_PROF
    pacc[8] = 1;
    if (lane == 0)
        for (int k = 0; k < 12; k++) atomicAdd(&nxg_fa_prof[k], (unsigned long long)pacc[k]);
#endif
}
#if NXG_FA_PROF
extern "C" int nxg_debug_fa_prof(unsigned long long* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(nxg_fa_prof), sizeof(nxg_fa_prof), 0,
                                    hipMemcpyDeviceToHost);
}
#endif

#ifndef NXG_FA_FIX_PASSES
#define NXG_FA_FIX_PASSES 2  // a second pass for tiles whose predecessor the first recounted (fix 69 -> 2 x 64, resolve 134 -> 52 us)
#endif
// fix: one wave per tile, all tiles at once. A tile whose guessed entry is not its predecessor's
// counted exit is recounted from that exit. A false guess almost always merges into the true
// chain inside its tile, so the counted exits are right and these recounts are independent: done
// here in parallel instead of one after another in the resolve pass's waves (942 of 46,598 tiles
// at 10^7 items). A predecessor being recounted at the same moment may be read before or after
// its rewrite: every descriptor written is a complete count from some entry, and the resolve
// pass checks the chain and recounts in order whatever still disagrees.
__global__ __launch_bounds__(TPB) void nxg_fa_fix_kernel(const uint8_t* __restrict__ buf,
                                                         uint64_t W, uint64_t nt,
                                                         FaDesc* __restrict__ td,
                                                         uint64_t* __restrict__ starts) {
    __shared__ __attribute__((aligned(16))) FaCountLds lds[TPB / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t t = (uint64_t)blockIdx.x * (TPB / 64) + w;
    if (t == 0 || t >= nt) return;
    const uint32_t px = __builtin_amdgcn_readfirstlane(td[t - 1].exit);
    const uint32_t pi = __builtin_amdgcn_readfirstlane(td[t - 1].items);
    const uint32_t e = __builtin_amdgcn_readfirstlane(td[t].entry);
    if (px == FAIL || (pi & BROKEN) || px - TILE == e || px - TILE >= TILE) return;
    uint8_t* img = lds[w].img;
    CountRegs g;
    count_load(g, buf, t * TILE, W, lane);
    count_store(img, g, lane);
    uint64_t bits;
    const FaDesc d = count_tile((lds_bytes)img, t, W, px - TILE, lane, bits);
    starts[t * 64 + lane] = bits;
    if (lane == 0) td[t] = d;
}

// The fix pass with a lane per tile (NXG_FA_FIXW): a wave checks 64 tiles as nxg_fa_fix_kernel
// checks one, and recounts the ones that disagree one after another -- 64x fewer waves launched
// than tiles, for the ~2 % of tiles that need it.
#ifndef NXG_FA_FIXW
#define NXG_FA_FIXW 0  // (A/B at 10^7 items: the serial recounts cost 227 us against 94 for a wave per tile)
#endif
__global__ __launch_bounds__(TPB) void nxg_fa_fixw_kernel(const uint8_t* __restrict__ buf,
                                                          uint64_t W, uint64_t nt,
                                                          FaDesc* __restrict__ td,
                                                          uint64_t* __restrict__ starts) {
    __shared__ __attribute__((aligned(16))) FaCountLds lds[TPB / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t t0 = ((uint64_t)blockIdx.x * (TPB / 64) + w) * 64;
    if (t0 >= nt) return;
    const uint64_t tl = t0 + lane;
    uint32_t pe = FAIL;
    if (tl > 0 && tl < nt) {
        const uint32_t px = td[tl - 1].exit, pi = td[tl - 1].items, e = td[tl].entry;
        if (!(px == FAIL || (pi & BROKEN) || px - TILE == e || px - TILE >= TILE)) pe = px - TILE;
    }
    uint8_t* img = lds[w].img;
#pragma unroll 1
    for (uint64_t m = __ballot(pe != FAIL); m; m &= m - 1) {
        const uint32_t j = (uint32_t)__builtin_ctzll(m);
        const uint64_t t = t0 + j;
        const uint32_t ej = (uint32_t)__builtin_amdgcn_readlane((int)pe, (int)j);
        CountRegs g;
        count_load(g, buf, t * TILE, W, lane);
        count_store(img, g, lane);
        uint64_t bits;
        const FaDesc d = count_tile((lds_bytes)img, t, W, ej, lane, bits);
        starts[t * 64 + lane] = bits;
        if (lane == 0) td[t] = d;
    }
}

// resolve: a lane per tile. A tile whose entry is not its (unbroken) predecessor's exit is
// recounted from that exit by its wave; then block scans of (items | child slots << 32) give each
// tile its offset in the block (tloc), and the last block to arrive (FaHead.arrived) scans the
// block sums (bpre). The chain itself is checked by the emit pass.
__global__ __launch_bounds__(TPB) void nxg_fa_resolve_kernel(
    const uint8_t* __restrict__ buf, uint64_t W, uint64_t nt, const FaDesc* __restrict__ td,
    FaDesc* __restrict__ td2, uint64_t* __restrict__ starts, uint64_t* __restrict__ tloc,
    uint64_t* __restrict__ bsum, uint64_t* __restrict__ bpre, uint64_t* __restrict__ wexit,
    FaHead* __restrict__ hp) {
    __shared__ __attribute__((aligned(16))) FaCountLds lds[TPB / 64];
    __shared__ uint64_t scan_tmp[TPB / 64];
    __shared__ uint32_t is_last;
    __shared__ uint32_t sh_tile;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // blocks by ticket: a wave waits only on waves that are running
    const uint32_t bid = next_tile((unsigned long long*)&hp->ticket, &sh_tile);
    const uint64_t tl = (uint64_t)bid * TPB + threadIdx.x;
    FaDesc d{FAIL, FAIL, BROKEN, 0};
    bool mis = false;
    uint8_t* img = lds[w].img;
    // the exit the chain leaves the wave's previous tile at (FAIL: unknown), by the whole wave
    const uint64_t tw = tl - lane;  // the wave's first tile
    uint32_t px0 = tw > 0 && tw < nt ? exit_before(buf, W, td, tw, img, lane) : FAIL;
    if (tw > 0 && tw < nt && px0 == FAIL) {
        // no tile of the count pass to start from within 64 (a batch of long text: nearly every
        // tile starts inside one): the previous wave's exit after its recounts, which it
        // publishes below. Only lower-numbered waves are waited on (dispatched earlier, so
        // resident or done); on the watchdog the emit pass's chain check fails the batch.
        const uint64_t t_start = rt_now();
        uint64_t v = ld_agent(&wexit[tw / 64 - 1]);
        uint32_t polls = 0;
#pragma unroll 1
        while (!(v >> 63) && !spin_expired(t_start, ++polls)) {
            __builtin_amdgcn_s_sleep(2);
            v = ld_agent(&wexit[tw / 64 - 1]);
        }
        px0 = (v >> 63) && !((v >> 62) & 1ull) ? (uint32_t)v : FAIL;
    }
    if (tl < nt) {
        d = td[tl];
        if (lane == 0) {
            mis = tl > 0 && px0 != FAIL && px0 - TILE != d.entry;
        } else {
            const FaDesc pd = td[tl - 1];
            mis = pd.exit != FAIL && !(pd.items & BROKEN) && pd.exit - TILE != d.entry;
        }
    }
    const uint64_t m = __ballot(mis);
    if (m) {
        // in tile order from the first mismatch: a tile is recounted when its entry is not its
        // predecessor's exit as it stands after the predecessor's own recount (a long item that
        // covers whole tiles moves the exits of the tiles after it)
        const uint32_t j0 = (uint32_t)__builtin_ctzll(m);
        uint32_t nrc = 0;
#pragma unroll 1
        for (uint32_t j = j0; j < 64 && tw + j < nt; j++) {
            const uint64_t t = tw + j;
            uint32_t px, pi;
            if (j == 0) {  // t >= 1: lane 0 of wave 0 never mismatches
                px = px0;
                pi = 0;
            } else {
                px = (uint32_t)__builtin_amdgcn_readlane((int)d.exit, (int)(j - 1));
                pi = (uint32_t)__builtin_amdgcn_readlane((int)d.items, (int)(j - 1));
            }
            const uint32_t ej = (uint32_t)__builtin_amdgcn_readlane((int)d.entry, (int)j);
            if (px == FAIL || (pi & BROKEN) || px - TILE == ej) continue;
            CountRegs g;
            count_load(g, buf, t * TILE, W, lane);
            count_store(img, g, lane);
            uint64_t bits;
            const FaDesc r = count_tile((lds_bytes)img, t, W, px - TILE, lane, bits);
            starts[t * 64 + lane] = bits;
            if (lane == j) d = r;
            nrc++;
        }
        if (lane == 0) atomicAdd((unsigned long long*)&hp->recounts, (unsigned long long)nrc);
    }
    if (tl < nt) td2[tl] = d;
    {  // the exit the chain leaves the wave's last tile at, for the next wave (bit 62: broken)
        const uint32_t lx = (uint32_t)__builtin_amdgcn_readlane((int)d.exit, 63);
        const uint32_t li = (uint32_t)__builtin_amdgcn_readlane((int)d.items, 63);
        if (lane == 0 && tw < nt)
            st_agent(&wexit[tw / 64],
                     (1ull << 63) | ((li & BROKEN) || lx == FAIL ? 1ull << 62 : 0ull) | lx);
    }
    const uint64_t v = tl < nt ? (uint64_t)(d.items & ~BROKEN) | ((uint64_t)d.kids << 32) : 0ull;
    uint64_t tot;
    const uint64_t ex = block_excl_scan<uint64_t, TPB>(v, scan_tmp, &tot);
    if (tl < nt) tloc[tl] = ex;
    if (threadIdx.x == 0) {
        st_agent(&bsum[bid], tot);
        drain_stores();
        is_last = atomicAdd(&hp->arrived, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!is_last) return;
    const uint32_t nb = gridDim.x;
    uint64_t run = 0;
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < nb; b0 += TPB) {
        const uint32_t b = b0 + threadIdx.x;
        const uint64_t x = b < nb ? ld_agent(&bsum[b]) : 0ull;
        uint64_t t2;
        const uint64_t e2 = block_excl_scan<uint64_t, TPB>(x, scan_tmp, &t2);
        if (b < nb) bpre[b] = run + e2;
        run += t2;
    }
    if (threadIdx.x == 0) {
        hp->items = run & 0xffffffffull;
    }
}

// emit: one wave per tile that holds rows < count
#ifndef NXG_FA_EOCC
#define NXG_FA_EOCC 1  // waves per SIMD asked of the emit's register allocation (LDS allows 5)
#endif
__global__ __launch_bounds__(TPB, NXG_FA_EOCC) void nxg_fa_emit_kernel(
    const uint8_t* __restrict__ buf, uint64_t W, uint64_t nt, uint32_t p0, uint64_t count,
    const FaDesc* __restrict__ td, const uint64_t* __restrict__ tloc,
    const uint64_t* __restrict__ bpre, const uint64_t* __restrict__ starts, ColsDesc cols,
    FaHead* __restrict__ hp, DevStatus* __restrict__ st) {
    __shared__ __attribute__((aligned(16))) FaEmitLds lds[TPB / 64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t t = (uint64_t)blockIdx.x * (TPB / 64) + w;
    if (t >= nt) return;
    const uint64_t base = bpre[t / TPB] + tloc[t];
    const uint64_t rb = base & 0xffffffffull;
    if (rb >= count) return;  // past the batch
    uint8_t* img = lds[w].img;
    uint16_t* msg = lds[w].msg;
    uint32_t* el = lds[w].el;
    const lds_bytes limg = (lds_bytes)img;
    const uint64_t t0 = t * TILE;
    const uint32_t wl = (uint32_t)min<uint64_t>(W - t0, 0xffffffffull);
    const uint32_t elim = min(wl, IMGL);  // Array elements end before this
    TileRegs g;
    tile_load(g, buf, t0, W, lane);
    uint64_t bits = starts[t * 64 + lane];
    const FaDesc d = td[t];
    const uint32_t items = d.items & ~BROKEN;
    // the chain: entered at the predecessor's exit (tile 0 after the count); a tile that stops
    // (a break, or the window's end) must hold the batch's last item
    bool bad = d.entry == FAIL;
    if (t == 0) {
        bad |= d.entry != p0;
    } else {
        const FaDesc pd = td[t - 1];
        bad |= pd.exit == FAIL || (pd.items & BROKEN) || pd.exit - TILE != d.entry;
    }
    uint32_t why = bad ? 1u : 0u;
    if (rb + items < count && ((d.items & BROKEN) || t + 1 == nt)) bad = true, why |= 2u;
    const uint32_t nm = (uint32_t)min<uint64_t>(items, count - rb);  // the batch's items here
    uint64_t cnext = base >> 32;
    // a batch already declined by the resolve pass (a plain read: one scalar load per CU, not an
    // agent-scope load per wave on one address)
    if (NXG_FF_CHECK && hp->fast_fail) return;
    tile_store(img, g, lane);
    const uint32_t n0 = (uint32_t)__popcll(bits);
    uint32_t at = wave_incl_scan<uint32_t>(n0) - n0;
    if (wave_last<uint32_t>(at + n0) != items) bad = true, why |= 4u;
#pragma unroll 1
    while (bits) {
        msg[at++] = (uint16_t)(lane * CH + (uint32_t)__builtin_ctzll(bits));
        bits &= bits - 1;
    }
    wave_lds_order();
    uint32_t ntxt = 0;  // deferred text checks in el[0, ntxt)
#pragma unroll 1
    for (uint32_t k = 0; k < nm && !bad; k += 64) {
        const uint32_t i = k + lane;
        const bool has = i < nm;
        const uint32_t p = has ? msg[i] : 0u;
        // Id varint (at most 5 bytes: the count pass), the Event's first byte, then 12 bytes
        uint32_t h[5];
        win_words<5>(limg, p, h);
        const uint32_t a = h[0], b = h[1];
        const uint32_t sa = ~a & 0x80808080u;
        const uint32_t nb = sa ? ((uint32_t)__builtin_ctz(sa) >> 3) + 1 : 5u;
        const uint64_t id = (uint64_t)compress7_32(nb >= 4u ? a : (a & ((1u << (8u * nb)) - 1u))) |
                            (nb == 5u ? (uint64_t)(b & 0x7fu) << 28 : 0ull);
        const uint32_t tg = (uint32_t)(((((uint64_t)b << 32) | a) >> (8u * nb)) & 0xffu);
        const uint32_t u = nb + 1u;  // the payload, relative to p: 2..6
        const bool up = u >= 4u;
        const uint32_t g0 = up ? h[1] : h[0], g1 = up ? h[2] : h[1], g2 = up ? h[3] : h[2],
                       g3 = up ? h[4] : h[3];
        const uint32_t su = u & 3u;
        const bool un = tg == UNSUB;
        FV o = val_decode(un ? 1u : tg, alignbyte(g1, g0, su), alignbyte(g2, g1, su),
                          alignbyte(g3, g2, su), p + u, wl, true, t0);
        if (un) o = FV{0ull, UNSUB, 0u, p + u, 0u, 0u, 0u, true};
        // text past the image: checked from global memory; everything else ends in it
        const bool far = has && o.ok && o.end > IMGL;
        const bool arr = o.tag == 19u;
        bool ok = !has || ((sa != 0u || !(b & 0x80u)) && o.ok && (!far || !arr) &&
                           (!arr || o.end <= elim));
        {  // (text past the image: the whole wave, one text after the other)
            const bool fw = far && ok && o.slen;
            const bool fo = far_text_ok(buf, fw, t0 + o.soff, o.slen, lane);
            if (fw) ok = fo;
        }
        bad = __any(!ok);
        if (bad) why |= 8u | (__any(has && !o.ok) ? 16u : 0u) | (__any(far && arr) ? 32u : 0u);
        if (!bad) {
            const bool tx = has && !far && o.slen;
            const uint64_t tm = __ballot(tx);
            const uint32_t tn = (uint32_t)__popcll(tm);
            if (ntxt + tn > MAXC) {
                bad = !text_flush(limg, el, ntxt, lds[w].mark, lane, st);
                if (bad) why |= 64u;
                ntxt = 0;
                wave_lds_order();
            }
            if (tx)
                el[ntxt + __builtin_amdgcn_mbcnt_hi((uint32_t)(tm >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)tm, 0u))] =
                    o.soff | (o.slen << 16);
            ntxt += tn;
        }
        if (bad) break;
        const uint32_t kd = has ? o.kids : 0u;
        const uint32_t kinc = wave_incl_scan<uint32_t>(kd);
        const uint32_t kpre = kinc - kd;
        const uint32_t rk = wave_last<uint32_t>(kinc);
        if (cnext + rk > cols.cap_children) {  // the exact decoder reports the capacity error
            bad = true;
            why |= 128u;
            break;
        }
        const uint64_t row = rb + i;
        if (has) {
            col_st(&cols.id[row], (uint64_t)(uint32_t)id);  // Id(decode_varint as u32) (logfile/mod.rs:162-164)
            col_st(&cols.tag[row], (uint8_t)o.tag);
            col_st(&cols.fixed[row], (uint64_t)(arr ? cnext + kpre : o.fixed));
            col_st(&cols.aux[row], (uint32_t)o.aux);
            if (row + 1 == count) {  // the batch's last item: where it ends
                const uint32_t nx = i + 1 < items ? (uint32_t)msg[i + 1] : d.exit;
                hp->end = t0 + nx + 1;
                hp->end_children = cnext + kpre + kd;
            }
        }
        if (rk) {
            bad = round_elements(img, lds[w].mark, el, kd, kpre, rk, o.end, elim, cnext, cols, t0,
                                 lane, ntxt, st);
            if (bad) {
                why |= 256u;
                break;
            }
        }
        cnext += rk;
    }
    if (!bad && ntxt) {
        bad = !text_flush(limg, el, ntxt, lds[w].mark, lane, st);
        if (bad) why |= 512u;
    }
    if (bad && lane == 0) {
        atomicOr(&hp->fast_fail, 1u);
        atomicOr((unsigned long long*)&hp->why, (unsigned long long)why);
        // the first declining tile and its reasons: ~t << 16 | why, kept by the maximum
        atomicMax((unsigned long long*)&hp->why_tile,
                  ((unsigned long long)(~t & 0xffffffffffffull) << 16) | (why & 0xffffu));
    }
}

// ---- launch (host) --------------------------------------------------------------------------------
uint64_t nxg_fa_scratch_bytes(uint64_t W) {
    const uint64_t nt = (W + TILE - 1) / TILE;
    // head 64 B; 2 descs 32 B, starts 512 B, tloc 8 B per tile; bsum + bpre 16 B per 256
    // tiles; one exit word per 64 tiles
    return 64 + nt * 552 + 16 * (nt / TPB + 1) + 8 * (nt / 64 + 1) + 7 * 16;
}

// One pass of the fast path over buf[0, W) (W < 2^32; the batch's count and its varint's length
// p0 parsed by the host). `scratch`: nxg_fa_scratch_bytes(W) bytes; its first 64 (the FaHead) are
// zeroed here, the rest needs no initialisation. The FaHead goes to `hhead` (host, pinned) when
// the stream reaches it.
hipError_t nxg_launch_dec_fa(const uint8_t* buf, uint64_t W, uint32_t p0, uint64_t count,
                             const ColsDesc& cols, uint8_t* scratch, void* hhead,
                             DevStatus* st, hipStream_t s) {
    const uint64_t nt = (W + TILE - 1) / TILE;
    uint8_t* p = scratch;
    auto take = [&](uint64_t bytes) {
        uint8_t* r = p;
        p += (bytes + 15) & ~15ull;
        return r;
    };
    FaHead* hp = reinterpret_cast<FaHead*>(take(sizeof(FaHead)));
    FaDesc* td = reinterpret_cast<FaDesc*>(take(16 * nt));
    FaDesc* td2 = reinterpret_cast<FaDesc*>(take(16 * nt));
    uint64_t* starts = reinterpret_cast<uint64_t*>(take(512 * nt));
    uint64_t* tloc = reinterpret_cast<uint64_t*>(take(8 * nt));
    const uint64_t nb = (nt + TPB - 1) / TPB;
    uint64_t* bsum = reinterpret_cast<uint64_t*>(take(8 * nb));
    uint64_t* bpre = reinterpret_cast<uint64_t*>(take(8 * nb));
    const uint64_t nwv = (nt + 63) / 64;
    uint64_t* wexit = reinterpret_cast<uint64_t*>(take(8 * nwv));
    hipError_t e;
    if ((e = hipMemsetAsync(hp, 0, sizeof(FaHead), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(wexit, 0, 8 * nwv, s)) != hipSuccess) return e;
    constexpr uint64_t WV = TPB / 64;
    const uint32_t gc = (uint32_t)((nt + WV - 1) / WV);
    hipLaunchKernelGGL(nxg_fa_count_kernel, dim3(gc), dim3(TPB), 0, s, buf, W, nt, p0, td, starts);
    // (a second pass would catch the tiles whose predecessor the first one recounted)
    for (int k = 0; k < NXG_FA_FIX_PASSES; k++) {
        if (NXG_FA_FIXW)
            hipLaunchKernelGGL(nxg_fa_fixw_kernel, dim3((uint32_t)((nt + 255) / 256)), dim3(TPB), 0,
                               s, buf, W, nt, td, starts);
        else
            hipLaunchKernelGGL(nxg_fa_fix_kernel, dim3(gc), dim3(TPB), 0, s, buf, W, nt, td,
                               starts);
    }
    hipLaunchKernelGGL(nxg_fa_resolve_kernel, dim3((uint32_t)nb), dim3(TPB), 0, s, buf, W, nt, td,
                       td2, starts, tloc, bsum, bpre, wexit, hp);
    hipLaunchKernelGGL(nxg_fa_emit_kernel, dim3(gc), dim3(TPB), 0, s, buf, W, nt, p0, count, td2,
                       tloc, bpre, starts, cols, hp, st);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return hipMemcpyAsync(hhead, hp, sizeof(FaHead), hipMemcpyDeviceToHost, s);
}
