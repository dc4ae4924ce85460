// nxg_decode_gen.hip -- general From-stream decode for gfx950: every From variant, every Value
// tag, nesting, errors. Replaces the receive_batch_fn loop (netidx/src/channel.rs:504-521) for
// frames the homogeneous-f64 kernels do not take.
//
// Message boundaries form a pointer chain (len_wrapped_decode, pack.rs:537-555): a message's
// length prefix says where the next one starts. The chain is followed in parallel, with the
// same run structure as the f64 decoder (nxg_decode_f64.hip):
//
//   count    wave v owns a contiguous run of 4 KiB tiles. In each tile, lane j owns the 64-byte
//            chunk j. Every lane guesses the first message start in its chunk, walks and
//            validates the messages that start there, and the wave then checks that lane j's
//            start is exactly the exit of the nearest lane below it that has a start; a lane
//            that disagrees re-walks from that exit (exact repair, one lane per round). The
//            first tile of a run has a guessed entry; each later tile's entry is the previous
//            tile's exit, so only a run's first entry is ever speculative. Per tile and lane the
//            wave stores one word (start offset, rows, control messages, children); per run, a
//            summary (guessed entry, exit, totals, first error).
//   resolve  one workgroup: checks that each run's guessed entry is the previous run's exit and
//            re-walks, in order, any run whose guess was wrong (its per-lane words are
//            rewritten); finds the first error on the true chain; prefix sums of the run totals.
//   emit     the same runs again: each lane decodes its messages from the stored start and
//            writes the columns at the bases from the prefix sums.
//
// The frame fails with the first error on the true chain, (PackError kind, offset of the
// failing message), as the sequential reference stops at its first error
// (netidx/src/subscriber/connection.rs:228-231).
// (the resolve pass runs 8 waves per workgroup; each wave may decode values)
#define NXG_DV_WAVES 8
#include "nxg_msg.h"

using namespace nxgmsg;

namespace {

constexpr int TPB = gdec2::TPB;
constexpr int WAVES = TPB / 64;
constexpr int CH = gdec2::CH;
constexpr uint32_t TILE = gdec2::TILE;
constexpr uint32_t IMG = gdec2::IMG;
constexpr uint64_t NONE = ~0ull;
constexpr uint32_t NOSTART = 127u;  // lane word: no message starts in the chunk
constexpr uint32_t CH_ESC = 8191u;  // lane word: children count did not fit (recount in emit)

// lane word: start offset (7 bits) | rows (6) | control messages (6) | children (13)
NXG_DEV uint32_t lw_pack(uint32_t off, uint32_t rows, uint32_t ctl, uint64_t ch) {
    return off | (rows << 7) | (ctl << 13) | ((uint32_t)(ch < CH_ESC ? ch : CH_ESC) << 19);
}
NXG_DEV uint32_t lw_off(uint32_t w) { return w & 127u; }
NXG_DEV uint32_t lw_rows(uint32_t w) { return (w >> 7) & 63u; }
NXG_DEV uint32_t lw_ctl(uint32_t w) { return (w >> 13) & 63u; }
NXG_DEV uint32_t lw_ch(uint32_t w) { return w >> 19; }

// run summary words
enum { R_SPEC = 0, R_EXIT, R_ROWS, R_CH, R_CTL, R_ERR, R_FIXED, R_PAD, R_WORDS };
static_assert(R_WORDS == gdec2::RUN_WORDS, "run summary");
// R_ERR: kind << 56 | offset (0 = none). R_SPEC: NONE when the run holds no message start.

constexpr uint64_t POSM = (1ull << 56) - 1;

// lane states
enum { S_NONE = 0, S_EXH = 1, S_OK = 2, S_ERR = 3 };

struct LaneRes {
    uint64_t x;  // exit (first message start at/after the chunk end), or the failing message
    uint32_t rows, ctl, hb;
    uint64_t children;
    uint32_t st;
    uint32_t ek;
};

// Structural walk of the messages that start in [e, end) (skim_msg: lengths, variants, child
// slots). Only a broken length prefix is an error here; content errors are the emit pass's.
NXG_DEV void walk(const Src& s, uint64_t e, uint64_t end, LaneRes& r, uint32_t budget) {
    r.x = e;
    r.rows = r.ctl = r.hb = 0;
    r.children = 0;
    r.st = S_OK;
    r.ek = 0;
    uint64_t pos = e;
    const uint64_t stop = end < s.W ? end : s.W;
    uint32_t work = 0;
#pragma unroll 1
    while (pos < stop) {
        MsgInfo mi;
        uint64_t ch = 0;
        const uint32_t err = skim_msg(s, pos, mi, ch, work, budget);
        if (err == E_BUDGET) {
            r.st = S_EXH;
            return;
        }
        if (err) {
            r.st = S_ERR;
            r.ek = err;
            r.x = pos;
            return;
        }
        if (mi.variant == 4) r.rows++;
        else r.ctl++;
        r.hb += mi.variant == 5;
        r.children += ch;
        pos = mi.next;
    }
    r.x = pos;
}

// Structural plausibility of an Update at p with an nb-byte length prefix L (minimal): the
// Update variant is already matched by the caller. Checks that the id varint and the value tag
// fit in the message, that a fixed-size value fills it exactly, and that the next position
// looks like a message start (length >= 2, variant <= 6) or is the frame end. Only the
// candidate's own bytes are guaranteed to be in the LDS image.
NXG_DEV bool plausible(const Src& s, uint64_t p, uint32_t nb, uint64_t L) {
    const uint64_t next = p + L;  // total size = nb + L - vl(L) = L for a minimal prefix
    if (next > s.W) return false;
    uint64_t q = p + nb + 1;  // id varint
    uint32_t k = 0;
    while (k < 10 && q + k < next && (s.img_byte(q + k) & 0x80u)) k++;
    const uint64_t tp = q + k + 1;  // value tag
    if (k == 10 || tp >= next) return false;
    const uint32_t t = s.img_byte(tp);
    if (t >= 28u) return false;
    const uint32_t f1 = fixed_size1(t);
    if (f1 && tp + f1 != next) return false;
    const bool vint = t == 1 || t == 3 || t == 5 || t == 7;
    const bool text = t == 12 || t == 13 || t == 18;
    if (vint || text) {  // the varint payload, or text length + text, fills the message exactly
        uint64_t v = 0, a = tp + 1;
        uint32_t i = 0, b;
        do {
            if (a + i >= next || i == 10) return false;
            b = s.any_byte(a + i);
            v |= (uint64_t)(b & 0x7fu) << (7 * i);
            i++;
        } while (b & 0x80u);
        if ((vint ? a + i : a + i + v) != next) return false;
    }
    if (t == 19) {  // Array: an empty one ends the message, elements fit, the first tag is valid
        uint64_t v = 0, a = tp + 1;
        uint32_t i = 0, b;
        do {
            if (a + i >= next || i == 10) return false;
            b = s.any_byte(a + i);
            v |= (uint64_t)(b & 0x7fu) << (7 * i);
            i++;
        } while (b & 0x80u);
        if (v == 0 ? a + i != next : (a + i + v > next || s.any_byte(a + i) >= 28u)) return false;
    }
    if (next == s.W) return true;
    if (next + 2 > s.W) return false;  // no room for a message (>= 2 bytes)
    const uint32_t b0 = s.any_byte(next);
    uint32_t v;
    if (b0 < 0x80u) {
        if (b0 < 2u) return false;
        v = s.any_byte(next + 1);
    } else {
        if (next + 3 > s.W) return false;
        const uint32_t b1 = s.any_byte(next + 1);
        if (b1 == 0u || b1 >= 0x80u) return false;
        v = s.any_byte(next + 2);
    }
    return v <= 6u;
}

// First position in [c, stop) that starts a plausible Update (see plausible). Candidates come
// from a SWAR scan for the Update variant byte (4) one or two bytes after a 1- or 2-byte length
// varint. Only Updates are guessed: a Heartbeat or Unsubscribed accepts almost any bytes; a
// chunk that starts with one, or a wrong guess, is resolved exactly by the repair.
NXG_DEV uint64_t speculate(const Src& s, uint64_t c, uint64_t stop, uint32_t& tries) {
    if (c >= stop) return NONE;
    const uint64_t rc = c - s.t0;  // 64-aligned, inside the image with 68 bytes to spare
    lds_words w = (lds_words)(s.lds + rc);
    uint64_t e4 = 0;  // bit q: byte c+1+q == 4, q in [0, 64)
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint32_t x = alignbyte(w[k + 1], w[k], 1);  // bytes c+4k+1 .. c+4k+4
        e4 |= (uint64_t)nib(zero_bytes(x ^ 0x04040404u)) << (4 * k);
    }
    const uint32_t x16 = alignbyte(w[17], w[16], 1);  // byte c+65 (for 2-byte-length starts)
    bool e4_64 = (x16 & 0xffu) == 4u;
#pragma unroll 1
    while (e4 || e4_64) {
        uint32_t q;  // variant byte at c+1+q
        if (e4) {
            q = (uint32_t)__builtin_ctzll(e4);
            e4 &= e4 - 1;
        } else {
            q = 64;
            e4_64 = false;
        }
        // p = c+q: 1-byte length (4..127) then the variant; p = c+q-1: 2-byte length. The
        // 1-byte form goes first: a 2-byte "shadow" (a payload byte >= 0x80 just before a true
        // 1-byte length) shares its variant byte, and only one of the two can be a start.
        for (int form = 1; form >= 0; form--) {
            const int64_t pr = form == 0 ? (int64_t)q - 1 : (int64_t)q;
            if (pr < 0) continue;
            const uint64_t p = c + (uint64_t)pr;
            if (p >= stop) continue;
            const uint32_t b0 = s.img_byte(p);
            uint64_t L;
            if (form == 0) {  // 2-byte length: b0 >= 128, next byte 1..127, then 4
                const uint32_t b1 = s.img_byte(p + 1);
                if (b0 < 0x80u || b1 == 0u || b1 >= 0x80u) continue;
                L = (b0 & 0x7fu) | (b1 << 7);
            } else {
                if (b0 < 4u || b0 >= 0x80u) continue;
                L = b0;
            }
            tries++;
            if (plausible(s, p, form == 0 ? 2u : 1u, L)) return p;
        }
    }
    return NONE;
}

struct TileOut {
    uint64_t anchor;  // entry the tile assumed: the given entry, or the first guess (NONE: none)
    uint64_t exit;    // first message start at/after the tile end (error: the failing message)
    uint32_t ek;      // error kind on the chain, 0 = none
    uint64_t rows, ch, ctl, hb;
    uint32_t rounds;
    uint64_t why;  // repairs by cause, 16 bits each: exhausted, wrong guess, missed, spurious
};

// Resolve one tile (its bytes are in the wave's LDS image `s`). `entry` is the exact first
// message start at/after the tile start, or NONE (guess it). Sets this lane's word (lwo)
// and returns the tile's totals. Wave-level: no block barriers.
NXG_DEV TileOut process_tile(const Src& s, uint64_t t0, uint64_t entry, uint32_t& lwo,
                             uint32_t& tries) {
    const uint32_t lane = __lane_id();
    const uint64_t W = s.W;
    TileOut to{entry, entry, 0, 0, 0, 0, 0, 0};
    if (entry != NONE && (entry >= t0 + TILE || entry >= s.W)) {  // inside one message, or done
        lwo = NOSTART;
        return to;
    }
    const uint64_t c = t0 + (uint64_t)lane * CH, cend = c + CH;
    const uint64_t stop = cend < W ? cend : W;  // message starts are positions < W
    bool has = false;
    uint64_t e = NONE;
    if (entry != NONE && entry >= c) {
        has = entry < stop;  // the anchor lane (lanes before it: no start)
        e = has ? entry : NONE;
    } else {
        e = speculate(s, c, stop, tries);
        has = e != NONE;
    }
    // anchor = the lane holding the entry, else the first lane with a guess
    uint32_t a;
    if (entry != NONE) {
        a = (uint32_t)((entry - t0) / CH);
    } else {
        const uint64_t m = __ballot(has);
        if (!m) {  // no guess anywhere: assume the tile lies inside one message
            lwo = NOSTART;
            to.anchor = NONE;
            to.exit = NONE;
            return to;
        }
        a = (uint32_t)__builtin_ctzll(m);
    }
    if (lane < a) has = false;
    to.anchor = __shfl(e, (int)a, 64);
    LaneRes r{e, 0, 0, 0, 0, S_NONE, 0};
    // Round 1 walks every lane with a start (the anchor exactly when its entry is known, the
    // guesses with a budget). Each later round repairs one lane, in lane order: lane j > a is
    // consistent when, with x the exit of the nearest lane below it that has a start, x < stop_j
    // and j starts exactly at x, or x >= stop_j and j has no start. Events: the first
    // inconsistent lane (re-walked from x, or cleared), a consistent lane whose bounded walk ran
    // out of budget (re-walked exactly), a consistent lane whose walk failed (the tile's error:
    // everything after it is moot).
    const uint64_t lt = (1ull << lane) - 1;
    const uint64_t from_a = ~0ull << a;
    int errlane = -1;
    uint32_t rounds = 0;
    bool need = has;
    uint32_t budget = (lane == a && entry != NONE) ? kExact.budget : kBounded.budget;
#pragma unroll 1
    for (;;) {
        if (need) walk(s, e, cend, r, budget);
        need = false;
        if (++rounds > 2 * 64 + 4) {
            errlane = -2;  // logic error guard: reported as a timeout, never a hang
            break;
        }
        const uint64_t m = __ballot(has);
        const uint64_t below = m & lt;
        const int pi = below ? 63 - __builtin_clzll(below) : (int)lane;
        const uint64_t px = __shfl(r.x, pi, 64);
        const uint32_t pst = __shfl(r.st, pi, 64);
        bool cons = true;
        if (lane > a && below && pst == S_OK) cons = px < stop ? (has && e == px) : !has;
        const bool ev_exh = cons && has && r.st == S_EXH;
        const bool ev_err = cons && has && r.st == S_ERR;
        const uint64_t fm = __ballot((!cons) || ev_exh || ev_err) & from_a;
        if (!fm) break;
        const int bl = __builtin_ctzll(fm);
        if (__shfl((uint32_t)ev_err, bl, 64)) {
            errlane = bl;
            break;
        }
        const uint32_t cause = ev_exh ? 0u : (px < stop ? (has ? 1u : 2u) : 3u);
        to.why += 1ull << (16 * __shfl(cause, bl, 64));
        if ((int)lane == bl) {
            budget = kExact.budget;
            if (ev_exh) {
                need = true;
            } else if (px < stop) {
                has = true;
                e = px;
                need = true;
            } else {
                has = false;
                e = NONE;
                r.st = S_NONE;
            }
        }
    }
    to.rounds = rounds;
    if (errlane == -2) {
        to.ek = NXG_TIMEOUT;
        to.exit = 0;
        lwo = NOSTART;
        return to;
    }
    // With a broken length prefix in lane errlane, that lane stays live: the emit pass decodes
    // its messages up to and including the broken one, so a content error earlier in the lane
    // still wins.
    bool live = has;
    if (errlane >= 0) {
        live = has && (int)lane <= errlane;
        to.ek = __shfl(r.ek, errlane, 64);
        to.exit = __shfl(r.x, errlane, 64);
    } else {
        const uint64_t m = __ballot(has);
        const int z = 63 - __builtin_clzll(m);  // lane a at least
        to.exit = __shfl(r.x, z, 64);
    }
    lwo = live ? lw_pack((uint32_t)(e - c), r.rows, r.ctl, r.children) : NOSTART;
    to.rows = wave_sum<uint64_t>(live ? r.rows : 0u);
    to.ctl = wave_sum<uint64_t>(live ? r.ctl : 0u);
    to.hb = wave_sum<uint64_t>(live ? r.hb : 0u);
    to.ch = wave_sum<uint64_t>(live ? r.children : 0ull);
    return to;
}

// ---- tile staging: 4 KiB + 1 KiB look-ahead per wave, 5 x 16 B per lane, zero past the end --
struct GRegs {
    uint4 v[5];
};
NXG_DEV uint4 ld16z(const uint8_t* __restrict__ wire, uint64_t off, uint64_t W) {
    if (off + 16 <= W) return *reinterpret_cast<const uint4*>(wire + off);
    uint32_t v[4] = {0, 0, 0, 0};
    for (int k = 0; k < 16; k++)
        if (off + k < W) v[k >> 2] |= (uint32_t)wire[off + k] << (8 * (k & 3));
    return make_uint4(v[0], v[1], v[2], v[3]);
}
NXG_DEV void g_load(GRegs& g, const uint8_t* __restrict__ wire, uint64_t t0, uint64_t W,
                    uint32_t lane) {
    if (t0 + IMG <= W) {
        const uint4* p = reinterpret_cast<const uint4*>(wire + t0);
#pragma unroll
        for (int i = 0; i < 5; i++) g.v[i] = p[i * 64 + lane];
    } else {
#pragma unroll
        for (int i = 0; i < 5; i++) g.v[i] = ld16z(wire, t0 + i * 1024 + lane * 16, W);
    }
}
NXG_DEV void g_stage(uint8_t* buf, const GRegs& g, uint32_t lane) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < 5; i++) *reinterpret_cast<uint4*>(buf + i * 1024 + lane * 16) = g.v[i];
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}
NXG_DEV Src g_src(const uint8_t* buf, const uint8_t* wire, uint64_t t0, uint64_t W) {
    const uint64_t n = W - t0;
    return Src{(lds_bytes)buf, t0, (uint32_t)(n < IMG ? n : IMG), (gbl_bytes)wire, W};
}

NXG_DEV uint64_t run_begin(uint64_t nt, uint32_t R, uint32_t r) { return nt * r / R; }

// First walk (or re-walk) of the tiles [b, e) of a run from `entry` (NONE: guessed). Lane words
// go to lws + 64*tile. Fills the run summary (in registers; lane 0 stores it).
//
// Re-walk (old_last != NONE): the run was walked before from a wrong entry and its lane words
// are valid for tiles up to old_last. As soon as some lane starts at the same position in both
// walks, the two message chains are the same from there on, so the re-walk stops (`merged`)
// and d[] holds the changes to the run's rows / children / control messages.
struct RunSum {
    uint64_t spec, exit, rows, ch, ctl, err;
    uint32_t rounds, tries;
    uint64_t why;
};
NXG_DEV RunSum run_tiles(const uint8_t* __restrict__ wire, uint64_t W, uint64_t b, uint64_t e,
                         uint64_t entry, uint32_t* __restrict__ lws, uint8_t* buf,
                         uint64_t old_last, bool& merged, int64_t* d) {
    const uint32_t lane = __lane_id();
    RunSum rs{NONE, entry, 0, 0, 0, 0, 0, 0};
    bool have_spec = entry != NONE;
    if (have_spec) rs.spec = entry;
    merged = false;
    bool cmp = old_last != NONE;
    int64_t dr = 0, dc = 0, dk = 0;
    GRegs g;
    if (b < e) g_load(g, wire, b * TILE, W, lane);
    uint64_t cur = entry;
#pragma unroll 1
    for (uint64_t t = b; t < e; t++) {
        const uint64_t t0 = t * TILE;
        g_stage(buf, g, lane);
        if (t + 1 < e) g_load(g, wire, (t + 1) * TILE, W, lane);
        const Src s = g_src(buf, wire, t0, W);
        uint32_t tries = 0;
        uint32_t lwv;
        const bool cmp_t = cmp && t <= old_last;
        const uint32_t ow = cmp_t ? lws[t * 64 + lane] : NOSTART;
        const TileOut to = process_tile(s, t0, cur, lwv, tries);
        lws[t * 64 + lane] = lwv;
        if (cmp_t && !to.ek) {
            const bool hn = lw_off(lwv) != NOSTART, ho = lw_off(ow) != NOSTART;
            const uint64_t same = __ballot(hn && ho && lw_off(lwv) == lw_off(ow));
            const uint32_t j0 = same ? (uint32_t)__builtin_ctzll(same) : 64u;
            const bool in = lane < j0;  // lanes before the chains meet
            const bool esc = in && ((hn && lw_ch(lwv) == CH_ESC) || (ho && lw_ch(ow) == CH_ESC));
            if (__any(esc)) {
                cmp = false;  // counts not in the words: finish with a full re-walk
            } else {
                dr += wave_sum<int64_t>(in ? (int64_t)(hn ? lw_rows(lwv) : 0u) -
                                                 (int64_t)(ho ? lw_rows(ow) : 0u)
                                           : 0);
                dk += wave_sum<int64_t>(in ? (int64_t)(hn ? lw_ctl(lwv) : 0u) -
                                                 (int64_t)(ho ? lw_ctl(ow) : 0u)
                                           : 0);
                dc += wave_sum<int64_t>(in ? (int64_t)(hn ? lw_ch(lwv) : 0u) -
                                                 (int64_t)(ho ? lw_ch(ow) : 0u)
                                           : 0);
                if (same) {
                    merged = true;
                    d[0] = dr;
                    d[1] = dc;
                    d[2] = dk;
                    return rs;
                }
            }
        }
        rs.tries += wave_sum<uint32_t>(tries);
        rs.rounds += to.rounds;
        rs.why += to.why;
        if (!have_spec && to.anchor != NONE) {
            rs.spec = to.anchor;
            have_spec = true;
        }
        rs.rows += to.rows;
        rs.ch += to.ch;
        rs.ctl += to.ctl;
        if (to.ek) {
            rs.err = ((uint64_t)to.ek << 56) | (to.exit & POSM);
            rs.exit = to.exit;
            return rs;
        }
        cur = to.exit;
        rs.exit = cur;
    }
    return rs;
}

}  // namespace

// ---- pass 1: count ---------------------------------------------------------------------------
#ifndef NXG_GEN_COUNT_OCC
#define NXG_GEN_COUNT_OCC 3  // waves per SIMD (4: 128 VGPRs, and 128 B/lane of scratch)
#endif
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(NXG_GEN_COUNT_OCC))) void nxg_gen_count_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, uint32_t* __restrict__ lws,
    uint64_t* __restrict__ runs, DevStatus* __restrict__ st, DevStatus* zst, uint64_t* __restrict__ fix) {
    zero_status(zst);
    if (blockIdx.x == 0 && threadIdx.x == 0) fix[0] = 0;  // emit's work list (read by fix)
    __shared__ __attribute__((aligned(16))) uint8_t bufs[WAVES][IMG + 16];  // +16: word reads past the image
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t R = gridDim.x * WAVES, r = blockIdx.x * WAVES + w;
    const uint64_t b = run_begin(nt, R, r), e = run_begin(nt, R, r + 1);
    bool merged;
    int64_t d[3];
    const RunSum rs =
        run_tiles(wire, W, b, e, b == 0 ? 0ull : NONE, lws, bufs[w], NONE, merged, d);
    if (lane < R_WORDS) {
        const uint64_t v[R_WORDS] = {rs.spec, rs.exit, rs.rows, rs.ch, rs.ctl, rs.err, 0, 0};
        uint64_t x = v[0];
#pragma unroll
        for (int i = 1; i < R_WORDS; i++)
            if ((int)lane == i) x = v[i];
        runs[(uint64_t)r * R_WORDS + lane] = x;
    }
    if (lane == 0) {
        atomicAdd(&st->diag[2], (unsigned long long)rs.rounds);
        atomicAdd(&st->diag[4], (unsigned long long)rs.tries);
        for (int i = 0; i < 4; i++)
            atomicAdd(&st->diag[i == 0 ? 1 : i == 1 ? 3 : i == 2 ? 5 : 6],
                      (unsigned long long)((rs.why >> (16 * i)) & 0xffffu));
    }
}

// ---- resolve: one workgroup ------------------------------------------------------------------
// Thread i owns runs [i*K, (i+1)*K). The exit entering run r is the exit of the latest run before
// it that holds a message start (run 0 always does: it starts at byte 0). Events, in run order
// from `from` on: a run whose guessed entry disagrees with its entering exit (wave 0 re-walks it
// from that exit, rewriting its lane words and summary), or the first run with an error (the
// frame's error). Then the run totals are prefix-summed into the emit pass's bases.
constexpr int RES_TPB = 512;  // (1024: 128 VGPRs at most, and the re-walk spilled 296 B/lane)
constexpr int RES_K = gdec2::MAX_RUNS / RES_TPB;
static_assert(gdec2::MAX_RUNS % RES_TPB == 0, "resolve geometry");

// exclusive block scan (sum) over RES_TPB threads
template <typename T>
NXG_DEV T res_scan(T v, T* tmp, T& total) {
    const uint32_t tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
    const T inc = wave_incl_scan(v);
    if (l == 63) tmp[wv] = inc;
    __syncthreads();
    T wb = 0, tot = 0;
    for (int i = 0; i < RES_TPB / 64; i++) {
        const T x = tmp[i];
        if ((uint32_t)i < wv) wb += x;
        tot += x;
    }
    __syncthreads();
    total = tot;
    return wb + inc - v;
}
// exclusive block scan (max) over RES_TPB threads
NXG_DEV uint64_t res_scan_max(uint64_t v, uint64_t* tmp) {
    const uint32_t tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
    uint64_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(inc, d, 64);
        if (l >= (uint32_t)d && o > inc) inc = o;
    }
    if (l == 63) tmp[wv] = inc;
    __syncthreads();
    uint64_t m = 0;
    for (uint32_t i = 0; i < wv; i++) m = tmp[i] > m ? tmp[i] : m;
    __syncthreads();
    uint64_t ex = __shfl_up(inc, 1, 64);
    if (l == 0) ex = 0;
    return ex > m ? ex : m;
}

__global__ __launch_bounds__(RES_TPB) void nxg_gen_resolve_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, uint32_t R,
    uint32_t* __restrict__ lws, uint64_t* __restrict__ runs, uint64_t* __restrict__ base,
    DevStatus* __restrict__ st) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[IMG + 16];
    __shared__ uint64_t tmp[RES_TPB / 64];
    __shared__ uint32_t sh_first;
    __shared__ uint64_t sh_x;
    const uint32_t tid = threadIdx.x;
    const uint32_t r0 = tid * RES_K;
    uint32_t from = 0, fixes = 0;
#pragma unroll 1
    for (;;) {
        // latest run (index + 1) with a start among this thread's runs, then across threads
        uint64_t mine = 0;
        for (int k = 0; k < RES_K; k++) {
            const uint32_t r = r0 + k;
            if (r < R && runs[(uint64_t)r * R_WORDS + R_SPEC] != NONE) mine = r + 1;
        }
        const uint64_t before = res_scan_max(mine, tmp);
        uint64_t X = before ? runs[(before - 1) * R_WORDS + R_EXIT] : 0ull;
        uint32_t first = 0xffffffffu;
        uint64_t xfirst = 0;
        for (int k = 0; k < RES_K; k++) {
            const uint32_t r = r0 + k;
            if (r >= R) break;
            const uint64_t* q = runs + (uint64_t)r * R_WORDS;
            const uint64_t spec = q[R_SPEC];
            const uint64_t rend = run_begin(nt, R, r + 1) * TILE;
            const bool ok = r == 0 || (spec == NONE ? (X >= rend || X >= W) : spec == X);
            if (r >= from && (!ok || q[R_ERR] != 0)) {
                first = r;
                xfirst = X;
                break;
            }
            if (spec != NONE) X = q[R_EXIT];
        }
        if (tid == 0) sh_first = 0xffffffffu;
        __syncthreads();
        if (first != 0xffffffffu) atomicMin(&sh_first, first);
        __syncthreads();
        const uint32_t F = sh_first;
        if (F != 0xffffffffu && first == F) sh_x = xfirst;
        __syncthreads();
        if (F == 0xffffffffu) break;  // every run verified, no error
        const uint64_t XF = sh_x;
        const uint64_t* q = runs + (uint64_t)F * R_WORDS;
        const uint64_t spec = q[R_SPEC];
        const uint64_t rend = run_begin(nt, R, F + 1) * TILE;
        const bool ok = F == 0 || (spec == NONE ? (XF >= rend || XF >= W) : spec == XF);
        if (ok) {
            // The first broken length prefix on the true chain: the chain ends in run F. The
            // emit pass decodes the runs up to F (an earlier content error still wins).
            if (tid == 0) {
                const uint64_t er = q[R_ERR];
                st->err_key = err_key(er & POSM, (uint32_t)(er >> 56));
                st->runs_valid = F + 1;
            }
            break;
        }
        __syncthreads();
        if (tid < 64) {  // wave 0 re-walks run F from its true entry
            const uint64_t b = run_begin(nt, R, F), e = run_begin(nt, R, F + 1);
            // pass 1 wrote lane words up to its last tile (its error tile, if it stopped early)
            const uint64_t oerr = q[R_ERR];
            const uint64_t old_last = oerr ? (oerr & POSM) / TILE : e - 1;
            bool merged;
            int64_t d[3];
            const RunSum rs = run_tiles(wire, W, b, e, XF, lws, buf, old_last, merged, d);
            if (tid < R_WORDS) {
                // merged: the old chain from the meeting point on stands (exit, error)
                const uint64_t v[R_WORDS] = {
                    XF,
                    merged ? q[R_EXIT] : rs.exit,
                    merged ? q[R_ROWS] + (uint64_t)d[0] : rs.rows,
                    merged ? q[R_CH] + (uint64_t)d[1] : rs.ch,
                    merged ? q[R_CTL] + (uint64_t)d[2] : rs.ctl,
                    merged ? q[R_ERR] : rs.err,
                    1,
                    0};
                uint64_t x = v[0];
#pragma unroll
                for (int i = 1; i < R_WORDS; i++)
                    if ((int)tid == i) x = v[i];
                runs[(uint64_t)F * R_WORDS + tid] = x;
            }
        }
        fixes++;
        __threadfence_block();
        __syncthreads();
        from = F;  // run F is now on the true chain; an error in it is found next round
    }
    if (tid == 0) {
        st->path = 2;
        st->diag[0] = fixes;
    }
    // prefix sums of the run totals -> bases
    uint64_t lr = 0, lc = 0, lk = 0;
    for (int k = 0; k < RES_K; k++) {
        const uint32_t r = r0 + k;
        if (r >= R) break;
        const uint64_t* q = runs + (uint64_t)r * R_WORDS;
        lr += q[R_ROWS];
        lc += q[R_CH];
        lk += q[R_CTL];
    }
    uint64_t tr, tc, tk;
    uint64_t br = res_scan<uint64_t>(lr, tmp, tr);
    uint64_t bc = res_scan<uint64_t>(lc, tmp, tc);
    uint64_t bk = res_scan<uint64_t>(lk, tmp, tk);
    for (int k = 0; k < RES_K; k++) {
        const uint32_t r = r0 + k;
        if (r >= R) break;
        const uint64_t* q = runs + (uint64_t)r * R_WORDS;
        base[(uint64_t)r * 4 + 0] = br;
        base[(uint64_t)r * 4 + 1] = bc;
        base[(uint64_t)r * 4 + 2] = bk;
        br += q[R_ROWS];
        bc += q[R_CH];
        bk += q[R_CTL];
    }
    if (tid == 0) {
        st->n_rows = tr;
        st->n_children = tc;
        st->n_ctl = tk;
    }
}

// ---- pass 3: emit ----------------------------------------------------------------------------
// Two kernels. The emit kernel is type-bucketed and message-parallel; per tile:
//   1. each lane walks only the length chain of the messages that start in its chunk (from the
//      start its lane word records) and lists their positions in LDS, in wire order;
//   2. message-parallel: every message's header is parsed and the message classified (fixed-size
//      scalar, text, DateTime/Duration, varint scalar, flat array of fixed-size scalars,
//      Heartbeat, or other); row / control / child indices are scanned in wire order;
//   3. a counting sort buckets the messages by class, and each bucket is decoded by all lanes
//      running the same code, 64 messages at a time.
// A tile holding an "other" message (other control messages, nested or unusual values, messages
// that leave the LDS image), a message a fast path does not accept (it may be an error), more
// than MAXM messages, or columns without the mixed layout goes on a work list with its row /
// control / child bases; a tile whose lane words lost a children count (CH_ESC) puts the rest of
// its run there (the bases after it are not known). The fix kernel then re-emits the listed tiles
// with the per-lane path (decode_msg for every message, exact errors). The emit kernel itself
// never runs the general decoder, which keeps it small (registers, instruction cache).
namespace {

constexpr int MAXM = 512;  // messages per tile on the bucketed path
enum { K_FIX = 0, K_TEXT, K_TIME, K_VAR, K_ARR, K_HB, K_OTHER, K_N };
constexpr int FIX_WORDS = 5;  // work list entry: first tile, end tile, row, control, child bases

struct EmitLds {
    uint16_t mpos[MAXM];  // message start, tile-relative
    uint8_t cls[MAXM];    // class | 0x80 for an Update
    uint16_t ridx[MAXM];  // row (Update) or control-message index within the tile
    uint16_t cb[MAXM];    // first child slot (Update; < 2^16: a message's elements are >= 1
                          // byte and lie in the 5 KiB image) or the row it precedes (control)
    uint16_t bucket[MAXM];
};

// the fixed-size scalar tags: payload bytes, or -1
NXG_DEV int fix_bytes(uint32_t t) {
    switch (t) {
    case 0: case 2: case 8: return 4;
    case 4: case 6: case 9: return 8;
    case 14: case 15: case 16: case 17: return 0;
    case 23: case 24: return 1;
    case 25: case 26: return 2;
    default: return -1;
    }
}
// column value of a fixed-size scalar whose n payload bytes start at p (Value::decode,
// lib.rs:470-506: signed types sign-extended, bool as 1/0, Null for 16/17)
NXG_DEV uint64_t fix_value(const LdsSrc& s, uint32_t t, uint64_t p, int n) {
    const uint64_t raw = ((uint64_t)bswap32(s.word(p)) << 32) | bswap32(s.word(p + 4));
    uint64_t v = n ? raw >> (64 - 8 * n) : 0ull;
    if (t == 2 || t == 24 || t == 26) {  // i32 / i8 / i16
        const int sh = 64 - 8 * n;
        v = (uint64_t)((int64_t)(v << sh) >> sh);
    }
    if (t == 14) v = 1;
    return v;
}

// Header of the message at p: returns the class in bits 0..3, bit 4 for an Update, and the
// number of child slots (K_ARR) from bit 8. The Update bit is exact for every well-formed
// message (it sets the row / control numbering); anything unusual, or a message not wholly in
// the image, is K_OTHER.
constexpr uint32_t C_UPD = 16;
NXG_DEV uint32_t classify(const Src& s, uint64_t p) {
    const LdsSrc ls{s.lds, s.t0};
    uint64_t q = p, L;
    const uint32_t e = p - s.t0 + 10 <= s.nlds ? dvar(ls, q, s.W, L) : dvar(GlbSrc{s.g}, q, s.W, L);
    if (e || L < 1 || q >= s.W) return K_OTHER;  // an error: the fix kernel reports it
    const uint64_t take = L - vl64(L);
    const uint64_t lim = take < s.W - q ? q + take : s.W;
    const uint32_t variant = s.any_byte(q++);
    if (variant == 5) return K_HB;  // Heartbeat: no fields (trailing bytes skipped, pack.rs:551)
    if (variant != 4) return K_OTHER;
    // wholly in the image (word reads reach at most 7 bytes past the message: the 16 spare
    // bytes after the image cover them)
    if (lim - s.t0 > s.nlds || q >= lim) return K_OTHER | C_UPD;
    uint64_t id;
    if (dvar(ls, q, lim, id) || q >= lim) return K_OTHER | C_UPD;
    const uint32_t t = ls.byte(q++);
    const int n = fix_bytes(t);
    uint32_t k = K_OTHER;
    if (n >= 0) k = q + n <= lim ? K_FIX : K_OTHER;
    else if (t == 12 || t == 13 || t == 18) k = K_TEXT;
    else if (t == 10 || t == 11) k = q + 12 <= lim ? K_TIME : K_OTHER;
    else if (t == 1 || t == 3 || t == 5 || t == 7) k = K_VAR;
    else if (t == 19) {  // an array of fixed-size scalars that fits: its children are its elements
        uint64_t cnt;
        bool ok = !dvar(ls, q, lim, cnt) && cnt <= (kMaxVec / 16) && cnt * 16 <= ((lim - q) << 8);
#pragma unroll 1
        for (uint64_t i = 0; ok && i < cnt; i++) {
            const int m = q < lim ? fix_bytes(ls.byte(q)) : -1;
            ok = m >= 0 && q + 1 + m <= lim;
            q += 1 + m;
        }
        if (ok) return K_ARR | C_UPD | ((uint32_t)cnt << 8);
    }
    return k | C_UPD;
}

NXG_DEV void put_row(const ColsDesc& cols, DevStatus* st, uint64_t row, uint64_t id, uint32_t tag,
                     uint64_t fixed, uint32_t aux) {
    if (row < cols.cap_rows) {
        cols.id[row] = id;
        cols.tag[row] = (uint8_t)tag;
        cols.fixed[row] = fixed;
        cols.aux[row] = aux;
    } else {
        atomicOr(&st->capacity, 1u);
    }
}

// Fast decode of one Update of class k at pos; false = not accepted (the caller falls back to
// emit_other, which reports any error exactly).
NXG_DEV bool emit_fast(uint32_t k, const Src& s, const ColsDesc& cols, DevStatus* st,
                       uint64_t pos, uint64_t row, uint64_t child) {
    const LdsSrc ls{s.lds, s.t0};
    uint64_t q = pos, L, id;
    dvar(ls, q, s.W, L);
    const uint64_t take = L - vl64(L);
    const uint64_t lim = take < s.W - q ? q + take : s.W;
    q++;  // variant 4
    dvar(ls, q, lim, id);
    const uint32_t t = ls.byte(q++);
    if (k == K_FIX) {
        const int n = fix_bytes(t);
        put_row(cols, st, row, id, t == 17 ? 16u : t, fix_value(ls, t, q, n), 0);
        return true;
    }
    if (k == K_TEXT) {
        uint64_t n;
        if (dvar(ls, q, lim, n) || n > lim - q) return false;
        if (t != 13 && !utf8_ok(ls, q, n)) return false;
        put_row(cols, st, row, id, t, q, (uint32_t)n);
        return true;
    }
    if (k == K_TIME) {
        uint64_t secs, v2;
        dfix(ls, q, lim, 8, secs);
        dfix(ls, q, lim, 4, v2);
        uint32_t ns = (uint32_t)v2;
        if (t == 10) {
            if (!datetime_valid((int64_t)secs, ns)) return false;
        } else if (ns >= 1000000000u) {  // Duration::new normalisation (overflow: error path)
            const uint64_t add = ns / 1000000000u;
            if (secs + add < secs) return false;
            secs += add;
            ns %= 1000000000u;
        }
        put_row(cols, st, row, id, t, secs, ns);
        return true;
    }
    if (k == K_VAR) {
        uint64_t v;
        if (dvar(ls, q, lim, v)) return false;
        uint64_t x = v;
        if (t == 1) x = (uint32_t)v;
        else if (t == 3) {
            const uint32_t u = (uint32_t)v;
            x = (uint64_t)(int64_t)((int32_t)(u >> 1) ^ (int32_t)(0u - (u & 1u)));
        } else if (t == 7) x = (v >> 1) ^ (0ull - (v & 1ull));
        put_row(cols, st, row, id, t, x, 0);
        return true;
    }
    // K_ARR: the elements were checked by classify
    uint64_t cnt;
    dvar(ls, q, lim, cnt);
    put_row(cols, st, row, id, 19, child, (uint32_t)cnt);
    for (uint64_t i = 0; i < cnt; i++) {
        const uint32_t et = ls.byte(q++);
        const int n = fix_bytes(et);
        const uint64_t slot = child + i;
        if (slot < cols.cap_children) {
            cols.ctag[slot] = (uint8_t)(et == 17 ? 16u : et);
            cols.cfixed[slot] = fix_value(ls, et, q, n);
            cols.caux[slot] = 0;
        } else {
            atomicOr(&st->capacity, 1u);
        }
        q += n;
    }
    return true;
}

// A Heartbeat at pos (validated by classify): its control-message columns.
NXG_DEV void emit_hb(const Src& s, const ColsDesc& cols, DevStatus* st, uint64_t pos, uint64_t row,
                     uint64_t ctl) {
    uint64_t q = pos, L;
    if (pos - s.t0 + 10 <= s.nlds) dvar(LdsSrc{s.lds, s.t0}, q, s.W, L);
    else dvar(GlbSrc{s.g}, q, s.W, L);
    const uint64_t take = L - vl64(L);
    const uint64_t lim = take < s.W - q ? q + take : s.W;
    if (ctl < cols.cap_ctl) {
        cols.ctl_row[ctl] = row;
        cols.ctl_off[ctl] = pos;
        cols.ctl_len[ctl] = (uint32_t)(lim - pos);
        cols.ctl_variant[ctl] = 5;
    } else {
        atomicOr(&st->capacity, 1u);
    }
}

// work list: fix[0] = entries, then FIX_WORDS words per entry (at most one per tile)
NXG_DEV void fix_push(uint64_t* fix, uint64_t tb, uint64_t te, uint64_t row, uint64_t ctl,
                      uint64_t child) {
    if (__lane_id() == 0) {
        const uint64_t i = atomicAdd((unsigned long long*)fix, 1ull);
        uint64_t* e = fix + 1 + i * FIX_WORDS;
        e[0] = tb;
        e[1] = te;
        e[2] = row;
        e[3] = ctl;
        e[4] = child;
    }
}

// the general path for one message: decode_msg writes the row / children; the control columns
// and the id are written here (as the per-lane path does)
NXG_DEV uint32_t emit_other(const Src& s, const Sink& sink, const ColsDesc& cols, DevStatus* st,
                            uint64_t pos, uint64_t row, uint64_t ctl, uint64_t child) {
    MsgInfo mi;
    uint32_t work = 0;
    uint64_t cn = child;
    const DMode md{0xffffffffu, 0, 1};
    const uint32_t err = decode_msg<true>(s, pos, mi, &sink, row, cn, work, md);
    if (err) {
        atomicMax((unsigned long long*)&st->err_key, (unsigned long long)err_key(pos, err));
        return 0;
    }
    if (mi.variant == 4) {
        if (row < cols.cap_rows) cols.id[row] = mi.id;
        else atomicOr(&st->capacity, 1u);
    } else if (!cols.ctl_row) {
        atomicOr(&st->nonf64, 1u);
    } else if (ctl < cols.cap_ctl) {
        cols.ctl_row[ctl] = row;
        cols.ctl_off[ctl] = pos;
        cols.ctl_len[ctl] = (uint32_t)(mi.next - pos);
        cols.ctl_variant[ctl] = (uint8_t)mi.variant;
    } else {
        atomicOr(&st->capacity, 1u);
    }
    return mi.variant;
}

// The per-lane path (tiles the bucketed path does not take): each lane decodes its messages in
// order with decode_msg.
NXG_DEV void emit_tile_lanes(const Src& s, const Sink& sink, const ColsDesc& cols, DevStatus* st,
                             uint32_t lw, uint64_t c, uint64_t& row, uint64_t& ctl,
                             uint64_t& child, uint32_t& hb) {
    const uint64_t stop = c + CH < s.W ? c + CH : s.W;
    const bool has = lw_off(lw) != NOSTART;
    uint32_t nr = has ? lw_rows(lw) : 0u, nk = has ? lw_ctl(lw) : 0u;
    uint64_t nch = has ? lw_ch(lw) : 0u;
    // A lane whose children count did not fit its word counts them first (phase 0, no
    // writes); then the wave scans the counts and every lane decodes + writes (phase 1).
    const bool recount = has && nch == CH_ESC;
    uint64_t myrow = 0, myctl = 0, mych = 0;
#pragma unroll 1
    for (int ph = __any(recount) ? 0 : 1; ph < 2; ph++) {
        if (ph == 1) {
            const uint32_t rin = wave_incl_scan(nr);
            const uint32_t kin = wave_incl_scan(nk);
            const uint64_t cin = wave_incl_scan<uint64_t>(nch);
            myrow = row + rin - nr;
            myctl = ctl + kin - nk;
            mych = child + cin - nch;
            row += wave_last(rin);
            ctl += wave_last(kin);
            child += wave_last(cin);
        }
        const bool act = ph == 1 ? has : recount;
        uint64_t pos = act ? c + lw_off(lw) : stop;
        uint64_t cn = ph == 1 ? mych : 0;
        uint32_t work = 0;
        const DMode md{0xffffffffu, 0, (uint32_t)ph};
#pragma unroll 1
        while (pos < stop) {
            MsgInfo mi;
            const uint32_t err = decode_msg<true>(s, pos, mi, &sink, myrow, cn, work, md);
            if (err) {  // the frame's first error is the earliest of these (and resolve's)
                atomicMax((unsigned long long*)&st->err_key, (unsigned long long)err_key(pos, err));
                break;
            }
            if (ph == 1) {
                hb += mi.variant == 5;
                if (mi.variant == 4) {
                    if (myrow < cols.cap_rows) cols.id[myrow] = mi.id;
                    else atomicOr(&st->capacity, 1u);
                    myrow++;
                } else if (!cols.ctl_row) {
                    atomicOr(&st->nonf64, 1u);
                    myctl++;
                } else {
                    if (myctl < cols.cap_ctl) {
                        cols.ctl_row[myctl] = myrow;
                        cols.ctl_off[myctl] = pos;
                        cols.ctl_len[myctl] = (uint32_t)(mi.next - pos);
                        cols.ctl_variant[myctl] = (uint8_t)mi.variant;
                    } else {
                        atomicOr(&st->capacity, 1u);
                    }
                    myctl++;
                }
            }
            pos = mi.next;
        }
        if (ph == 0 && recount) nch = cn;
    }
}

}  // namespace

__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(4))) void nxg_gen_emit_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, const uint32_t* __restrict__ lws,
    const uint64_t* __restrict__ base, ColsDesc cols, DevStatus* __restrict__ st,
    uint64_t* __restrict__ fix) {
    __shared__ __attribute__((aligned(16))) uint8_t bufs[WAVES][IMG + 16];  // +16: word reads past the image
    __shared__ EmitLds tabs[WAVES];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t R = gridDim.x * WAVES, r = blockIdx.x * WAVES + w;
    const uint64_t b = run_begin(nt, R, r), e = run_begin(nt, R, r + 1);
    // a broken length prefix (resolve) ends the chain: later runs and tiles hold no messages
    const uint32_t rv = st->runs_valid;
    const uint64_t ck = st->err_key;
    const uint64_t chain_end = ck ? (~ck) >> 8 : ~0ull;
    if (b >= e || (rv && r >= rv)) return;
    uint8_t* buf = bufs[w];
    EmitLds& T = tabs[w];
    uint64_t row = base[(uint64_t)r * 4 + 0];
    uint64_t child = base[(uint64_t)r * 4 + 1];
    uint64_t ctl = base[(uint64_t)r * 4 + 2];
    if (cols.tag == nullptr || cols.ctl_row == nullptr) {  // not the mixed layout: all per lane
        fix_push(fix, b, e, row, ctl, child);
        return;
    }
    uint32_t hb = 0;  // heartbeats in tiles this kernel completes
    GRegs g;
    g_load(g, wire, b * TILE, W, lane);
    uint32_t lwn = lws[b * 64 + lane];
#pragma unroll 1
    for (uint64_t t = b; t < e; t++) {
        const uint64_t t0 = t * TILE;
        if (t0 > chain_end) break;
        const uint32_t lw = lwn;
        g_stage(buf, g, lane);
        if (t + 1 < e) {
            g_load(g, wire, (t + 1) * TILE, W, lane);
            lwn = lws[(t + 1) * 64 + lane];
        }
        const Src s = g_src(buf, wire, t0, W);
        const uint64_t c = t0 + (uint64_t)lane * CH;
        const bool has = lw_off(lw) != NOSTART;
        const uint32_t nr = has ? lw_rows(lw) : 0u, nk = has ? lw_ctl(lw) : 0u;
        const uint32_t nch = has ? lw_ch(lw) : 0u;
        if (__any(nch == CH_ESC)) {  // this tile's children are not in the words: the rest per lane
            fix_push(fix, t, e, row, ctl, child);
            break;
        }
        const uint32_t nm = nr + nk;
        const uint32_t minc = wave_incl_scan(nm);
        const uint32_t nmsg = wave_last(minc);
        const uint64_t row_t = row, ctl_t = ctl, child_t = child;
        row += wave_sum<uint32_t>(nr);
        ctl += wave_sum<uint32_t>(nk);
        child += wave_sum<uint32_t>(nch);
        if (nmsg > (uint32_t)MAXM) {
            fix_push(fix, t, t + 1, row_t, ctl_t, child_t);
            continue;
        }
        // 1. message starts (length chain only), in wire order
        {
            uint64_t pos = c + lw_off(lw);
            uint32_t m = minc - nm;
            const LdsSrc ls{s.lds, s.t0};
            for (uint32_t i = 0; i < nm; i++) {
                T.mpos[m++] = (uint16_t)(pos - t0);
                uint64_t q = pos, L = 1;
                if (pos - t0 + 10 <= s.nlds) dvar(ls, q, W, L);
                else dvar(GlbSrc{s.g}, q, W, L);
                const uint64_t take = L - vl64(L);
                pos = take < W - q ? q + take : W;
            }
        }
        wave_lds_order();
        // 2. classify, scan the row / control / child indices in wire order
        uint32_t rcar = 0, kcar = 0, ccar = 0;
        uint32_t kcnt[K_N] = {0, 0, 0, 0, 0, 0, 0};
        for (uint32_t m0 = 0; m0 < nmsg; m0 += 64) {
            const uint32_t m = m0 + lane;
            const bool in = m < nmsg;
            const uint32_t cw = in ? classify(s, t0 + T.mpos[m]) : (uint32_t)K_OTHER;
            const uint32_t k = cw & 15u;
            const bool upd = cw & C_UPD;
            const uint32_t kids = cw >> 8;
            const uint32_t ri = wave_incl_scan((uint32_t)(in && upd));
            const uint32_t ki = wave_incl_scan((uint32_t)(in && !upd));
            const uint32_t ci = wave_incl_scan(in ? kids : 0u);
            if (in) {  // control messages keep the row they precede in cb
                T.cls[m] = (uint8_t)(k | (upd ? 0x80u : 0u));
                T.ridx[m] = (uint16_t)(upd ? rcar + ri - 1 : kcar + ki - 1);
                T.cb[m] = (uint16_t)(upd ? ccar + ci - kids : rcar + ri);
            }
            rcar += wave_last(ri);
            kcar += wave_last(ki);
            ccar += wave_last(ci);
#pragma unroll
            for (int kk = 0; kk < K_N; kk++) kcnt[kk] += __popcll(__ballot(in && k == (uint32_t)kk));
        }
        if (kcnt[K_OTHER]) {  // a message only decode_msg handles
            fix_push(fix, t, t + 1, row_t, ctl_t, child_t);
            wave_lds_order();
            continue;
        }
        wave_lds_order();
        // 3. counting sort by class, then one uniform pass per class
        uint32_t koff[K_N];
        uint32_t acc = 0;
#pragma unroll
        for (int kk = 0; kk < K_N; kk++) {
            koff[kk] = acc;
            acc += kcnt[kk];
        }
        {
            uint32_t fill[K_N];
#pragma unroll
            for (int kk = 0; kk < K_N; kk++) fill[kk] = koff[kk];
            for (uint32_t m0 = 0; m0 < nmsg; m0 += 64) {
                const uint32_t m = m0 + lane;
                const uint32_t k = m < nmsg ? (T.cls[m] & 0x7fu) : (uint32_t)K_N;
#pragma unroll
                for (int kk = 0; kk < K_N; kk++) {
                    const uint64_t bm = __ballot(k == (uint32_t)kk);
                    if (k == (uint32_t)kk)
                        T.bucket[fill[kk] + __popcll(bm & ((1ull << lane) - 1))] = (uint16_t)m;
                    fill[kk] += __popcll(bm);
                }
            }
        }
        wave_lds_order();
        bool fail = false;
#pragma unroll 1
        for (int kk = 0; kk < K_OTHER; kk++) {
            for (uint32_t i = koff[kk] + lane; i < koff[kk] + kcnt[kk]; i += 64) {
                const uint32_t m = T.bucket[i];
                const uint64_t pos = t0 + T.mpos[m];
                if (kk == K_HB) emit_hb(s, cols, st, pos, row_t + T.cb[m], ctl_t + T.ridx[m]);
                else fail |= !emit_fast((uint32_t)kk, s, cols, st, pos, row_t + T.ridx[m],
                                        child_t + T.cb[m]);
            }
        }
        if (__any(fail)) fix_push(fix, t, t + 1, row_t, ctl_t, child_t);  // exact errors there
        else hb += kcnt[K_HB];
        wave_lds_order();
    }
    if (lane == 0 && hb) atomicAdd((unsigned long long*)&st->n_heartbeat, (unsigned long long)hb);
}

// Re-emits the work list's tiles with the per-lane path (every message through decode_msg).
__global__ __launch_bounds__(TPB) void nxg_gen_fix_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, const uint32_t* __restrict__ lws, ColsDesc cols,
    DevStatus* __restrict__ st, const uint64_t* __restrict__ fix) {
    __shared__ __attribute__((aligned(16))) uint8_t bufs[WAVES][IMG + 16];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t n = fix[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) st->diag[7] = n;  // tiles re-emitted per lane
    const uint64_t ck = st->err_key;
    const uint64_t chain_end = ck ? (~ck) >> 8 : ~0ull;
    uint8_t* buf = bufs[w];
    const Sink sink{cols, &st->capacity, &st->nonf64};
    uint32_t hb = 0;
#pragma unroll 1
    for (uint64_t i = (uint64_t)blockIdx.x * WAVES + w; i < n; i += (uint64_t)gridDim.x * WAVES) {
        const uint64_t* en = fix + 1 + i * FIX_WORDS;
        uint64_t row = en[2], ctl = en[3], child = en[4];
#pragma unroll 1
        for (uint64_t t = en[0]; t < en[1]; t++) {
            const uint64_t t0 = t * TILE;
            if (t0 > chain_end) break;
            GRegs g;
            g_load(g, wire, t0, W, lane);
            g_stage(buf, g, lane);
            const Src s = g_src(buf, wire, t0, W);
            emit_tile_lanes(s, sink, cols, st, lws[t * 64 + lane], t0 + (uint64_t)lane * CH, row,
                            ctl, child, hb);
        }
    }
    hb = wave_sum<uint32_t>(hb);
    if (lane == 0 && hb) atomicAdd((unsigned long long*)&st->n_heartbeat, (unsigned long long)hb);
}

uint64_t nxg_dec_gen_tiles(uint64_t W) { return (W + TILE - 1) / TILE; }
uint64_t nxg_dec_gen_scratch_bytes(uint64_t W) {
    const uint64_t nt = nxg_dec_gen_tiles(W);
    return 256 * nt + 8 * (1 + FIX_WORDS * nt);  // lane words, then emit's work list
}

hipError_t nxg_launch_dec_gen(const uint8_t* wire, uint64_t W, const ColsDesc& cd, uint32_t* lws,
                              uint64_t* runs, uint64_t* base, int wgs, DevStatus* st,
                              hipStream_t s) {
    const uint64_t nt = nxg_dec_gen_tiles(W);
    if (nt == 0) return hipSuccess;
    if (wgs <= 0 || wgs * WAVES > gdec2::MAX_RUNS) return hipErrorInvalidValue;
    // no more runs than tiles: empty runs only cost a pass-through in resolve
    uint64_t g = (nt + WAVES - 1) / WAVES;
    if (g > (uint64_t)wgs) g = wgs;
    const uint32_t R = (uint32_t)g * WAVES;
    uint64_t* fix = reinterpret_cast<uint64_t*>(lws + 64 * nt);  // nxg_dec_gen_scratch_bytes
    hipLaunchKernelGGL(nxg_gen_count_kernel, dim3(g), dim3(TPB), 0, s, wire, W, nt, lws, runs, st,
                       nxg_take_zero_slot(), fix);
    hipLaunchKernelGGL(nxg_gen_resolve_kernel, dim3(1), dim3(RES_TPB), 0, s, wire, W, nt, R, lws,
                       runs, base, st);
    hipLaunchKernelGGL(nxg_gen_emit_kernel, dim3(g), dim3(TPB), 0, s, wire, W, nt, lws, base, cd,
                       st, fix);
    hipLaunchKernelGGL(nxg_gen_fix_kernel, dim3(g), dim3(TPB), 0, s, wire, W, lws, cd, st, fix);
    return hipGetLastError();
}

int nxg_dec_gen_wgs(int ncu) {
    int a = 0, b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, nxg_gen_count_kernel, TPB, 0) !=
            hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, nxg_gen_emit_kernel, TPB, 0) !=
            hipSuccess)
        return ncu;
    // the passes share the run partition, so one grid for both; neither waits on another
    // workgroup, so the grid follows the larger occupancy (extra count workgroups just queue)
    const int occ = a > b ? a : b;
    int g = ncu * (occ > 0 ? occ : 1);
    return g < gdec2::MAX_RUNS / WAVES ? g : gdec2::MAX_RUNS / WAVES;
}
