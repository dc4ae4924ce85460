// nxg_decode_general.hip -- general From-stream decode for gfx950 (every From variant, every
// Value tag, nesting, errors), single pass over the wire.
//
// This is the receive_batch_fn loop (netidx/src/channel.rs:504-521) for arbitrary frames.
// Message boundaries form a pointer chain (len_wrapped_decode, pack.rs:537-555), and a message
// may be arbitrarily long. They are resolved in parallel by speculation with exact repair:
//
//  * lane: each lane owns a 32-byte chunk. It guesses its first message start: the first
//    position from which two consecutive messages decode plausibly. From that guess it walks
//    the messages that START inside its chunk with the full validating decoder. This walk has a
//    work budget: a wrong guess must not wander through megabytes. The lane records its exit
//    (the first message start past its chunk) and its counts.
//  * block repair: a lane whose guess differs from its predecessor's exit re-walks from that
//    exit. Iterating to a fixed point makes every lane consistent with the tile's entry.
//  * tile: descriptors {speculated entry, exit, counts, first error} are published as
//    aggregates, and later as inclusive prefixes, through a decoupled look-back. A tile
//    composes its predecessors' aggregates only when each aggregate's entry equals the exit of
//    the tile before it. Otherwise it waits for its predecessor's inclusive prefix.
//  * exact phase: once the true entry is known, the tile re-runs the repair from it if its
//    guess was wrong or a walk ran out of budget. Walks in this phase are unbounded and start
//    only at true message starts, so their cost is proportional to the real data.
//  * emit: every lane decodes its messages again and writes the columns at global bases.
//
// The first error on the true chain is carried forward through the inclusive prefixes. The
// frame is rejected with that (kind, message offset), just as the sequential reference stops at
// its first error (netidx/src/subscriber/connection.rs:228-231).
#include "nxg_msg.h"

using namespace gdec;
using namespace nxgmsg;

namespace {

constexpr uint64_t NONE = ~0ull;  // no speculated entry (lane) / not composable (tile)
constexpr uint64_t POSM = (1ull << 56) - 1;

// descriptor word indices (SLOT_WORDS = 16 u64 per tile)
enum {
    W_FLAG = 0,   // flag(63:62) | epoch | rows (aggregate) or rows prefix (inclusive)
    A_CHILD = 1,
    A_CTLHB = 2,  // ctl (lo 32) | heartbeats (hi 32)
    A_SPEC = 3,   // speculated entry; NONE => not composable
    A_EXIT = 4,
    A_ERR = 5,    // kind << 56 | offset; 0 = none
    I_CHILD = 8,
    I_CTLHB = 9,
    I_EXIT = 10,
    I_ERR = 11,
};

// lane states (LDS word: state << 8 | error kind)
enum { S_NONE = 0, S_EXH = 1, S_OK = 2, S_ERR = 3 };

struct LaneRes {
    uint64_t x;  // exit (first message start at/after the chunk end), or error position
    uint32_t rows, ctl, hb;
    uint64_t children;
    uint32_t st;  // S_*
    uint32_t ek;  // error kind when S_ERR
};

NXG_DEV void lane_set(LaneRes& r, uint32_t state, uint64_t x) {
    r.x = x;
    r.rows = r.ctl = r.hb = 0;
    r.children = 0;
    r.st = state;
    r.ek = 0;
}

// validating walk of the messages starting in [e, end)
template <int MODE>
NXG_DEV void walk(const Src& s, uint64_t e, uint64_t end, LaneRes& r) {
    lane_set(r, S_OK, e);
    uint64_t pos = e;
    const uint64_t stop = end < s.W ? end : s.W;
    uint32_t work = 0;
    while (pos < stop) {
        MsgInfo mi;
        uint64_t ch = 0;
        const uint32_t err = decode_msg<false, MODE>(s, pos, mi, nullptr, 0, ch, work);
        if (err == E_BUDGET) {
            r.st = S_EXH;
            return;
        }
        if (err) {
            r.st = S_ERR;
            r.ek = err;
            break;
        }
        if (mi.variant == 4) r.rows++;
        else r.ctl++;
        r.hb += mi.variant == 5;
        r.children += ch;
        pos = mi.next;
    }
    r.x = pos;  // on error: the failing message's start
}

// First position in [c, end) where an Update message decodes plausibly and is followed by
// another Update (or the frame end). Only Updates are guessed: a Heartbeat (`L 05 ...`) or
// Unsubscribed accepts almost any bytes inside its length, so those would be false starts.
// A chunk whose first messages are control messages simply guesses later (or nothing), and
// the repair resolves it exactly.
NXG_DEV uint64_t speculate(const Src& s, uint64_t c, uint64_t end, uint32_t& tries) {
    const uint64_t stop = end < s.W ? end : s.W;
    for (uint64_t p = c; p < stop; p++) {
        MsgInfo mi;
        uint64_t ch = 0;
        uint32_t work = 0;
        tries++;
        if (decode_msg<false, M_SPEC>(s, p, mi, nullptr, 0, ch, work) || mi.variant != 4)
            continue;
        if (mi.next >= s.W) return p;
        MsgInfo m2;
        work = 0;
        if (decode_msg<false, M_SPEC>(s, mi.next, m2, nullptr, 0, ch, work) == E_OK &&
            m2.variant == 4)
            return p;
    }
    return NONE;
}

// Index of the nearest lane below this one whose state is not S_NONE, or -1. Lanes in S_NONE
// have no message start in their chunk: the chain passes straight through them.
NXG_DEV int nearest_def(bool def, uint32_t* wtop) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t m = __ballot(def);
    if (lane == 0) wtop[wv] = m ? wv * 64 + 63 - (uint32_t)__builtin_clzll(m) : 0xffffffffu;
    __syncthreads();
    const uint64_t below = m & ((1ull << lane) - 1);
    int src = -1;
    if (below) {
        src = (int)(wv * 64 + 63 - (uint32_t)__builtin_clzll(below));
    } else {
        for (int i = (int)wv - 1; i >= 0; i--)
            if (wtop[i] != 0xffffffffu) {
                src = (int)wtop[i];
                break;
            }
    }
    return src;
}

// Block repair from an anchor lane. A lane is VERIFIED when every lane from the anchor up to it
// is consistent: a lane with an entry starts exactly at the exit of the nearest lane below it
// that has an entry; a lane without one (S_NONE) lies wholly before that exit (pass-through).
// Each round, the first unverified lane (the "break") is fixed from its verified predecessor:
// - lanes whose whole chunk lies before the predecessor's exit become pass-through;
// - the lane whose chunk contains that exit re-walks from it;
// - after a dead predecessor, every remaining lane inherits the error.
// An unverified exit is never propagated, so a wrong guess cannot corrupt correct lanes.
// Rounds = number of breaks + 1. In M_BOUNDED mode the repair stops at a predecessor whose walk
// ran out of budget; `complete` stays false and the tile is then not composable. On completion,
// *texit / *tek receive the tile's exit (the effective exit of the last lane).
template <int MODE>
NXG_DEV uint32_t repair(const Src& s, uint64_t cend, uint32_t anchor, uint64_t& e, LaneRes& r,
                        uint64_t* sx, uint32_t* sst, uint32_t* wtop, uint32_t* wbreak,
                        uint64_t* bx, uint32_t* nwalks, bool& complete, uint64_t* texit,
                        uint32_t* tek) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // messages can start in [cend - CHUNK, stop): the chunk, clipped to the frame
    const uint64_t stop = cend < s.W ? cend : s.W;
    uint32_t rounds = 0;
    complete = false;
    for (;;) {
        // every round fixes the first break and breaks only move forward: TPB + 1 rounds
        // suffice. The cap turns a logic error into a reported failure, never a hang.
        if (++rounds > 2 * TPB + 4) {
            __syncthreads();
            return rounds;  // complete == false
        }
        sx[tid] = r.x;
        sst[tid] = (r.st << 8) | r.ek;
        const int src = nearest_def(r.st != S_NONE, wtop);  // contains the barrier
        uint32_t pst = S_NONE, pek = 0;
        uint64_t px = 0;
        if (src >= 0) {
            pst = sst[src] >> 8;
            pek = sst[src] & 0xff;
            px = sx[src];
        }
        bool cons = true;
        if (tid > anchor) {
            if (pst == S_ERR) cons = r.st == S_ERR && e == NONE && r.x == px;
            else if (pst == S_OK)
                cons = r.st == S_NONE ? px >= stop
                                      : (e == px && (MODE != M_EXACT || r.st != S_EXH));
            else cons = false;  // behind an exhausted walk: unverifiable here
        } else if (tid == anchor) {
            cons = MODE != M_EXACT || r.st != S_EXH;
        }
        const uint64_t bad = __ballot(!cons);
        if (lane == 0) wbreak[wv] = bad ? wv * 64 + (uint32_t)__builtin_ctzll(bad) : TPB;
        __syncthreads();
        uint32_t brk = TPB;
        for (int i = 0; i < 4; i++) brk = min(brk, wbreak[i]);
        if (brk >= TPB) {
            complete = true;
            if (tid == TPB - 1) {
                *texit = r.st != S_NONE ? r.x : px;
                *tek = r.st == S_ERR ? r.ek : (r.st == S_NONE && pst == S_ERR ? pek : 0u);
            }
            __syncthreads();
            return rounds;
        }
        if (tid == brk) {  // broadcast the break's predecessor
            bx[0] = px;
            bx[1] = ((uint64_t)pst << 8) | pek;
        }
        __syncthreads();
        const uint64_t X = bx[0];
        const uint32_t xst = (uint32_t)(bx[1] >> 8), xek = (uint32_t)(bx[1] & 0xff);
        bool progressed = true;
        if (brk == anchor) {  // anchor exhausted in exact mode: walk it unbounded
            if (tid == anchor) {
                walk<MODE>(s, e, cend, r);
                atomicAdd(nwalks, 1u);
            }
        } else if (xst == S_ERR) {
            if (tid >= brk) {
                e = NONE;
                lane_set(r, S_ERR, X);
                r.ek = xek;
            }
        } else if (xst == S_OK) {
            if (tid >= brk) {
                if (stop <= X) {  // pass-through (including chunks past the frame end)
                    e = NONE;
                    lane_set(r, S_NONE, NONE);
                } else if (cend - CHUNK <= X) {  // this chunk contains X
                    e = X;
                    walk<MODE>(s, e, cend, r);
                    atomicAdd(nwalks, 1u);
                }
            }
        } else {
            progressed = false;
        }
        __syncthreads();
        if (!progressed) return rounds;
    }
}

// Summary of a contiguous run of tiles (or of an inclusive prefix), composed old -> young.
struct Seg {
    bool any;        // covers at least one tile
    bool ok;         // internally consistent
    uint64_t in;     // entry the run requires (NONE: not composable)
    uint64_t out;    // exit (or error offset when dead)
    uint32_t ek;     // error kind when dead
    uint64_t rows, ch, ctl, hb;
};

// old ∘ young
NXG_DEV Seg compose(const Seg& o, const Seg& y) {
    if (!o.any) return y;
    if (!y.any || o.ek) return o;
    Seg r = y;
    r.ok = o.ok && y.ok && y.in == o.out;
    r.in = o.in;
    r.rows = o.rows + y.rows;
    r.ch = o.ch + y.ch;
    r.ctl = o.ctl + y.ctl;
    r.hb = o.hb + y.hb;
    return r;
}

}  // namespace

__global__ __launch_bounds__(TPB) void nxg_dec_general_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, ColsDesc cols, uint64_t* __restrict__ slots,
    uint32_t ntiles, uint32_t epoch, DevStatus* __restrict__ st, int emit, DevStatus* zst) {
    zero_status(zst);
    __shared__ __attribute__((aligned(16))) uint8_t buf[TILE + HALO];
    __shared__ uint64_t sx[TPB];
    __shared__ uint32_t sst[TPB];
    __shared__ uint64_t se[TPB];
    __shared__ uint64_t scan64[4];
    __shared__ uint32_t scan32[4];
    __shared__ uint32_t wfirst[4];
    __shared__ uint32_t wtop[4];
    __shared__ uint64_t bx[2];
    __shared__ uint64_t sh_texit;
    __shared__ uint32_t sh_tek;
    __shared__ uint32_t sh_flag;
    __shared__ uint64_t sh_E, sh_rows, sh_ch, sh_ctl, sh_hb;
    __shared__ uint32_t sh_ek, sh_timeout, sh_fallback;
    __shared__ uint32_t dg_walks, dg_tries, dg_exh;

    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const Sink sink{cols, &st->capacity, &st->nonf64};

    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t t0 = (uint64_t)tile * TILE;
        const uint64_t navail = W - t0;
        const uint32_t nlds = (uint32_t)(navail < (uint64_t)(TILE + HALO) ? navail : (TILE + HALO));
        if (tid == 0) {
            dg_walks = 0;
            dg_tries = 0;
            dg_exh = 0;
        }
        for (uint32_t i = tid; i < (TILE + HALO) / 16; i += TPB) {
            const uint64_t o = t0 + 16ull * i;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (o + 16 <= W) {
                v = *reinterpret_cast<const uint4*>(wire + o);
            } else if (o < W) {
                uint32_t w[4] = {0, 0, 0, 0};
                for (int k = 0; k < 16; k++)
                    if (o + k < W) w[k >> 2] |= (uint32_t)wire[o + k] << (8 * (k & 3));
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            *reinterpret_cast<uint4*>(buf + 16 * i) = v;
        }
        __syncthreads();
        const Src s{buf, t0, nlds, wire, W};
        const uint64_t c = t0 + (uint64_t)tid * CHUNK;
        const uint64_t cend = c + CHUNK;

        // 1. speculate + bounded walk + block repair
        uint32_t tries = 0;
        uint64_t e = (tile == 0 && tid == 0) ? 0 : speculate(s, c, cend, tries);
        LaneRes r;
        if (e != NONE) walk<M_BOUNDED>(s, e, cend, r);
        else lane_set(r, S_NONE, NONE);
        atomicAdd(&dg_tries, tries);
        if (e != NONE) atomicAdd(&dg_walks, 1u);
        {
            const uint64_t m = __ballot(e != NONE);
            if (lane == 0) wfirst[wv] = m ? wv * 64 + (uint32_t)__builtin_ctzll(m) : 0xffffu;
        }
        __syncthreads();
        uint32_t jstar = 0xffffu;
        for (int i = 0; i < 4; i++) jstar = min(jstar, wfirst[i]);
        __syncthreads();
        // the tile's guess = the first lane with a guess; repair the chain from there
        bool complete = false;
        uint32_t rounds1 = 0;
        if (tid == 0) {
            sh_texit = NONE;
            sh_tek = 0;
        }
        if (jstar < TPB)
            rounds1 = repair<M_BOUNDED>(s, cend, jstar, e, r, sx, sst, wtop, wfirst, bx,
                                        &dg_walks, complete, &sh_texit, &sh_tek);
        if (r.st == S_EXH) atomicAdd(&dg_exh, 1u);

        // 2. tile aggregate: entry = the anchor's guess, exit = last lane's exit; composable
        // only if the repair verified every lane from the anchor on
        uint32_t trows, tctl, thb;
        uint64_t tch;
        block_excl_scan<uint32_t, TPB>(r.rows, scan32, &trows);
        block_excl_scan<uint32_t, TPB>(r.ctl, scan32, &tctl);
        block_excl_scan<uint32_t, TPB>(r.hb, scan32, &thb);
        block_excl_scan<uint64_t, TPB>(r.children, scan64, &tch);
        if (tid == jstar) se[0] = e;
        __syncthreads();
        const bool composable = jstar < TPB && complete;
        const uint64_t tspec = jstar < TPB ? se[0] : NONE;
        const uint64_t texit = sh_texit;
        const uint32_t tek = sh_tek;
        __syncthreads();
        uint64_t* d = slots + (uint64_t)tile * SLOT_WORDS;
        if (tid == 0 && tile != 0) {
            st_agent(d + A_CHILD, tch);
            st_agent(d + A_CTLHB, (uint64_t)tctl | ((uint64_t)thb << 32));
            st_agent(d + A_SPEC, composable ? tspec : NONE);
            st_agent(d + A_EXIT, texit);
            st_agent(d + A_ERR, tek ? (((uint64_t)tek << 56) | (texit & POSM)) : 0ull);
            drain_stores();
            st_agent(d + W_FLAG, lb_word(kFlagAgg, epoch, trows));
        }

        // 3. look-back (wave 0): compose predecessors old -> young into the true entry
        if (wv == 0) {
            Seg acc{false, true, NONE, 0, 0, 0, 0, 0, 0};
            uint32_t timeout = 0;
            bool fallback = false;
            if (tile == 0) {
                acc = Seg{true, true, 0, 0, 0, 0, 0, 0, 0};
            } else {
                const uint64_t t_start = rt_now();
                int64_t pred = (int64_t)tile - 1;
                bool done = false;
                while (!done) {
                    const int64_t idx = pred - (int64_t)lane;
                    const uint64_t* q = slots + (uint64_t)(idx < 0 ? 0 : idx) * SLOT_WORDS;
                    uint64_t f = idx >= 0 ? ld_agent(q + W_FLAG) : lb_word(kFlagInc, epoch, 0);
                    while (!__all(lb_flag(f, epoch) != 0)) {
                        __builtin_amdgcn_s_sleep(1);
                        if (lb_flag(f, epoch) == 0) f = ld_agent(q + W_FLAG);
                        if (rt_now() - t_start > kSpinTicks) {
                            timeout = 1;
                            break;
                        }
                    }
                    if (timeout) break;
                    const bool isinc = lb_flag(f, epoch) == kFlagInc;
                    uint64_t xch = 0, xctlhb = 0, xspec = NONE, xexit = 0, xerr = 0;
                    if (idx >= 0) {
                        if (isinc) {
                            xch = ld_agent(q + I_CHILD);
                            xctlhb = ld_agent(q + I_CTLHB);
                            xexit = ld_agent(q + I_EXIT);
                            xerr = ld_agent(q + I_ERR);
                        } else {
                            xch = ld_agent(q + A_CHILD);
                            xctlhb = ld_agent(q + A_CTLHB);
                            xspec = ld_agent(q + A_SPEC);
                            xexit = ld_agent(q + A_EXIT);
                            xerr = ld_agent(q + A_ERR);
                        }
                    }
                    const uint64_t incm = __ballot(isinc);
                    const int fi = incm ? __builtin_ctzll(incm) : 64;  // youngest inclusive
                    const int hi = fi - 1;                              // aggregate lanes [0, hi]
                    Seg w{hi >= 0, true, NONE, 0, 0, 0, 0, 0, 0};
                    if (hi >= 0) {
                        const uint64_t errm = __ballot((int)lane <= hi && xerr != 0);
                        const int ms = errm ? 63 - __builtin_clzll(errm) : -1;  // oldest error
                        const uint64_t older_exit = __shfl_down(xexit, 1, 64);
                        bool bad = false;
                        if ((int)lane <= hi && (int)lane >= (ms < 0 ? 0 : ms)) {
                            if (xspec == NONE) bad = true;
                            else if ((int)lane < hi && older_exit != xspec) bad = true;
                        }
                        w.ok = !__any(bad);
                        w.in = __shfl(xspec, hi, 64);
                        if (ms >= 0) {
                            const uint64_t er = __shfl(xerr, ms, 64);
                            w.ek = (uint32_t)(er >> 56);
                            w.out = er & POSM;
                        } else {
                            w.out = __shfl(xexit, 0, 64);
                        }
                        const bool in = (int)lane <= hi;
                        w.rows = wave_sum<uint64_t>(in ? (f & kValMask) : 0ull);
                        w.ch = wave_sum<uint64_t>(in ? xch : 0ull);
                        w.ctl = wave_sum<uint64_t>(in ? (xctlhb & 0xffffffffull) : 0ull);
                        w.hb = wave_sum<uint64_t>(in ? (xctlhb >> 32) : 0ull);
                    }
                    acc = compose(w, acc);
                    if (!acc.ok) {
                        fallback = true;
                        break;
                    }
                    if (fi < 64) {
                        Seg inc{true, true, 0, 0, 0, 0, 0, 0, 0};
                        inc.rows = __shfl(f & kValMask, fi, 64);
                        inc.ch = __shfl(xch, fi, 64);
                        const uint64_t cb = __shfl(xctlhb, fi, 64);
                        inc.ctl = cb & 0xffffffffull;
                        inc.hb = cb >> 32;
                        const uint64_t er = __shfl(xerr, fi, 64);
                        inc.ek = (uint32_t)(er >> 56);
                        inc.out = inc.ek ? (er & POSM) : __shfl(xexit, fi, 64);
                        acc = compose(inc, acc);
                        if (!acc.ok) fallback = true;
                        done = true;
                    } else {
                        pred -= 64;
                    }
                }
                if (!timeout && fallback) {
                    // wait for the immediate predecessor's inclusive prefix
                    const uint64_t* q = slots + (uint64_t)(tile - 1) * SLOT_WORDS;
                    uint64_t f = ld_agent(q + W_FLAG);
                    while (lb_flag(f, epoch) != kFlagInc) {
                        __builtin_amdgcn_s_sleep(2);
                        f = ld_agent(q + W_FLAG);
                        if (rt_now() - t_start > kSpinTicks) {
                            timeout = 1;
                            break;
                        }
                    }
                    acc.any = true;
                    acc.ok = true;
                    acc.rows = f & kValMask;
                    acc.ch = ld_agent(q + I_CHILD);
                    const uint64_t cb = ld_agent(q + I_CTLHB);
                    acc.ctl = cb & 0xffffffffull;
                    acc.hb = cb >> 32;
                    const uint64_t er = ld_agent(q + I_ERR);
                    acc.ek = (uint32_t)(er >> 56);
                    acc.out = acc.ek ? (er & POSM) : ld_agent(q + I_EXIT);
                }
            }
            if (lane == 0) {
                sh_E = acc.out;
                sh_ek = acc.ek;
                sh_rows = acc.rows;
                sh_ch = acc.ch;
                sh_ctl = acc.ctl;
                sh_hb = acc.hb;
                sh_timeout = timeout;
                sh_fallback = fallback;
                if (timeout) atomicOr(&st->timeout, 1u);
            }
        }
        __syncthreads();
        const uint64_t E = sh_E;
        const bool dead = sh_ek != 0 || sh_timeout != 0;

        // 4. exact phase from the true entry when the guess was wrong or a walk gave up
        const bool redo = !dead && (E != tspec || !composable);
        uint32_t rounds2 = 0;
        if (redo) {
            if (tid == 0) {
                e = E;
                walk<M_EXACT>(s, e, cend, r);
                atomicAdd(&dg_walks, 1u);
            }
            bool done;
            rounds2 = repair<M_EXACT>(s, cend, 0, e, r, sx, sst, wtop, wfirst, bx, &dg_walks,
                                      done, &sh_texit, &sh_tek);
            if (!done && tid == 0) atomicOr(&st->timeout, 1u);  // unreachable by design
        }

        // 5. per-lane bases; tile exit
        const bool live = !dead && e != NONE && r.st == S_OK;
        uint32_t r_tot, c_tot, h_tot;
        uint64_t ch_tot;
        const uint32_t rb = block_excl_scan<uint32_t, TPB>(live ? r.rows : 0u, scan32, &r_tot);
        const uint32_t cb = block_excl_scan<uint32_t, TPB>(live ? r.ctl : 0u, scan32, &c_tot);
        block_excl_scan<uint32_t, TPB>(live ? r.hb : 0u, scan32, &h_tot);
        const uint64_t chb =
            block_excl_scan<uint64_t, TPB>(live ? r.children : 0ull, scan64, &ch_tot);
        uint64_t out_x = sh_texit;  // from the last completed repair
        uint32_t out_ek = sh_tek;
        if (dead) {
            out_x = E;
            out_ek = sh_ek;
        }
        const uint64_t row0 = sh_rows, ch0 = sh_ch, ctl0 = sh_ctl, hb0 = sh_hb;
        __syncthreads();

        // 6. publish the inclusive prefix (+ final status from the last tile)
        if (tid == 0) {
            st_agent(d + I_CHILD, ch0 + ch_tot);
            st_agent(d + I_CTLHB, (ctl0 + c_tot) | ((hb0 + h_tot) << 32));
            st_agent(d + I_EXIT, out_x);
            st_agent(d + I_ERR, out_ek ? (((uint64_t)out_ek << 56) | (out_x & POSM)) : 0ull);
            drain_stores();
            st_agent(d + W_FLAG, lb_word(kFlagInc, epoch, row0 + r_tot));
            if (tile == ntiles - 1) {
                st->n_rows = row0 + r_tot;
                st->n_children = ch0 + ch_tot;
                st->n_ctl = ctl0 + c_tot;
                st->n_heartbeat = hb0 + h_tot;
                st->err_kind = out_ek;
                st->err_offset = out_ek ? out_x : 0;
                st->path = 2;
            }
            atomicAdd(&st->diag[0], redo ? 1ull : 0ull);
            atomicAdd(&st->diag[1], sh_fallback ? 1ull : 0ull);
            atomicAdd(&st->diag[2], (unsigned long long)(rounds1 + rounds2));
            atomicAdd(&st->diag[3], (unsigned long long)dg_walks);
            atomicAdd(&st->diag[4], (unsigned long long)dg_tries);
            atomicAdd(&st->diag[5], jstar < TPB ? 0ull : 1ull);
            atomicAdd(&st->diag[6], (unsigned long long)dg_exh);
        }

        // 7. emit: decode again, writing the columns (skipped once the frame is rejected)
        if (emit && live && out_ek == 0) {
            uint64_t row = row0 + rb, ctl = ctl0 + cb, child = ch0 + chb;
            uint64_t pos = e;
            const uint64_t stop = cend < W ? cend : W;
            uint32_t work = 0;
            while (pos < stop) {
                MsgInfo mi;
                const uint32_t err =
                    decode_msg<true, M_EXACT>(s, pos, mi, &sink, row, child, work);
                if (err) break;  // unreachable: the walk validated this chain
                if (mi.variant == 4) {
                    if (row < cols.cap_rows) cols.id[row] = mi.id;
                    else atomicOr(&st->capacity, 1u);
                    row++;
                } else if (!cols.ctl_row) {
                    atomicOr(&st->nonf64, 1u);
                    ctl++;
                } else {
                    if (ctl < cols.cap_ctl) {
                        cols.ctl_row[ctl] = row;
                        cols.ctl_off[ctl] = pos;
                        cols.ctl_len[ctl] = (uint32_t)(mi.next - pos);
                        cols.ctl_variant[ctl] = (uint8_t)mi.variant;
                    } else {
                        atomicOr(&st->capacity, 1u);
                    }
                    ctl++;
                }
                pos = mi.next;
            }
        }
        __syncthreads();
    }
}

hipError_t nxg_launch_dec_general(const uint8_t* wire, uint64_t W, const ColsDesc& cd,
                                  uint64_t* tslots, uint32_t epoch, DevStatus* st, int emit,
                                  int grid, hipStream_t s) {
    const uint64_t nt = (W + TILE - 1) / TILE;
    if (nt == 0) return hipSuccess;
    const uint64_t g = grid <= 0 ? nt : (nt < (uint64_t)grid ? nt : (uint64_t)grid);
    hipLaunchKernelGGL(nxg_dec_general_kernel, dim3(g), dim3(TPB), 0, s, wire, W, cd, tslots,
                       (uint32_t)nt, epoch, st, emit, nxg_zero_slot);
    return hipGetLastError();
}

int nxg_occupancy_dec_general() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, nxg_dec_general_kernel, TPB, 0) !=
        hipSuccess)
        return 1;
    return n;
}
