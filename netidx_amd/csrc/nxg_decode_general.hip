// nxg_decode_general.hip -- general From-stream decode for gfx950 (every From variant, every
// Value tag, nesting, errors), single pass over the wire.
//
// This is the receive_batch_fn loop (netidx/src/channel.rs:504-521) for arbitrary frames.
// Message boundaries form a pointer chain (len_wrapped_decode, pack.rs:537-555), and a message
// may be arbitrarily long. They are resolved in parallel by speculation with exact repair:
//
//  * lane: each lane owns a 32-byte chunk. It guesses its first message start: the first
//    position from which two consecutive messages decode plausibly. From that guess it walks the
//    messages that START inside its chunk with the full validating decoder, and records its
//    exit (the first message start past its chunk) and its counts.
//  * block repair: a lane whose guess differs from its predecessor's exit re-walks from that
//    exit. Iterating to a fixed point makes every lane exact relative to the tile's entry.
//  * tile: descriptors {speculated entry, exit, counts, first error} are published as
//    aggregates, and later as inclusive prefixes, through a decoupled look-back. A tile
//    composes its predecessors' aggregates only when each aggregate's entry equals the exit of
//    the tile before it. Otherwise it waits for its predecessor's inclusive prefix. If its own
//    guess proves wrong, the tile re-runs the block repair from the true entry.
//  * emit: with exact lane entries and global bases, every lane decodes its messages again and
//    writes the columns.
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
    W_FLAG = 0,   // flag(63:62) | rows (aggregate) or rows prefix (inclusive)
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

struct LaneRes {
    uint64_t x;  // exit (first message start at/after the chunk end), or error position
    uint32_t rows, ctl, hb;
    uint64_t children;
    uint32_t ek;  // error kind, 0 = none
};

NXG_DEV void lane_clear(LaneRes& r, uint64_t x) {
    r.x = x;
    r.rows = r.ctl = r.hb = 0;
    r.children = 0;
    r.ek = 0;
}

// full validating walk of the messages starting in [e, end)
NXG_DEV void walk(const Src& s, uint64_t e, uint64_t end, LaneRes& r) {
    lane_clear(r, e);
    uint64_t pos = e;
    const uint64_t stop = end < s.W ? end : s.W;
    while (pos < stop) {
        MsgInfo mi;
        uint64_t ch = 0;
        const uint32_t err = decode_msg<false, false>(s, pos, mi, nullptr, 0, ch);
        if (err) {
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

// first position in [c, end) from which two messages decode plausibly (cheap checks only)
NXG_DEV uint64_t speculate(const Src& s, uint64_t c, uint64_t end) {
    const uint64_t stop = end < s.W ? end : s.W;
    for (uint64_t p = c; p < stop; p++) {
        MsgInfo mi;
        uint64_t ch = 0;
        if (decode_msg<false, true>(s, p, mi, nullptr, 0, ch)) continue;
        if (mi.next >= s.W) return p;
        MsgInfo m2;
        if (decode_msg<false, true>(s, mi.next, m2, nullptr, 0, ch) == E_OK) return p;
    }
    return NONE;
}

// Block repair: every lane's entry becomes its predecessor's exit (lane 0 is fixed). A lane
// whose predecessor died inherits the error. Lanes before the first definite entry stay NONE.
NXG_DEV void repair(const Src& s, uint64_t cend, uint64_t& e, LaneRes& r, uint64_t* sx,
                    uint32_t* sek, uint32_t* sflag) {
    const uint32_t tid = threadIdx.x;
    for (;;) {
        sx[tid] = r.x;
        sek[tid] = r.ek | (e == NONE ? 0x80000000u : 0u);
        if (tid == 0) *sflag = 0;
        __syncthreads();
        bool ch = false;
        if (tid > 0) {
            const uint32_t pk = sek[tid - 1];
            const uint64_t px = sx[tid - 1];
            const bool pnone = (pk & 0x80000000u) && (pk & 0x7fffffffu) == 0;
            const uint32_t perr = pk & 0x7fffffffu;
            if (perr) {  // chain dies before this lane: no messages, inherit the error
                if (!(r.ek == perr && r.x == px && e == NONE)) {
                    e = NONE;
                    lane_clear(r, px);
                    r.ek = perr;
                    ch = true;
                }
            } else if (!pnone && px != e) {
                e = px;
                walk(s, e, cend, r);
                ch = true;
            }
        }
        if (ch) atomicOr(sflag, 1u);
        __syncthreads();
        const bool any = *sflag != 0;
        __syncthreads();
        if (!any) return;
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
    __shared__ uint32_t sek[TPB];
    __shared__ uint64_t se[TPB];
    __shared__ uint64_t scan64[4];
    __shared__ uint32_t scan32[4];
    __shared__ uint32_t wfirst[4];
    __shared__ uint32_t sh_flag;
    __shared__ uint64_t sh_E, sh_rows, sh_ch, sh_ctl, sh_hb;
    __shared__ uint32_t sh_ek, sh_timeout;

    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const Sink sink{cols, &st->capacity, &st->nonf64};

    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t t0 = (uint64_t)tile * TILE;
        const uint64_t navail = W - t0;
        const uint32_t nlds = (uint32_t)(navail < (uint64_t)(TILE + HALO) ? navail : (TILE + HALO));
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

        // 1. speculate + walk + block repair
        uint64_t e = (tile == 0 && tid == 0) ? 0 : speculate(s, c, cend);
        LaneRes r;
        if (e != NONE) walk(s, e, cend, r);
        else lane_clear(r, NONE);
        repair(s, cend, e, r, sx, sek, &sh_flag);

        // 2. tile aggregate: entry = first definite lane's entry, exit = last lane's exit
        {
            const uint64_t m = __ballot(e != NONE);
            if (lane == 0) wfirst[wv] = m ? wv * 64 + (uint32_t)__builtin_ctzll(m) : 0xffffu;
            se[tid] = e;
        }
        uint32_t trows, tctl, thb;
        uint64_t tch;
        block_excl_scan<uint32_t, TPB>(r.rows, scan32, &trows);
        block_excl_scan<uint32_t, TPB>(r.ctl, scan32, &tctl);
        block_excl_scan<uint32_t, TPB>(r.hb, scan32, &thb);
        block_excl_scan<uint64_t, TPB>(r.children, scan64, &tch);
        uint32_t jstar = 0xffffu;
        for (int i = 0; i < 4; i++) jstar = min(jstar, wfirst[i]);
        const uint64_t tspec = jstar < TPB ? se[jstar] : NONE;
        const uint64_t texit = sx[TPB - 1];
        const uint32_t tek = sek[TPB - 1] & 0x7fffffffu;
        uint64_t* d = slots + (uint64_t)tile * SLOT_WORDS;
        if (tid == 0 && tile != 0) {
            st_agent(d + A_CHILD, tch);
            st_agent(d + A_CTLHB, (uint64_t)tctl | ((uint64_t)thb << 32));
            st_agent(d + A_SPEC, tek ? tspec : (tspec == NONE ? NONE : tspec));
            st_agent(d + A_EXIT, texit);
            st_agent(d + A_ERR, tek ? (((uint64_t)tek << 56) | (texit & POSM)) : 0ull);
            drain_stores();
            st_agent(d + W_FLAG, lb_word(kFlagAgg, epoch, trows));
        }

        // 3. look-back (wave 0): compose predecessors old -> young into the true entry
        if (wv == 0) {
            Seg acc{false, true, NONE, 0, 0, 0, 0, 0, 0};
            uint32_t timeout = 0;
            if (tile == 0) {
                acc = Seg{true, true, 0, 0, 0, 0, 0, 0, 0};
            } else {
                const uint64_t t_start = rt_now();
                int64_t pred = (int64_t)tile - 1;
                bool fallback = false, done = false;
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
                    // window summary of the aggregate lanes (young part of this window)
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
                        if (idx < 0 && fi == (int)lane) {
                        }
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
                if (timeout) atomicOr(&st->timeout, 1u);
            }
        }
        __syncthreads();
        const uint64_t E = sh_E;
        const bool dead = sh_ek != 0 || sh_timeout != 0;

        // 4. redo from the true entry when the speculation was wrong
        if (!dead && tile != 0 && E != tspec) {
            if (tid == 0) {
                e = E;
                walk(s, e, cend, r);
            }
            repair(s, cend, e, r, sx, sek, &sh_flag);
        }

        // 5. per-lane bases; tile exit
        const bool live = !dead && e != NONE;
        uint32_t r_tot, c_tot, h_tot;
        uint64_t ch_tot;
        const uint32_t rb = block_excl_scan<uint32_t, TPB>(live ? r.rows : 0u, scan32, &r_tot);
        const uint32_t cb = block_excl_scan<uint32_t, TPB>(live ? r.ctl : 0u, scan32, &c_tot);
        block_excl_scan<uint32_t, TPB>(live ? r.hb : 0u, scan32, &h_tot);
        const uint64_t chb = block_excl_scan<uint64_t, TPB>(live ? r.children : 0ull, scan64, &ch_tot);
        if (tid == TPB - 1) {
            sx[0] = r.x;
            sek[0] = r.ek;
        }
        __syncthreads();
        uint64_t out_x = sx[0];
        uint32_t out_ek = sek[0];
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
        }

        // 7. emit: decode again, writing the columns (skipped once the frame is rejected)
        if (emit && live && out_ek == 0) {
            uint64_t row = row0 + rb, ctl = ctl0 + cb, child = ch0 + chb;
            uint64_t pos = e;
            const uint64_t stop = cend < W ? cend : W;
            while (pos < stop) {
                MsgInfo mi;
                const uint32_t err = decode_msg<true, false>(s, pos, mi, &sink, row, child);
                if (err) break;  // unreachable: the walk validated this chain
                if (mi.variant == 4) {
                    if (row < cols.cap_rows) cols.id[row] = mi.id;
                    else atomicOr(&st->capacity, 1u);
                    row++;
                } else if (!cols.ctl_row) {
                    atomicOr(&st->nonf64, 1u);
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
    const int g = (int)(nt < (uint64_t)grid ? nt : (uint64_t)grid);
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
