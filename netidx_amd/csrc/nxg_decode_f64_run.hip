// nxg_decode_f64_run.hip -- homogeneous-f64 decode by length-run speculation, for gfx950.
// Replaces the receive_batch_fn loop (netidx/src/channel.rs:504-521) for frames in which every
// message is From::Update(Id, F64):
//     varint(L) 04 varint(id) 09 f64be     L = lw(10 + vl(id)) = 11 + vl(id)
// (len_wrapped_encode pack.rs:527-535, derive lib.rs:289-381, Value::encode lib.rs:404-407).
// Ids of 1..5 varint bytes (< 2^35) are decoded here, so records are 12..16 bytes long.
//
// Why speculation works. Record k+1 starts at s_k + L_k: the boundaries are a pointer chain.
// But L depends only on the id's varint width, and publisher ids come from a per-process
// counter (netidx-core/src/utils.rs:130-134), so the ids of a batch change width only at 2^7,
// 2^14, 2^21, 2^28: almost every 16 KiB tile is a run of records of ONE length. For such a tile
// the record count follows from its first record alone: n = ceil((T - e) / L).
//
//   probe  (one lane per tile): the tile's entry e (the unique valid record start in its first
//          16 bytes), L from that record, n, and a check of the predicted last record. A tile
//          whose prediction fails (a width change, a false candidate) is counted exactly by the
//          whole wave (merge points, below). Counts -> block scan -> decoupled look-back across
//          workgroups -> each tile's first record index. Reads ~64 B per tile.
//   emit   (one wave per tile, no inter-workgroup waits): every record of a uniform tile is at
//          e + kL; lane j decodes records j, j+64, ... with two 16-byte loads each, checks it
//          completely (length, variant 4, id varint width, value tag 9) and stores straight to
//          the id / value columns (64 consecutive rows per store: coalesced). Exact tiles are
//          re-walked from their merge points. Each tile's chain exit must equal the next
//          tile's entry (and the last one the frame end), so a wrong speculation can cost
//          speed, never correctness: any failed check raises fast_fail and the host reruns the
//          frame on the general decoder.
//
// Merge points (exact tiles): the first record at or after a chunk start c lies in [c, c+16);
// every valid record start in that window starts a walk, and the walks are advanced in position
// order until they coincide. The true chain passes through the merge point, which depends only
// on the bytes, so the lane that owns the previous chunk computes the same position.
#include <vector>

#include "nxg_device.h"
#include "nxg_f64_rec16.h"

namespace f64r {
#ifndef NXG_F64R_T
#define NXG_F64R_T 32768
#endif
constexpr uint32_t T = NXG_F64R_T;  // tile bytes (the probe's unit)
#ifndef NXG_F64R_EREC
#define NXG_F64R_EREC 256
#endif
constexpr uint32_t EREC = NXG_F64R_EREC;  // records per emit wave (a tile's records, in order)
constexpr uint32_t ESUB = (T / 12 + EREC) / EREC;  // emit waves per tile (records >= 12 B)
static_assert(T + 16 <= 65535, "Desc.x is 16 bits");
constexpr uint32_t IMGB = f64rec16::kXImg;  // exact path (nxg_f64_rec16.h): LDS image per wave
constexpr int TPB = 256;
constexpr uint32_t MODE_EXACT = 0;  // Desc.mode: 12..16 = uniform record length

constexpr uint32_t F_FORCE_EXACT = 1;  // probe flags (tests): every tile on the exact path
constexpr uint32_t F_NO_BAIL = 2;      //   never give up on an irregular frame
constexpr uint32_t F_FIRST = 4;        // the decoded range starts at the frame's first byte
constexpr uint32_t F_LAST = 8;         // the decoded range ends at the frame's last byte
constexpr uint32_t F_XCD = 16;         // emit: XCD-contiguous workgroup -> tile mapping
constexpr uint64_t kXcdMin = 256ull << 20;  // ranges past the Infinity Cache (256 MiB)

// Per-tile descriptor written by the probe, read by the emit pass. A tile is one or two runs of
// records of one length each: records [0, ks) of length L from `entry`, then records [ks, count)
// of length L2; or an exact tile (mode 0: merge points).
struct Desc {
    uint64_t base;   // first record index
    uint16_t count;  // records starting in the tile (<= T / 12)
    uint16_t ks;     // records in the first run
    uint16_t x;      // chain exit, relative to the tile start (next tile's entry + T)
    uint8_t entry;   // first record start, relative to the tile start (0..15)
    uint8_t mode;    // bits 0-2: L - 11, bits 3-5: L2 - 11; 0 = exact tile
};
static_assert(sizeof(Desc) == 16, "Desc is one 16-byte load");
}  // namespace f64r

namespace {
using namespace f64r;
using namespace f64rec16;

}  // namespace

// 32 bytes at frame offset off (16-aligned) as dwords
NXG_DEV void ld32(const uint8_t* __restrict__ wire, uint64_t off, uint64_t W, uint32_t (&q)[8]) {
    const uint4 a = ld16g(wire, off, W), b = ld16g(wire, off + 16, W);
    q[0] = a.x, q[1] = a.y, q[2] = a.z, q[3] = a.w;
    q[4] = b.x, q[5] = b.y, q[6] = b.z, q[7] = b.w;
}
// length of the valid record at tile-relative position p (0 if none)
NXG_DEV uint32_t rec_len_at(const uint8_t* __restrict__ wire, uint64_t W, uint64_t t0,
                            uint32_t p) {
    uint32_t q[8], e0, e1, e2, e3;
    ld32(wire, t0 + (p & ~15u), W, q);
    extract16(q, p & 15u, e0, e1, e2, e3);
    return rec_check16(e0, e1, W - t0 - p);
}

// length of the valid record at tile-relative position p (0 if none) and its id
NXG_DEV uint32_t rec_at(const uint8_t* __restrict__ wire, uint64_t W, uint64_t t0, uint32_t p,
                        uint64_t& id) {
    uint32_t q[8], e0, e1, e2, e3;
    ld32(wire, t0 + (p & ~15u), W, q);
    extract16(q, p & 15u, e0, e1, e2, e3);
    const uint32_t L = rec_check16(e0, e1, W - t0 - p);
    uint64_t v;
    rec_decode16(e0, e1, e2, e3, L ? L : 12u, id, v);
    return L;
}

// Two-run search, by the whole wave, for a tile whose records do not all have the first
// record's length L: the first k whose position e + kL holds no record of length L (64 samples,
// then the 64 positions after the last good sample), the second run's length L2 there, and a
// check of that run's middle and last records. Returns false if the tile is not two runs.
NXG_DEV bool run_search(const uint8_t* __restrict__ wire, uint64_t W, uint64_t t0, uint32_t e,
                        uint32_t L, uint32_t lim, uint32_t lane, uint32_t& ks, uint32_t& L2,
                        uint32_t& n, uint32_t& x) {
    const uint32_t n1 = (lim - e + L - 1) / L;  // records if the whole tile were one run
    const uint32_t step = (n1 + 62) / 63;
    const uint32_t ki = lane == 63 ? n1 - 1 : min(lane * step, n1 - 1);
    const bool good = rec_len_at(wire, W, t0, e + ki * L) == L;
    const uint64_t badm = __ballot(!good);
    if (!badm) return false;
    const uint32_t ib = __builtin_ctzll(badm);  // first bad sample (never lane 0: k = 0 is good)
    const uint32_t khi = (uint32_t)__builtin_amdgcn_readlane((int)ki, ib);
    const uint32_t klo = ib ? (uint32_t)__builtin_amdgcn_readlane((int)ki, ib - 1) + 1 : 0u;
    const uint32_t k2 = min(klo + lane, khi);
    const uint32_t l2 = rec_len_at(wire, W, t0, e + k2 * L);
    const uint64_t bm2 = __ballot(l2 != L);
    const uint32_t j = __builtin_ctzll(bm2);  // bm2 != 0: k = khi is bad
    ks = klo + j;
    L2 = (uint32_t)__builtin_amdgcn_readlane((int)l2, j);
    if (L2 == 0 || L2 == L) return false;
    const uint32_t p2 = e + ks * L;
    const uint32_t n2 = (lim - p2 + L2 - 1) / L2;
    // the second run: 64 samples, its last record included
    const uint32_t kc = lane == 63 ? n2 - 1 : lane * (n2 - 1) / 63;
    const bool ok = rec_len_at(wire, W, t0, p2 + kc * L2) == L2;
    if (!__all(ok)) return false;
    n = ks + n2;
    x = p2 + n2 * L2;
    return true;
}

// The probe's fast path for tile t (one lane): the entry, the run model (one or two runs of one
// record length each, split where consecutive ids change width) and samples that confirm it.
// state 0: the model holds (count, x set); 1: one length, the split not found (run_search);
// 2: no unique entry or forced (exact path). `bad`: the frame cannot be decoded from here.
NXG_DEV void probe_fast(const uint8_t* __restrict__ wire, uint64_t W, uint64_t t, uint32_t lim,
                        bool first, uint32_t flags, int& state, uint32_t& e, uint32_t& L,
                        uint32_t& L2, uint32_t& ks, uint32_t& count, uint32_t& x, bool& bad,
                        bool& nof) {
    const uint64_t t0 = t * T;
    const uint64_t rem0 = W - t0;
    uint32_t d[8];
    ld32(wire, t0, W, d);
    uint32_t cand = cand16(d[0], d[1], d[2], d[3], d[4]);
    uint32_t V = 0;  // valid record starts (and the frame end) in [0, 16)
    if (rem0 < 16) V |= 1u << rem0;
    while (cand) {
        const uint32_t s = __builtin_ctz(cand);
        cand &= cand - 1;
        uint32_t e0, e1, e2, e3;
        extract16(d, s, e0, e1, e2, e3);
        if (rec_check16(e0, e1, rem0 - s)) V |= 1u << s;
    }
    // the entry is the lowest valid start; the only other start allowed in the window is
    // its successor (a record of <= 16 bytes leaves room for one more)
    const uint32_t s1 = V ? (uint32_t)__builtin_ctz(V) : 32u;
    uint32_t L1 = 0;
    if (s1 < 16 && s1 != rem0) {
        uint32_t e0, e1, e2, e3;
        extract16(d, s1, e0, e1, e2, e3);
        L1 = e0 & 0xffu;
    }
    const uint32_t p2 = s1 + L1;
    // every 16 bytes of an f64 frame hold a record start (records are 12..16 bytes): none here,
    // or no record at the frame's first byte, and the frame is not an f64 frame at all
    nof = V == 0u || (t == 0 && first && !(V & 1u));
    if (t == 0 && first && !(V & 1u)) {
        bad = true;
    } else if (s1 < 16 && (s1 == rem0 || s1 >= lim)) {
        // the frame (or the range) ends here: no record of this range starts in the tile
        e = x = s1;
        L = L2 = 12;
    } else if (s1 < 16 && V == ((1u << s1) | (p2 < 16 ? 1u << p2 : 0u))) {
        e = s1;
        L = L2 = L1;
        uint32_t n = (lim - e + L - 1) / L;
        ks = n;
        // Ids from the publisher's counter are consecutive (utils.rs:130-134): if the first
        // id plus n crosses the next varint width, the tile is predicted as two runs split
        // where the ids reach it.
        uint64_t id0;
        {
            uint32_t e0, e1, e2, e3;
            extract16(d, e, e0, e1, e2, e3);
            uint64_t v0;
            rec_decode16(e0, e1, e2, e3, L, id0, v0);
            const uint32_t nb = L - 11u;
            const uint64_t next = 1ull << (7u * nb);
            if (nb < 5 && id0 < next && id0 + n > next) {
                ks = (uint32_t)(next - id0);
                L2 = L + 1;
                const uint32_t q2 = e + ks * L;
                n = ks + (lim - q2 + L2 - 1) / L2;
            }
        }
        // the prediction's last record and both sides of the split must have the predicted
        // lengths and ids (one HBM line per sample; the emit pass checks every record)
        auto at = [&](uint32_t k) { return k < ks ? e + k * L : e + ks * L + (k - ks) * L2; };
        auto len = [&](uint32_t k) { return k < ks ? L : L2; };
        const uint32_t m = n - 1;
        const uint32_t ke = ks < n ? ks - 1 : m, kf = ks < n ? ks : m;
        // the three samples are independent: loaded together (one memory round trip)
        uint64_t ia, ie, iff;
        const uint32_t la = rec_at(wire, W, t0, at(m), ia);
        const uint32_t le = rec_at(wire, W, t0, at(ke), ie);
        const uint32_t lf = rec_at(wire, W, t0, at(kf), iff);
        const bool lok =
            ((int)(la == len(m)) & (int)(le == len(ke)) & (int)(lf == len(kf))) != 0;
        bool ok = lok && ia == id0 + m && ie == id0 + ke && iff == id0 + kf;
        if (!ok && lok && ks == n) {
            // one length, ids not consecutive: one more sample, the middle record
            uint64_t ib;
            ok = rec_at(wire, W, t0, at(m / 2), ib) == L;
        }
        if (ok) {
            count = n;
            x = at(n);
        } else {
            ks = n = (lim - e + L - 1) / L;  // back to one run for the wave's search
            L2 = L;
            state = 1;
        }
    } else {
        state = 2;  // a false candidate, or no valid start: let the merge points decide
    }
    if ((flags & F_FORCE_EXACT) && !bad) state = 2;

}

// ---- probe: one lane per tile ------------------------------------------------------------------
// wire: the decoded range's first byte; W: bytes from there to the frame end; R (<= W): the
// range's length (records that START before R are the range's; the rest is look-ahead)
// One frame's probe (or emit) launch arguments. The fused launch (nxg_f64r_fused_kernel) takes
// one of each: the emit of frame j and the probe of frame j + 1 of a stream of frames.
struct ProbeArgs {
    const uint8_t* wire;
    uint64_t W, R, pre, nt;
    Desc* desc;
    uint64_t* tstat;
    uint32_t epoch, flags;
    DevStatus* st;
    DevStatus* zst;
};
struct EmitArgs {
    const uint8_t* wire;
    uint64_t W, R, pre, nt;
    const Desc* desc;
    uint64_t* oid;
    uint64_t* oval;
    uint64_t cap;
    uint32_t flags, ne;  // ne: the emit's workgroups (the XCD remap's grid)
    DevStatus* st;
};

// bid: this workgroup's probe index (the workgroups of one probe are numbered 0.. in dispatch
// order: the look-back waits only on lower ones)
NXG_DEV void probe_body(const ProbeArgs& a, uint32_t bid, uint8_t (*img)[IMGB],
                        uint64_t* scan_tmp, uint64_t& sh_base) {
    const uint8_t* __restrict__ wire = a.wire;
    const uint64_t W = a.W, R = a.R, pre = a.pre, nt = a.nt;
    Desc* __restrict__ desc = a.desc;
    uint64_t* tstat = a.tstat;
    const uint32_t epoch = a.epoch, flags = a.flags;
    DevStatus* __restrict__ st = a.st;
    if (bid == 0 && threadIdx.x == 0 && a.zst) *a.zst = DevStatus{};
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t t = (uint64_t)bid * TPB + tid;
    const bool has = t < nt;
    const uint64_t t0 = t * T;
    const uint32_t lim = has ? (R - t0 < T ? (uint32_t)(R - t0) : T) : 0u;
    const bool first = flags & F_FIRST;
    uint32_t count = 0, e = 0, x = 0, L = 0, L2 = 0, ks = 0;
    int state = 0;  // 0 done, 1 run search, 2 exact
    bool bad = false, nof = false;
    if (has) probe_fast(wire, W, t, lim, first, flags, state, e, L, L2, ks, count, x, bad, nof);
    // a frame that is not f64 at all (DevStatus.irregular bit 1): the host goes on to the mixed
    // decoders. An irregular frame (record lengths that change from record to record: more than
    // 1 tile in 8 off the runs, here or in any workgroup so far; bit 0) is left to the
    // single-pass decoder, which the host reruns it on.
    const int nnof = __syncthreads_count(nof);
    const int nirr = __syncthreads_count(state != 0);
    const uint64_t ntg = nt - (uint64_t)bid * TPB < TPB ? nt - (uint64_t)bid * TPB
                                                               : TPB;
    const bool bail = !(flags & F_NO_BAIL) &&
                      (nnof || (uint64_t)nirr * 8 > ntg || (nirr && ld_agent32(&st->irregular)));
    if (bail) {
        if (tid == 0) {
            atomicOr(&st->irregular, nnof ? 2u : 1u);
            atomicOr(&st->fast_fail, 1u);
        }
        state = 0;
    }
    // width changes inside a tile: two runs, found by the whole wave
    uint64_t em = __ballot(state == 1);
    while (em) {
        const uint32_t j = __builtin_ctzll(em);
        em &= em - 1;
        const uint64_t tj = (uint64_t)bid * TPB + w * 64 + j;
        const uint32_t ej = (uint32_t)__builtin_amdgcn_readlane((int)e, j);
        const uint32_t Lj = (uint32_t)__builtin_amdgcn_readlane((int)L, j);
        const uint32_t limj = (uint32_t)__builtin_amdgcn_readlane((int)lim, j);
        uint32_t ksj, L2j, nj, xj;
        const bool two = run_search(wire, W, tj * T, ej, Lj, limj, lane, ksj, L2j, nj, xj);
        if (lane == j) {
            if (two) {
                state = 0;
                ks = ksj;
                L2 = L2j;
                count = nj;
                x = xj;
            } else {
                state = 2;
            }
        }
    }
    // anything else: counted exactly by the whole wave
    em = __ballot(state == 2);
    while (em) {
        const uint32_t j = __builtin_ctzll(em);
        em &= em - 1;
        uint32_t c, en, xx;
        bool b = false, ov = false;
        exact_tile<false, T>(wire, W, R, first, pre, (uint64_t)bid * TPB + w * 64 + j,
                          img[w], lane, 0, nullptr, nullptr, 0, c, en, xx, b, ov);
        if (lane == j) {
            count = c;
            e = en;
            x = xx;
            L = 0;
            bad |= b;
        }
        if (lane == 0) atomicAdd(&st->diag[0], 1ull);  // exact tiles (diagnostics)
    }
    if (__any(bad) && lane == 0) atomicOr(&st->fast_fail, 1u);
    uint64_t total;
    const uint64_t excl = block_excl_scan<uint64_t, TPB>(count, scan_tmp, &total);
    if (w == 0) {
        uint64_t base = 0;
        if (bid == 0) {
            if (lane == 0) st_agent(&tstat[0], lb_word(kFlagInc, epoch, total));
        } else {
            if (lane == 0) st_agent(&tstat[bid], lb_word(kFlagAgg, epoch, total));
            bool give_up;
            base = lookback_prefix<4>(tstat, bid, epoch, nullptr, give_up);
            if (give_up) {
                if (lane == 0) {
                    atomicOr(&st->timeout, 1u);
                    atomicOr(&st->fast_fail, 1u);
                }
            } else if (lane == 0) {
                st_agent(&tstat[bid], lb_word(kFlagInc, epoch, base + total));
            }
        }
        if (lane == 0) sh_base = base;
    }
    __syncthreads();
    if (has) {
        Desc o;
        o.base = sh_base + excl;
        o.count = (uint16_t)count;
        o.ks = (uint16_t)ks;
        o.x = (uint16_t)x;
        o.entry = (uint8_t)e;
        o.mode = L ? (uint8_t)((L - 11u) | ((L2 - 11u) << 3)) : (uint8_t)MODE_EXACT;
        desc[t] = o;
    }
}

// The probe's workgroups take their tile groups by ticket (DevStatus.diag[6], zeroed with the
// slot): its look-back then waits only on workgroups that are running (next_tile).
__global__ __launch_bounds__(TPB) void nxg_f64r_probe_kernel(ProbeArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t img[TPB / 64][IMGB];
    __shared__ uint64_t scan_tmp[TPB / 64];
    __shared__ uint64_t sh_base;
    __shared__ uint32_t sh_tile;
    probe_body(a, next_tile(&a.st->diag[6], &sh_tile), img, scan_tmp, sh_base);
}

// ---- emit: one wave per tile ---------------------------------------------------------------------
#ifndef NXG_F64R_NT
#define NXG_F64R_NT 0  // bit 0: nontemporal column stores, bit 1: nontemporal wire loads,
#endif                 // bit 2: nontemporal stores only for lines no other wave writes
#ifndef NXG_F64R_R
#define NXG_F64R_R 4   // records per lane loaded together
#endif
#ifndef NXG_F64R_DPP
#define NXG_F64R_DPP 1  // a record's second 16-byte block from the next lane (one load per record)
#endif
#ifndef NXG_F64R_LDS
#define NXG_F64R_LDS 0  // 64 records' bytes as one aligned 1 KiB load per wave, through LDS
#endif
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
NXG_DEV uint4 ld16s(const uint8_t* __restrict__ p) {
    if (NXG_F64R_NT & 2) {
        const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return ld16r(p);
}
NXG_DEV void st_col(uint64_t* p, uint64_t v, bool inner) {
    if ((NXG_F64R_NT & 1) || ((NXG_F64R_NT & 4) && inner)) __builtin_nontemporal_store(v, p);
    else *p = v;
}
// A run tile: record k < ks at e + kL, record k >= ks at e + ks L + (k - ks) L2; lane j decodes
// records j, j + 64, ...; R records per lane are loaded together.
template <bool GUARD>
NXG_DEV bool emit_runs(const uint8_t* __restrict__ wire, uint64_t W, uint64_t t0, uint32_t e,
                       uint32_t L, uint32_t ks, uint32_t L2, uint32_t klo, uint32_t n,
                       uint64_t base,
                       uint64_t* __restrict__ oid, uint64_t* __restrict__ oval, uint64_t cap,
                       uint32_t lane, uint8_t* lbuf, bool& over) {
    constexpr int R = NXG_F64R_R;
    bool bad = false;
    const uint64_t r1 = t0 + e, r2 = t0 + e + (uint64_t)ks * L;
    // rows in the first and last 128-byte line of the tile's rows share the line with the
    // neighbouring tiles' rows
    const uint64_t lfirst = (base + klo) >> 4, llast = (base + n - 1) >> 4;
    auto pos = [&](uint32_t k) -> uint64_t {
        return k < ks ? r1 + (uint64_t)k * L : r2 + (uint64_t)(k - ks) * L2;
    };
    for (uint32_t kb = klo; kb < n; kb += 64 * R) {
        uint32_t d[R][8];
        uint64_t p[R];
        if (NXG_F64R_LDS) {
            // the R x 64 records' bytes: one aligned, fully coalesced 1 KiB load per wave and
            // batch (lane i: block i; lane 0 also block 64), then each lane reads the two blocks
            // holding its record from LDS. Records are <= 16 bytes, so 64 of them starting in
            // block 0 end by block 64.
            uint64_t ab[R];
            uint4 A[R], X[R];
#pragma unroll
            for (int r = 0; r < R; r++) {
                const uint32_t kf = kb + r * 64 < n ? kb + r * 64 : n - 1;
                ab[r] = pos(kf) & ~15ull;
                A[r] = GUARD ? ld16g(wire, ab[r] + 16 * lane, W) : ld16s(wire + ab[r] + 16 * lane);
                if (lane == 0)
                    X[r] = GUARD ? ld16g(wire, ab[r] + 1024, W) : ld16s(wire + ab[r] + 1024);
            }
            wave_lds_order();
#pragma unroll
            for (int r = 0; r < R; r++) {
                uint4* blk = reinterpret_cast<uint4*>(lbuf + r * 1040);
                blk[lane] = A[r];
                if (lane == 0) blk[64] = X[r];
            }
            wave_lds_order();
#pragma unroll
            for (int r = 0; r < R; r++) {
                const uint32_t k0 = kb + r * 64 + lane;
                p[r] = pos(k0 < n ? k0 : n - 1);
                const uint32_t q = (uint32_t)(p[r] - ab[r]) >> 4;
                const uint4* blk = reinterpret_cast<const uint4*>(lbuf + r * 1040);
                const uint4 a = blk[q], b = blk[q + 1];
                d[r][0] = a.x, d[r][1] = a.y, d[r][2] = a.z, d[r][3] = a.w;
                d[r][4] = b.x, d[r][5] = b.y, d[r][6] = b.z, d[r][7] = b.w;
            }
        } else {
            uint4 B[R];
#pragma unroll
            for (int r = 0; r < R; r++) {
                const uint32_t k0 = kb + r * 64 + lane;
                const uint32_t k = k0 < n ? k0 : n - 1;  // clamp: the loads stay unconditional
                p[r] = pos(k);
                const uint64_t a = p[r] & ~15ull;
                const uint4 A = GUARD ? ld16g(wire, a, W) : ld16s(wire + a);
                d[r][0] = A.x, d[r][1] = A.y, d[r][2] = A.z, d[r][3] = A.w;
                if (!NXG_F64R_DPP) {
                    B[r] = GUARD ? ld16g(wire, a + 16, W) : ld16s(wire + a + 16);
                } else if (lane == 63 || k0 + 1 >= n) {
                    B[r] = GUARD ? ld16g(wire, a + 16, W) : ld16s(wire + a + 16);
                }
            }
#pragma unroll
            for (int r = 0; r < R; r++) {
                if (NXG_F64R_DPP) {
                    // Records are <= 16 bytes and lane j + 1 holds the record after lane j's, so
                    // when lane j's record runs past its 16-byte block, the next block is exactly
                    // lane j + 1's first one; when it does not, bytes 16..31 are never read. Lane
                    // 63 and the lanes at or past the last record loaded it themselves.
                    const uint32_t k0 = kb + r * 64 + lane;
                    const bool own = lane == 63 || k0 + 1 >= n;
                    const uint32_t n0 = wave_next(d[r][0]), n1 = wave_next(d[r][1]),
                                   n2 = wave_next(d[r][2]), n3 = wave_next(d[r][3]);
                    d[r][4] = own ? B[r].x : n0;
                    d[r][5] = own ? B[r].y : n1;
                    d[r][6] = own ? B[r].z : n2;
                    d[r][7] = own ? B[r].w : n3;
                } else {
                    d[r][4] = B[r].x, d[r][5] = B[r].y, d[r][6] = B[r].z, d[r][7] = B[r].w;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; r++) {
            const uint32_t k = kb + r * 64 + lane;
            const uint32_t Lk = (k < n ? k : n - 1) < ks ? L : L2;
            uint32_t e0, e1, e2, e3;
            extract16(d[r], (uint32_t)p[r] & 15u, e0, e1, e2, e3);
            bad |= rec_check16(e0, e1, W - p[r]) != Lk;
            uint64_t id, val;
            rec_decode16(e0, e1, e2, e3, Lk, id, val);
            const uint64_t row = base + k;
            if (k < n) {
                if (row < cap) {
                    const bool inner = (row >> 4) != lfirst && (row >> 4) != llast;
                    st_col(&oid[row], id, inner);
                    st_col(&oval[row], val, inner);
                } else {
                    over = true;
                }
            }
        }
    }
    return bad;
}


#ifndef NXG_F64R_PAIR
#define NXG_F64R_PAIR 0  // 1: lane j decodes two consecutive records, one 16-byte store per column
                         // (measured: 10^8 equal, 10^7 4 % slower than one 8-byte store per row)
#endif
constexpr int RP = 2;  // pair slots per lane loaded together (128 records each)

// A run tile in pairs of rows (record k is row base + k). The lane of pair P decodes rows 2P and
// 2P + 1 and writes each column's two rows with ONE 16-byte store (2P is even, so the store is
// 16-byte aligned): a wave stores 1 KiB per instruction instead of 512 B. Its two records lie in
// the 48 bytes from the aligned 16-byte block of the first: the lane loads blocks A and B, and
// the third, C, is the next lane's A or B (the next lane's first record starts 24..32 bytes after
// ours, so its aligned block is 16 or 32 bytes past ours); lane 63 and the lanes at the end of
// the range load C themselves. Edge pairs with one row of the range store that row alone.
template <bool GUARD>
NXG_DEV bool emit_pairs(const uint8_t* __restrict__ wire, uint64_t W, uint64_t t0, uint32_t e,
                        uint32_t L, uint32_t ks, uint32_t L2, uint32_t klo, uint32_t n,
                        uint64_t base, uint64_t* __restrict__ oid, uint64_t* __restrict__ oval,
                        uint64_t cap, uint32_t lane, bool& over) {
    bool bad = false;
    const uint64_t r1 = t0 + e, r2 = t0 + e + (uint64_t)ks * L;
    auto pos = [&](uint32_t k) -> uint64_t {
        return k < ks ? r1 + (uint64_t)k * L : r2 + (uint64_t)(k - ks) * L2;
    };
    const uint64_t P0 = (base + klo) >> 1, P1 = ((base + n - 1) >> 1) + 1;
    const int64_t lo = klo, hi = (int64_t)n - 1;
    for (uint64_t Pb = P0; Pb < P1; Pb += 64 * RP) {
        uint32_t A[RP][4], B[RP][4], C[RP][4];
        int64_t k0[RP];
        uint64_t pa[RP], pb[RP], ab[RP];
        uint32_t la[RP], lb[RP];
        bool own[RP];
#pragma unroll
        for (int r = 0; r < RP; r++) {
            k0[r] = (int64_t)(2 * (Pb + (uint64_t)r * 64 + lane)) - (int64_t)base;
            // clamped into the range: the loads stay unconditional (edge lanes decode a
            // neighbour again and store nothing for it)
            const uint32_t ka = (uint32_t)min(max(k0[r], lo), hi);
            const uint32_t kb = (uint32_t)min(max(k0[r] + 1, lo), hi);
            pa[r] = pos(ka);
            pb[r] = pos(kb);
            la[r] = ka < ks ? L : L2;
            lb[r] = kb < ks ? L : L2;
            ab[r] = pa[r] & ~15ull;
            const uint4 x = GUARD ? ld16g(wire, ab[r], W) : ld16s(wire + ab[r]);
            const uint4 y = GUARD ? ld16g(wire, ab[r] + 16, W) : ld16s(wire + ab[r] + 16);
            A[r][0] = x.x, A[r][1] = x.y, A[r][2] = x.z, A[r][3] = x.w;
            B[r][0] = y.x, B[r][1] = y.y, B[r][2] = y.z, B[r][3] = y.w;
            own[r] = lane == 63 || k0[r] + 2 > hi;
            if (own[r]) {
                const uint4 z = ld16g(wire, ab[r] + 32, W);
                C[r][0] = z.x, C[r][1] = z.y, C[r][2] = z.z, C[r][3] = z.w;
            }
        }
#pragma unroll
        for (int r = 0; r < RP; r++) {
            uint32_t nA[4], nB[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                nA[q] = wave_next(A[r][q]);
                nB[q] = wave_next(B[r][q]);
            }
            if (!own[r]) {
                const bool at32 = ((pb[r] + lb[r]) & ~15ull) == ab[r] + 32;
#pragma unroll
                for (int q = 0; q < 4; q++) C[r][q] = at32 ? nA[q] : nB[q];
            }
        }
#pragma unroll
        for (int r = 0; r < RP; r++) {
            const uint32_t d[8] = {A[r][0], A[r][1], A[r][2], A[r][3],
                                   B[r][0], B[r][1], B[r][2], B[r][3]};
            uint32_t e0, e1, e2, e3;
            extract16(d, (uint32_t)(pa[r] - ab[r]), e0, e1, e2, e3);
            bad |= rec_check16(e0, e1, W - pa[r]) != la[r];
            uint64_t ida, va;
            rec_decode16(e0, e1, e2, e3, la[r], ida, va);
            const uint32_t sb = (uint32_t)(pb[r] - ab[r]);  // 0..31
            const bool up = sb >= 16;
            uint32_t d2[8];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                d2[q] = up ? B[r][q] : A[r][q];
                d2[q + 4] = up ? C[r][q] : B[r][q];
            }
            extract16(d2, sb & 15u, e0, e1, e2, e3);
            bad |= rec_check16(e0, e1, W - pb[r]) != lb[r];
            uint64_t idb, vb;
            rec_decode16(e0, e1, e2, e3, lb[r], idb, vb);
            const uint64_t row = base + (uint64_t)k0[r];  // even
            const bool oka = k0[r] >= lo && k0[r] <= hi, okb = k0[r] + 1 >= lo && k0[r] + 1 <= hi;
            if (oka && okb && row + 1 < cap) {
                *reinterpret_cast<uint4*>(oid + row) =
                    make_uint4((uint32_t)ida, (uint32_t)(ida >> 32), (uint32_t)idb,
                               (uint32_t)(idb >> 32));
                *reinterpret_cast<uint4*>(oval + row) =
                    make_uint4((uint32_t)va, (uint32_t)(va >> 32), (uint32_t)vb,
                               (uint32_t)(vb >> 32));
            } else {
                if (oka) {
                    if (row < cap) {
                        oid[row] = ida;
                        oval[row] = va;
                    } else {
                        over = true;
                    }
                }
                if (okb) {
                    if (row + 1 < cap) {
                        oid[row + 1] = idb;
                        oval[row + 1] = vb;
                    } else {
                        over = true;
                    }
                }
            }
        }
    }
    return bad;
}

// wave g of the emit: tile g / ESUB, its records [EREC * (g % ESUB), EREC * (g % ESUB + 1)) (in
// pair mode the inner boundaries move down by base & 1, so that every wave but the first starts
// on an even row)
NXG_DEV void emit_body(const EmitArgs& a, uint32_t blk, uint8_t (*img)[IMGB]) {
    const uint8_t* __restrict__ wire = a.wire;
    const uint64_t W = a.W, R = a.R, pre = a.pre, nt = a.nt;
    const Desc* __restrict__ desc = a.desc;
    const uint32_t flags = a.flags;
    DevStatus* __restrict__ st = a.st;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // Workgroups go to the 8 XCDs round-robin. A frame larger than the Infinity Cache streams
    // from HBM: there each XCD takes a contiguous eighth of it (10^8 records: 0.567-0.574 vs
    // 0.579-0.583 ms over 4 interleaved runs); a cache-resident frame keeps the plain order
    // (10^7: 0.063-0.066 vs 0.062-0.063 ms).
    uint64_t bid = blk;
    if (flags & F_XCD) {
        const uint32_t nb = a.ne, q = nb / 8, r = nb % 8, x = blk % 8;
        bid = (uint64_t)x * q + min(x, r) + blk / 8;
    }
    const uint64_t g = bid * (TPB / 64) + w;
    const uint64_t t = g / ESUB;
    const uint32_t sub = (uint32_t)(g % ESUB);
    if (t >= nt) return;
    if (st->fast_fail) return;  // the probe rejected the frame (previous launch: plain load)
    const Desc D = desc[t];
    const uint32_t shift = NXG_F64R_PAIR ? (uint32_t)(D.base & 1) : 0u;
    const uint32_t klo = sub ? sub * EREC - shift : 0u;
    if (D.mode == MODE_EXACT ? sub != 0 : (sub && klo >= D.count)) return;
    const uint32_t kend = (sub + 1) * EREC - shift;
    const uint32_t khi = D.count < kend ? D.count : kend;
    const uint64_t t0 = t * T;
    bool bad = false, over = false;
    if (sub == 0) {
        // the chain: this tile's exit is the next tile's entry; the last tile ends at the
        // frame end
        if (t + 1 < nt) bad |= (uint32_t)D.x != T + desc[t + 1].entry;
        else if (flags & F_LAST) bad |= t0 + D.x != W;  // a range's exit is linked by the host
        if (t == nt - 1 && lane == 0) {
            st->n_rows = D.base + D.count;
            st->path = 1;
        }
    }
    if (D.mode != MODE_EXACT) {
        if (khi > klo) {
            const uint32_t L = 11u + (D.mode & 7u), L2 = 11u + ((D.mode >> 3) & 7u);
            const bool guard = t0 + T + 32 > W;
            if (NXG_F64R_PAIR) {
                if (!guard)
                    bad |= emit_pairs<false>(wire, W, t0, D.entry, L, D.ks, L2, klo, khi, D.base,
                                             a.oid, a.oval, a.cap, lane, over);
                else
                    bad |= emit_pairs<true>(wire, W, t0, D.entry, L, D.ks, L2, klo, khi, D.base,
                                            a.oid, a.oval, a.cap, lane, over);
            } else {
                if (!guard)
                    bad |= emit_runs<false>(wire, W, t0, D.entry, L, D.ks, L2, klo, khi, D.base,
                                            a.oid, a.oval, a.cap, lane, img[w], over);
                else
                    bad |= emit_runs<true>(wire, W, t0, D.entry, L, D.ks, L2, klo, khi, D.base,
                                           a.oid, a.oval, a.cap, lane, img[w], over);
            }
        }
    } else {
        uint32_t c, en, xx;
        bool b = false;
        exact_tile<true, T>(wire, W, R, flags & F_FIRST, pre, t, img[w], lane, D.base, a.oid, a.oval,
                         a.cap, c, en, xx, b, over);
        bad |= b || c != D.count || en != D.entry || xx != D.x;
    }
    if (__any(bad) && lane == 0) atomicOr(&st->fast_fail, 1u);
    if (__any(over) && lane == 0) atomicOr(&st->capacity, 1u);
}

__global__ __launch_bounds__(TPB) void nxg_f64r_emit_kernel(EmitArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t img[TPB / 64][IMGB];
    emit_body(a, blockIdx.x, img);
}

// A stream of frames (nxg_decode_frames_async): the emit of frame j and the probe of frame j + 1
// in ONE launch. Workgroups [0, npg) are the probe's (its real workgroups, then idle ones up to a
// multiple of 8, so that the emit's workgroups keep their XCD), dispatched first; the probe's
// look-back waits only on lower-numbered probe workgroups, and no emit workgroup waits on
// anything, so every wait is on a workgroup dispatched earlier. The probe is latency-bound (about
// one wave per 8 KiB tiles' worth of CUs): beside the streaming emit it costs the emit little,
// and it leaves the critical path of back-to-back decodes.
__global__ __launch_bounds__(TPB) void nxg_f64r_fused_kernel(EmitArgs ea, ProbeArgs pa,
                                                             uint32_t npg) {
    __shared__ __attribute__((aligned(16))) uint8_t img[TPB / 64][IMGB];
    __shared__ uint64_t scan_tmp[TPB / 64];
    __shared__ uint64_t sh_base;
    __shared__ uint32_t sh_tile;
    if (blockIdx.x < npg) {
        const uint32_t bid = next_tile(&pa.st->diag[6], &sh_tile);
        if ((uint64_t)bid * TPB < pa.nt) probe_body(pa, bid, img, scan_tmp, sh_base);
        return;
    }
    emit_body(ea, blockIdx.x - npg, img);
}

uint64_t nxg_dec_f64r_tiles(uint64_t W) { return (W + T - 1) / T; }
uint64_t nxg_dec_f64r_tile_bytes() { return T; }
uint64_t nxg_dec_f64r_groups(uint64_t W) { return (nxg_dec_f64r_tiles(W) + TPB - 1) / TPB; }

namespace {
// the launch arguments of the records that start in [begin, end) of a W-byte frame
bool f64r_args(const uint8_t* wire, uint64_t W, uint64_t begin, uint64_t end, uint64_t* oid,
               uint64_t* oval, uint64_t cap, void* desc, uint64_t* tstat, uint32_t epoch,
               uint32_t flags, DevStatus* st, DevStatus* zst, ProbeArgs& pa, EmitArgs& ea,
               uint32_t& ng) {
    if (begin > end || end > W) return false;
    const uint64_t R = end - begin;
    const uint64_t nt = nxg_dec_f64r_tiles(R);
    const uint64_t ne = (nt * ESUB + TPB / 64 - 1) / (TPB / 64);
    if (ne > 0x7fffffffull) return false;
    flags = (flags & (F_FORCE_EXACT | F_NO_BAIL)) | (begin == 0 ? F_FIRST : 0u) |
            (end == W ? F_LAST : 0u) | (R > kXcdMin ? F_XCD : 0u);
    const uint64_t pre = begin < 64 ? begin : 64;
    pa = ProbeArgs{wire + begin, W - begin, R, pre, nt, reinterpret_cast<Desc*>(desc), tstat,
                   epoch, flags, st, zst};
    ea = EmitArgs{wire + begin, W - begin, R, pre, nt, reinterpret_cast<const Desc*>(desc),
                  oid, oval, cap, flags, (uint32_t)ne, st};
    ng = (uint32_t)nxg_dec_f64r_groups(R);
    return true;
}
}  // namespace

// Decodes the records that start in [begin, end) of a frame of W bytes (a whole frame: 0, W).
// `desc` holds nxg_dec_f64r_tiles(end - begin) 16-byte descriptors, `tstat`
// nxg_dec_f64r_groups(end - begin) epoch-tagged words; neither needs initialisation.
// flags: F_FORCE_EXACT / F_NO_BAIL (tests); F_FIRST / F_LAST are set here.
hipError_t nxg_launch_dec_f64r(const uint8_t* wire, uint64_t W, uint64_t begin, uint64_t end,
                               uint64_t* oid, uint64_t* oval, uint64_t cap, void* desc,
                               uint64_t* tstat, uint32_t epoch, uint32_t flags, DevStatus* st,
                               hipStream_t s) {
    ProbeArgs pa;
    EmitArgs ea;
    uint32_t ng;
    if (!f64r_args(wire, W, begin, end, oid, oval, cap, desc, tstat, epoch, flags, st, nullptr, pa,
                   ea, ng))
        return hipErrorInvalidValue;
    if (pa.nt == 0) return hipSuccess;
    pa.zst = nxg_take_zero_slot();
    hipLaunchKernelGGL(nxg_f64r_probe_kernel, dim3(ng), dim3(TPB), 0, s, pa);
    hipLaunchKernelGGL(nxg_f64r_emit_kernel, dim3(ea.ne), dim3(TPB), 0, s, ea);
    return hipGetLastError();
}

// A stream of whole frames, decoded in order: probe(0), then per frame j one fused launch of
// (10^8 records, warm streams on one box: 0.549-0.550 ms per frame fused against 0.555-0.557 ms
// with probe and emit launched apart; 10^7: 0.057-0.062 against 0.063-0.070 ms per call)
// emit(j) + probe(j + 1). Consecutive frames alternate between two descriptor arrays (fr[j].desc),
// since probe(j + 1) runs beside emit(j). Frames of no bytes launch nothing.
hipError_t nxg_launch_dec_f64r_stream(const NxgF64rFrame* fr, uint32_t n, uint64_t* tstat,
                                      uint32_t flags, hipStream_t s) {
    std::vector<ProbeArgs> pa(n);
    std::vector<EmitArgs> ea(n);
    std::vector<uint32_t> ng(n);
    for (uint32_t j = 0; j < n; j++)
        if (!f64r_args(fr[j].wire, fr[j].W, 0, fr[j].W, fr[j].oid, fr[j].oval, fr[j].cap,
                       fr[j].desc, tstat, fr[j].epoch, flags, fr[j].st, fr[j].zst, pa[j], ea[j],
                       ng[j]))
            return hipErrorInvalidValue;
    int32_t prev = -1;  // the last frame whose probe ran, its emit not yet launched
    for (uint32_t j = 0; j <= n; j++) {
        const bool has = j < n && pa[j].nt > 0;
        if (j < n && !has) continue;
        if (prev < 0) {
            if (has) hipLaunchKernelGGL(nxg_f64r_probe_kernel, dim3(ng[j]), dim3(TPB), 0, s, pa[j]);
        } else if (!has) {
            hipLaunchKernelGGL(nxg_f64r_emit_kernel, dim3(ea[prev].ne), dim3(TPB), 0, s, ea[prev]);
        } else {
            const uint32_t npg = (ng[j] + 7u) & ~7u;
            if ((uint64_t)npg + ea[prev].ne > 0x7fffffffull) return hipErrorInvalidValue;
            hipLaunchKernelGGL(nxg_f64r_fused_kernel, dim3(npg + ea[prev].ne), dim3(TPB), 0, s,
                               ea[prev], pa[j], npg);
        }
        prev = has ? (int32_t)j : -1;
    }
    return hipGetLastError();
}
