// nxg_decode_f64_seq.hip -- one-launch decode of an f64 frame whose ids count up by one, for gfx950.
// Replaces the receive_batch_fn loop (netidx/src/channel.rs:504-521) for the commonest publisher
// batch: every value of a publisher updated in publication order. Publisher ids come from a
// per-process counter (netidx-core/src/utils.rs:130-134), so such a batch is
//     record k = varint(L_k) 04 varint(i0 + k) 09 f64be,    L_k = 11 + vl(i0 + k)
// (len_wrapped_encode pack.rs:527-535, derive lib.rs:289-381, Value::encode lib.rs:404-407), and
// where record k starts is a closed form of k: the id widths change only at 2^7, 2^14, 2^21, 2^28,
// so pos(k) is linear in k between those points. Nothing has to be searched or scanned:
//
//   - every wave reads the frame's first record (i0) and solves pos(N) = W for the record count N
//     (no solution: the frame is not such a batch);
//   - wave g decodes records [256 g, 256 g + 256): lane j takes records j, j + 64, ... four at a
//     time, one 16-byte load each (the record's second block is lane j + 1's first, by DPP), and
//     checks every record completely: length byte, variant 4, id varint width, value tag 9, AND
//     id == i0 + k; then 64 consecutive rows per column store.
//
// Why that is the reference's decode exactly: record 0 starts at byte 0; if record k at pos(k) is a
// valid Update of length L_k then the sequential decoder's next message starts at
// pos(k) + L_k = pos(k + 1); by induction it visits exactly pos(0..N) and pos(N) = W ends the frame.
// Non-canonical varints, other ids or other messages fail a check: the frame is rejected with
// DevStatus.irregular bit 2 (bit 1: the first record is not an f64 Update at all) and the host
// reruns it on the length-run decoder (nxg_decode_f64_run.hip), which takes any f64 frame. A wrong
// guess costs one pass, never correctness; the host then skips this decoder for a while.
//
// No descriptors, no look-back, no inter-workgroup waits: a pure streaming kernel, W bytes read and
// 16 N written, nothing else but the 32-byte head every wave reads (an L2 hit).
#include "nxg_device.h"
#include "nxg_f64_rec16.h"

namespace f64s {
constexpr int TPB = 256;
#ifndef NXG_F64S_R
#define NXG_F64S_R 8  // records per lane loaded together (4 pairs), frames past the Infinity Cache
#endif
#ifndef NXG_F64S_R_SMALL
#define NXG_F64S_R_SMALL 4  // ... and frames within it (A/B: 4 is 2 % faster at 10^7, 8 at 10^8)
#endif
#ifndef NXG_F64S_NT
#define NXG_F64S_NT 1  // bit 0: nontemporal column stores, bit 1: nontemporal wire loads
#endif
constexpr uint64_t kXcdMin = 256ull << 20;  // frames past the Infinity Cache (256 MiB)
// records per lane for a frame of W bytes
inline int r_for(uint64_t W) { return W >= kXcdMin ? NXG_F64S_R : NXG_F64S_R_SMALL; }
#ifndef NXG_F64S_XCD
#define NXG_F64S_XCD 1  // XCD-contiguous record ranges for frames past the Infinity Cache
#endif
#ifndef NXG_F64S_LDS
#define NXG_F64S_LDS 0  // dynamic LDS per workgroup (A/B: caps the waves per CU)
#endif
constexpr uint32_t F_XCD = 1;
#ifndef NXG_F64S_XRUN
#define NXG_F64S_XRUN 64  // workgroups per XCD run (frames past the Infinity Cache)
#endif
constexpr uint64_t XRUN = NXG_F64S_XRUN;

// pos(k), the byte where record k starts (f64rec16::seq_pos)
NXG_DEV uint64_t pos_of(uint64_t i0, uint64_t k) { return f64rec16::seq_pos(i0, k); }

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
NXG_DEV uint4 ld16s(const uint8_t* __restrict__ p) {
    if (NXG_F64S_NT & 2) {
        const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return f64rec16::ld16r(p);
}
NXG_DEV void st_col(uint64_t* p, uint64_t v) {
    if (NXG_F64S_NT & 1) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// The wave's records k0 + k, k in [0, n): k < ks at p0 + k L, then at p0 + ks L + (k - ks)(L + 1).
// The frame's last wave (and any wave within 32 bytes of its end): one record per lane at a time,
// both blocks loaded with the frame-end guard (rare; kept lean so it does not set the kernel's
// register count). Returns true if any record fails a check.
NXG_DEV bool emit_edge(const uint8_t* __restrict__ wire, uint64_t W, uint64_t p0, uint32_t L,
                       uint32_t ks, uint32_t n, uint64_t k0, uint64_t i0,
                       uint64_t* __restrict__ oid, uint64_t* __restrict__ oval, uint64_t cap,
                       uint32_t lane, bool& over) {
    using namespace f64rec16;
    const uint32_t L2 = L + 1;
    bool bad = false;
#pragma unroll 1
    for (uint32_t k = lane; k < n; k += 64) {
        const uint64_t p = p0 + (k < ks ? (uint64_t)k * L : (uint64_t)ks * L + (uint64_t)(k - ks) * L2);
        const uint64_t a = p & ~15ull;
        const uint4 A = ld16g(wire, a, W), B = ld16g(wire, a + 16, W);
        const uint32_t d[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
        const uint32_t Lk = k < ks ? L : L2;
        uint32_t e0, e1, e2, e3;
        extract16(d, (uint32_t)p & 15u, e0, e1, e2, e3);
        uint64_t id, val;
        rec_decode16(e0, e1, e2, e3, Lk, id, val);
        const uint64_t row = k0 + k;
        bad |= (rec_check16(e0, e1, W - p) != Lk) | (id != i0 + row);
        if (row < cap) {
            oid[row] = id;
            oval[row] = val;
        } else {
            over = true;
        }
    }
    return bad;
}

// A whole wave of WREC records away from the frame's end (the common case). Offsets are 32-bit
// from the 16-byte block holding record k0 (a wave spans at most 4 KiB), so the loads take a
// scalar base and the wave keeps only the R blocks it loaded in registers: lane j's record's second
// block is lane j + 1's first (DPP), and lane 63's is lane 0's of the next batch (readlane), or
// for the last batch one more block that lane 63 loads.
template <int R>
NXG_DEV bool emit_full(const uint8_t* __restrict__ wire, uint64_t W, uint64_t p0, uint32_t L,
                       uint32_t ks, uint64_t k0, uint64_t i0, uint64_t* __restrict__ oid,
                       uint64_t* __restrict__ oval, uint64_t cap, uint32_t lane, bool& over) {
    using namespace f64rec16;
    const uint64_t a0 = p0 & ~15ull;
    const uint8_t* __restrict__ base = wire + a0;
    const uint32_t s0 = (uint32_t)(p0 & 15u);
    const uint32_t L2 = L + 1;
    auto off = [&](uint32_t k) -> uint32_t {  // record k0 + k, from base
        return s0 + (k < ks ? k * L : ks * L + (k - ks) * L2);
    };
    uint4 A[R];
    uint32_t o[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
        o[r] = off(r * 64 + lane);
        A[r] = ld16s(base + (o[r] & ~15u));
    }
    // lane 63 of the last batch: the block after its record's
    uint4 E = make_uint4(0, 0, 0, 0);
    if (lane == 63) E = ld16s(base + (o[R - 1] & ~15u) + 16);
    bool bad = false;
    const uint64_t ib = i0 + k0;  // the id of record k0
#pragma unroll
    for (int r = 0; r < R; r++) {
        uint32_t d[8] = {A[r].x, A[r].y, A[r].z, A[r].w, 0, 0, 0, 0};
        d[4] = wave_next(A[r].x);
        d[5] = wave_next(A[r].y);
        d[6] = wave_next(A[r].z);
        d[7] = wave_next(A[r].w);
        uint4 nx;
        if (r + 1 < R) {
            nx = make_uint4((uint32_t)__builtin_amdgcn_readfirstlane((int)A[r + 1].x),
                            (uint32_t)__builtin_amdgcn_readfirstlane((int)A[r + 1].y),
                            (uint32_t)__builtin_amdgcn_readfirstlane((int)A[r + 1].z),
                            (uint32_t)__builtin_amdgcn_readfirstlane((int)A[r + 1].w));
        } else {
            nx = E;
        }
        if (lane == 63) {
            // the next batch's first record starts right after lane 63's: its aligned block is
            // lane 63's block + 16 exactly when lane 63's record crosses into it; otherwise bytes
            // 16..31 are never read
            d[4] = nx.x, d[5] = nx.y, d[6] = nx.z, d[7] = nx.w;
        }
        const uint32_t k = r * 64 + lane;
        const uint32_t Lk = k < ks ? L : L2;
        uint32_t e0, e1, e2, e3;
        extract16(d, o[r] & 15u, e0, e1, e2, e3);
        uint64_t id, val;
        rec_decode16(e0, e1, e2, e3, Lk, id, val);
        bad |= (rec_check16(e0, e1, W - (a0 + o[r])) != Lk) | (id != ib + k);
        const uint64_t row = k0 + k;
        if (row < cap) {
            st_col(&oid[row], id);
            st_col(&oval[row], val);
        } else {
            over = true;
        }
    }
    return bad;
}

#ifndef NXG_F64S_PAIR
#define NXG_F64S_PAIR 1  // 1: a lane decodes two consecutive records, one 16-byte store per column
#endif
// A whole wave in pairs: lane j of batch r takes records k = 2 (64 r + j) and k + 1 (rows k0 + k,
// even: one 16-byte aligned store per column). The two records lie in the 48 bytes from the
// aligned block of the first: blocks A and B are loaded, C is the next lane's A or B (DPP; its
// first record starts 24..32 bytes after ours), lane 63 loads its C itself.
template <int R>
NXG_DEV bool emit_full_pairs(const uint8_t* __restrict__ wire, uint64_t W, uint64_t p0, uint32_t L,
                             uint32_t ks, uint64_t k0, uint64_t i0, uint64_t* __restrict__ oid,
                             uint64_t* __restrict__ oval, uint64_t cap, uint32_t lane,
                             bool& over) {
    using namespace f64rec16;
    constexpr int RP = R / 2;
    const uint64_t a0 = p0 & ~15ull;
    const uint8_t* __restrict__ base = wire + a0;
    const uint32_t s0 = (uint32_t)(p0 & 15u);
    const uint32_t L2 = L + 1;
    auto off = [&](uint32_t k) -> uint32_t {
        return s0 + (k < ks ? k * L : ks * L + (k - ks) * L2);
    };
    uint4 A[RP], B[RP], Cq[RP];
    uint32_t oa[RP], ob[RP];
#pragma unroll
    for (int r = 0; r < RP; r++) {
        const uint32_t k = 2 * (r * 64 + lane);
        oa[r] = off(k);
        ob[r] = off(k + 1);
        const uint32_t ab = oa[r] & ~15u;
        A[r] = ld16s(base + ab);
        B[r] = ld16s(base + ab + 16);
        if (lane == 63) Cq[r] = ld16s(base + ab + 32);
    }
    bool bad = false;
    const uint64_t ib = i0 + k0;
#pragma unroll
    for (int r = 0; r < RP; r++) {
        const uint32_t k = 2 * (r * 64 + lane);
        const uint32_t ab = oa[r] & ~15u;
        const uint32_t nA[4] = {wave_next(A[r].x), wave_next(A[r].y), wave_next(A[r].z),
                                wave_next(A[r].w)};
        const uint32_t nB[4] = {wave_next(B[r].x), wave_next(B[r].y), wave_next(B[r].z),
                                wave_next(B[r].w)};
        const bool at32 = (off(k + 2) & ~15u) == ab + 32;
        uint32_t C[4];
        C[0] = at32 ? nA[0] : nB[0];
        C[1] = at32 ? nA[1] : nB[1];
        C[2] = at32 ? nA[2] : nB[2];
        C[3] = at32 ? nA[3] : nB[3];
        if (lane == 63) C[0] = Cq[r].x, C[1] = Cq[r].y, C[2] = Cq[r].z, C[3] = Cq[r].w;
        const uint32_t La = k < ks ? L : L2, Lb = k + 1 < ks ? L : L2;
        const uint32_t d[8] = {A[r].x, A[r].y, A[r].z, A[r].w, B[r].x, B[r].y, B[r].z, B[r].w};
        uint32_t e0, e1, e2, e3;
        extract16(d, oa[r] & 15u, e0, e1, e2, e3);
        uint64_t ida, va;
        rec_decode16(e0, e1, e2, e3, La, ida, va);
        bad |= (rec_check16(e0, e1, W - (a0 + oa[r])) != La) | (ida != ib + k);
        const uint32_t sb = ob[r] - ab;  // 12..31
        const bool up = sb >= 16;
        const uint32_t d2[8] = {up ? B[r].x : A[r].x, up ? B[r].y : A[r].y, up ? B[r].z : A[r].z,
                                up ? B[r].w : A[r].w, up ? C[0] : B[r].x, up ? C[1] : B[r].y,
                                up ? C[2] : B[r].z, up ? C[3] : B[r].w};
        extract16(d2, sb & 15u, e0, e1, e2, e3);
        uint64_t idb, vb;
        rec_decode16(e0, e1, e2, e3, Lb, idb, vb);
        bad |= (rec_check16(e0, e1, W - (a0 + ob[r])) != Lb) | (idb != ib + k + 1);
        const uint64_t row = k0 + k;
        if (row + 1 < cap) {
            const uint4 iv = make_uint4((uint32_t)ida, (uint32_t)(ida >> 32), (uint32_t)idb,
                                        (uint32_t)(idb >> 32));
            const uint4 vv = make_uint4((uint32_t)va, (uint32_t)(va >> 32), (uint32_t)vb,
                                        (uint32_t)(vb >> 32));
            if (NXG_F64S_NT & 1) {
                __builtin_nontemporal_store(*reinterpret_cast<const v4u*>(&iv),
                                            reinterpret_cast<v4u*>(oid + row));
                __builtin_nontemporal_store(*reinterpret_cast<const v4u*>(&vv),
                                            reinterpret_cast<v4u*>(oval + row));
            } else {
                *reinterpret_cast<uint4*>(oid + row) = iv;
                *reinterpret_cast<uint4*>(oval + row) = vv;
            }
        } else {
            if (row < cap) {
                oid[row] = ida;
                oval[row] = va;
            }
            over = true;
        }
    }
    return bad;
}

}  // namespace f64s

// One wave per WREC records; the grid covers the most records W bytes can hold (W / 12), and the
// waves past the frame's last record exit after the head read. Everything before the loads is
// wave-uniform (scalar registers): the head, the closed-form position of the wave's first record
// and the width change inside the wave.
template <int R>
__global__ __launch_bounds__(f64s::TPB) void nxg_f64s_kernel(const uint8_t* __restrict__ wire,
                                                             uint64_t W, uint64_t* __restrict__ oid,
                                                             uint64_t* __restrict__ oval,
                                                             uint64_t cap, uint32_t flags,
                                                             DevStatus* __restrict__ st,
                                                             DevStatus* zst) {
    using namespace f64s;
    using namespace f64rec16;
    constexpr uint32_t WREC = 64 * R;  // records per wave
    // another wave rejected the frame already (a plain read before any store: a scalar load)
    const uint32_t failed = st->fast_fail;
    zero_status(zst);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // the frame head: record 0 and its id (every wave; a scalar load, kept in scalar registers)
    uint4 h0;
    if (W >= 16) {
        h0 = *reinterpret_cast<const uint4*>(wire);
    } else {
        uint32_t v[4] = {0, 0, 0, 0};
        for (uint32_t k = 0; k < (uint32_t)W; k++) v[k >> 2] |= (uint32_t)wire[k] << (8 * (k & 3));
        h0 = make_uint4(v[0], v[1], v[2], v[3]);
    }
    h0.x = (uint32_t)__builtin_amdgcn_readfirstlane((int)h0.x);
    h0.y = (uint32_t)__builtin_amdgcn_readfirstlane((int)h0.y);
    h0.z = (uint32_t)__builtin_amdgcn_readfirstlane((int)h0.z);
    h0.w = (uint32_t)__builtin_amdgcn_readfirstlane((int)h0.w);
    const uint32_t hl = rec_check16(h0.x, h0.y, W);
    if (!hl) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            atomicOr(&st->irregular, 2u);  // not an f64 frame: the host goes on to the mixed path
            atomicOr(&st->fast_fail, 1u);
        }
        return;
    }
    uint64_t i0, v0;
    rec_decode16(h0.x, h0.y, h0.z, h0.w, hl, i0, v0);
    // Workgroups go to the 8 XCDs round-robin; a frame larger than the Infinity Cache streams from
    // HBM, and there each XCD takes runs of XRUN consecutive workgroups' records (XRUN x 1024
    // records, ~1 MB of wire): XCD x's k-th workgroup decodes run (k / XRUN) * 8 + x, at position
    // k % XRUN. A bijection on the whole groups of 8 runs; the grid's last partial group keeps its
    // indices. (No record count is needed: the waves past the frame's end exit.)
    uint64_t blk = blockIdx.x;
    if (flags & F_XCD) {
        const uint64_t full = (uint64_t)gridDim.x / (8 * XRUN) * (8 * XRUN);
        if (blk < full) {
            const uint64_t x = blk % 8, k = blk / 8;
            blk = ((k / XRUN) * 8 + x) * XRUN + k % XRUN;
        }
    }
    const uint64_t k0 = (blk * (TPB / 64) + w) * WREC;
    const uint64_t p0 = pos_of(i0, k0);
    if (p0 >= W || failed) return;
    const uint64_t id0 = i0 + k0;
    const uint32_t b = vl64(id0);
    const uint64_t nxt = 1ull << (7 * b);  // the next width change (ids < 2^35: b <= 5)
    const uint32_t L = 11u + b;
    const uint32_t ks = nxt - id0 < WREC ? (uint32_t)(nxt - id0) : WREC;
    const uint64_t pend = p0 + (uint64_t)ks * L + (uint64_t)(WREC - ks) * (L + 1);  // pos(k0 + WREC)
    bool over = false, bad = b > 5;
    if (!bad && pend + 48 <= W) {
        bad = NXG_F64S_PAIR ? emit_full_pairs<R>(wire, W, p0, L, ks, k0, i0, oid, oval, cap, lane, over)
                            : emit_full<R>(wire, W, p0, L, ks, k0, i0, oid, oval, cap, lane, over);
    } else if (!bad) {
        // near the frame's end: n = #{k < WREC : pos(k0 + k) < W} (pos increases by 12..16 per
        // record); the frame's last record must end exactly at W
        uint32_t n = WREC;
        if (pend > W) {
            uint32_t lo = 0, hi = WREC;  // pos(k0 + lo) < W <= pos(k0 + hi)
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) / 2;
                if (pos_of(i0, k0 + mid) < W) lo = mid;
                else hi = mid;
            }
            n = hi;
        }
        const uint64_t pn = pos_of(i0, k0 + n);
        if (pn == W && lane == 0) {  // this wave holds the frame's last record
            st->n_rows = k0 + n;
            st->path = 1;
            st->diag[1] = 1;  // decoded by the sequential-id kernel (diagnostics)
        }
        if (pn < W && n < WREC) bad = true;  // (cannot happen: pos(k0 + n) >= W by the search)
        else if (pn > W) bad = true;         // the frame does not end at a record boundary
        else bad = emit_edge(wire, W, p0, L, ks, n, k0, i0, oid, oval, cap, lane, over);
    }
    if (__any(bad) && lane == 0) {
        atomicOr(&st->irregular, 4u);  // ids do not count up by one: the length-run decoder
        atomicOr(&st->fast_fail, 1u);
    }
    if (__any(over) && lane == 0) atomicOr(&st->capacity, 1u);
}

uint64_t nxg_dec_f64s_groups(uint64_t W) {
    const uint64_t maxrec = W / 12 + 1;
    const uint64_t wrec = 64ull * (uint64_t)f64s::r_for(W);
    const uint64_t waves = (maxrec + wrec - 1) / wrec;
    return (waves + f64s::TPB / 64 - 1) / (f64s::TPB / 64);
}

// Decodes a whole frame of W bytes (W > 0) if its ids count up by one; else sets fast_fail with
// DevStatus.irregular bit 1 (not f64) or bit 2 (another f64 frame).
hipError_t nxg_launch_dec_f64s(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                               uint64_t cap, DevStatus* st, DevStatus* zst, hipStream_t s) {
    if (W == 0) return hipSuccess;
    const uint64_t ng = nxg_dec_f64s_groups(W);
    if (ng > 0x7fffffffull) return hipErrorInvalidValue;
    const uint32_t flags = NXG_F64S_XCD && W > f64s::kXcdMin ? f64s::F_XCD : 0u;
    if (f64s::r_for(W) == NXG_F64S_R)
        hipLaunchKernelGGL(nxg_f64s_kernel<NXG_F64S_R>, dim3((uint32_t)ng), dim3(f64s::TPB),
                           NXG_F64S_LDS, s, wire, W, oid, oval, cap, flags, st, zst);
    else
        hipLaunchKernelGGL(nxg_f64s_kernel<NXG_F64S_R_SMALL>, dim3((uint32_t)ng), dim3(f64s::TPB),
                           NXG_F64S_LDS, s, wire, W, oid, oval, cap, flags, st, zst);
    return hipGetLastError();
}
