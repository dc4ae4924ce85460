// nxg_encode_f64_seq.hip -- one-launch encode of (id u64[N], f64 bits u64[N]) to wire bytes when
// the ids count up by one, for gfx950.
//
// Replaces the handle_updates -> queue_send loop (netidx/src/publisher/server.rs:604-629,
// netidx/src/channel.rs:177-202) for the commonest publisher batch: every value of a publisher
// updated in publication order, so the ids come from the per-process counter
// (netidx-core/src/utils.rs:130-134) and count up by one. Each record is what len_wrapped_encode
// (pack.rs:527-535) + the derived enum encode (netidx-derive/src/lib.rs:289-381) + Value::encode
// (netidx-value/src/lib.rs:404-407) write:
//     varint(L) 04 varint(id) 09 f64be,    L = 11 + vl(id)
// and record k starts at the closed form f64rec16::seq_pos(i0, k) (the decoder's, nxg_decode_f64_seq.hip).
// So no length scan and no look-back: every wave knows where its records go.
//
//   - Every wave reads id[0] (= i0) and computes the frame's length T = seq_pos(i0, N) in scalar
//     registers (capacity, MAX_BATCH split: block 0).
//   - Wave g takes records [64 R g, 64 R (g + 1)); lane j its R consecutive records, loaded as
//     16-byte pairs and checked: id == i0 + k. Any other id makes the wave write nothing and
//     raise fast_fail (DevStatus.irregular bit 2); the host reruns the batch on the tiled encoder
//     (nxg_encode_f64.hip), which takes any ids, and skips this one for a while.
//   - A wave whose records all have one length L (no varint width change inside it: all but at
//     most four waves of a frame) builds each lane's R*L bytes in registers at compile-time
//     positions (a template per L), appends the first 16 bytes of the next lane's stream (DPP; the
//     wave's last lane builds the next wave's first records itself), shifts the stream to the
//     output's 16-byte phase (two select levels + v_alignbyte), and writes the aligned 16-byte
//     blocks that start inside the lane's bytes -- through the wave's LDS stage, so that the
//     global stores are 64 consecutive blocks per instruction. The bytes before the wave's first
//     aligned block are written by its lane 0 (the previous wave's last block holds them too).
//   - Other waves (a width change inside, the frame's last partial wave) write their records
//     byte by byte: rare, and the same bytes.
// With out == NULL (sizing) the kernel reads and checks the ids and reports T only.
#include "nxg_device.h"
#include "nxg_f64_rec16.h"

namespace f64es {
constexpr int TPB = 256;
#ifndef NXG_ENCS_R
#define NXG_ENCS_R 4  // records per lane
#endif
#ifndef NXG_ENCS_LDS
#define NXG_ENCS_LDS 1  // 1: blocks leave through the wave's LDS stage (coalesced stores)
#endif
#ifndef NXG_ENCS_NT
#define NXG_ENCS_NT 1  // nontemporal frame stores
#endif
constexpr int R = NXG_ENCS_R;
static_assert(R % 2 == 0 && R >= 4 && R <= 8, "records per lane");
constexpr uint32_t WREC = 64 * R;  // records per wave
constexpr uint32_t SBLK = 64 * R + 3;  // stage blocks per wave (<= 16 bytes per record + edges)
constexpr uint64_t kXcdMin = 256ull << 20;  // frames past the Infinity Cache
#ifndef NXG_ENCS_XRUN
#define NXG_ENCS_XRUN 64
#endif
constexpr uint64_t XRUN = NXG_ENCS_XRUN;
constexpr uint32_t F_XCD = 1;

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// L 04 varint(id) 09 as the low VL + 3 bytes of a 64-bit value (VL = vl(id), 1..5)
template <int VL>
NXG_DEV uint64_t head64(uint64_t id) {
    uint64_t v = (uint64_t)(11 + VL) | (4ull << 8);
#pragma unroll
    for (int m = 0; m < VL; m++) {
        uint64_t b = (id >> (7 * m)) & 0x7f;
        if (m < VL - 1) b |= 0x80;
        v |= b << (16 + 8 * m);
    }
    return v | (9ull << (16 + 8 * VL));
}

// bytes [O, O + NB) of the little-endian dword stream E = the low NB bytes of v (NB <= 8; v is
// zero above them). O and NB are constants after unrolling, so E stays in registers.
template <int ND>
NXG_DEV void put_bytes(uint32_t (&E)[ND], int O, int NB, uint64_t v) {
    const int d = O >> 2, c = O & 3;
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    if (c == 0) {
        E[d] |= lo;
        if (NB > 4) E[d + 1] |= hi;
    } else {
        E[d] |= lo << (8 * c);
        if (NB + c > 4) E[d + 1] |= (lo >> (32 - 8 * c)) | (hi << (8 * c));
        if (NB + c > 8) E[d + 2] |= hi >> (32 - 8 * c);
    }
}

// one record (any id < 2^35) as 16 record-aligned bytes, zero past its length
NXG_DEV uint32_t rec16_dyn(uint64_t id, uint64_t val, uint32_t (&d)[4]) {
    const uint32_t vl = vl64(id), L = 11 + vl;
    uint64_t h = (uint64_t)L | (4ull << 8);
#pragma unroll
    for (uint32_t m = 0; m < 5; m++) {
        uint64_t b = (id >> (7 * m)) & 0x7f;
        if (m + 1 < vl) b |= 0x80;
        if (m < vl) h |= b << (16 + 8 * m);
    }
    h |= 9ull << (16 + 8 * vl);
    const uint64_t be = __builtin_bswap64(val);
    const uint32_t sh = 8 * (3 + vl);  // 32..64
    const uint64_t lo = h | (sh < 64 ? be << sh : 0ull);
    const uint64_t hi = sh < 64 ? be >> (64 - sh) : be;
    d[0] = (uint32_t)lo;
    d[1] = (uint32_t)(lo >> 32);
    d[2] = (uint32_t)hi;
    d[3] = (uint32_t)(hi >> 32);
    return L;
}

// the slow path: one record's bytes straight to the frame
NXG_DEV void put_rec_global(uint8_t* out, uint64_t o, uint64_t id, uint64_t val) {
    uint32_t d[4];
    const uint32_t L = rec16_dyn(id, val, d);
#pragma unroll
    for (uint32_t k = 0; k < 16; k++)
        if (k < L) out[o + k] = (uint8_t)(d[k >> 2] >> (8 * (k & 3)));
}

NXG_DEV void st_block(uint8_t* p, v4u x) {
    if (NXG_ENCS_NT) __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(p));
    else *reinterpret_cast<v4u*>(p) = x;
}
// the frame's last block: only the bytes before T
NXG_DEV void st_block_tail(uint8_t* out, uint64_t pos, uint64_t T, v4u x) {
    if (pos + 16 <= T) {
        st_block(out + pos, x);
        return;
    }
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int k = 0; k < 16; k++)
        if (pos + k < T) out[pos + k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
}

// A wave of WREC records of one length L = 11 + VL. Lane j's records start at byte
// p0 + j R L of the frame; `ph` is the output pointer's 16-byte phase.
template <int VL>
NXG_DEV void emit_fast(const uint64_t (&ids)[R], const uint64_t (&vals)[R], uint8_t* __restrict__ out,
                       uint64_t T, uint64_t p0, uint32_t ph, uint64_t k0, uint64_t n, uint64_t i0,
                       const uint64_t* __restrict__ val, v4u* __restrict__ stg, uint32_t lane) {
    constexpr int L = 11 + VL;
    constexpr int LB = R * L;              // the lane's bytes
    constexpr int MB = (LB + 15) / 16;     // at most this many blocks start inside them
    constexpr int NE = 4 * MB + 4;         // stream dwords: the lane's bytes + 16 of the next
    uint32_t E[NE];
#pragma unroll
    for (int d = 0; d < NE; d++) E[d] = 0;
#pragma unroll
    for (int r = 0; r < R; r++) {
        put_bytes(E, r * L, VL + 3, head64<VL>(ids[r]));
        put_bytes(E, r * L + VL + 3, 8, __builtin_bswap64(vals[r]));
    }
    // the next lane's first 16 bytes (lane 63: the next wave's first records, if any)
    uint32_t N[4];
#pragma unroll
    for (int i = 0; i < 4; i++) N[i] = wave_next(E[i]);
    if (lane == 63) {
        N[0] = N[1] = N[2] = N[3] = 0;
        const uint64_t kn = k0 + WREC;
        if (kn < n) {
            uint32_t a[4], b[4] = {0, 0, 0, 0};
            const uint32_t L1 = rec16_dyn(i0 + kn, val[kn], a);
            if (kn + 1 < n) rec16_dyn(i0 + kn + 1, val[kn + 1], b);
            N[0] = a[0], N[1] = a[1], N[2] = a[2], N[3] = a[3];
            if (L1 < 16) N[3] |= b[0] << (8 * (L1 - 12));
        }
    }
    {
        constexpr int D0 = LB / 4, c = LB % 4;
        if (c == 0) {
#pragma unroll
            for (int i = 0; i < 4; i++) E[D0 + i] |= N[i];
        } else {
            E[D0] |= N[0] << (8 * c);
#pragma unroll
            for (int i = 1; i < 4; i++) E[D0 + i] |= (N[i - 1] >> (32 - 8 * c)) | (N[i] << (8 * c));
            E[D0 + 4] |= N[3] >> (32 - 8 * c);
        }
    }
    // the lane's first aligned block starts delta bytes into its stream
    const uint64_t vj = (uint64_t)ph + p0 + (uint64_t)lane * LB;  // virtual: 16-aligned = aligned
    const uint32_t delta = (16u - (uint32_t)(vj & 15u)) & 15u;
    const uint32_t q = delta >> 2, s = delta & 3u;
    const uint32_t m1 = 0u - (q & 1u), m2 = 0u - ((q >> 1) & 1u);
    uint32_t A1[NE - 1];
#pragma unroll
    for (int d = 0; d < NE - 1; d++) A1[d] = E[d] ^ ((E[d] ^ E[d + 1]) & m1);
    uint32_t A2[NE - 3];
#pragma unroll
    for (int d = 0; d < NE - 3; d++) A2[d] = A1[d] ^ ((A1[d] ^ A1[d + 2]) & m2);
    const uint64_t vw = (uint64_t)ph + p0;       // the wave's first byte (virtual)
    const uint64_t xw = vw & ~15ull;             // its aligned base
    if (NXG_ENCS_LDS) {
        const uint32_t b0 = (uint32_t)((vj + delta - xw) >> 4);
#pragma unroll
        for (int m = 0; m < MB; m++) {
            if (delta + 16 * m < (uint32_t)LB) {
                v4u x;
                x.x = alignbyte(A2[4 * m + 1], A2[4 * m], s);
                x.y = alignbyte(A2[4 * m + 2], A2[4 * m + 1], s);
                x.z = alignbyte(A2[4 * m + 3], A2[4 * m + 2], s);
                x.w = alignbyte(A2[4 * m + 4], A2[4 * m + 3], s);
                stg[b0 + m] = x;
            }
        }
        wave_lds_order();
        const uint64_t vend = vw + (uint64_t)WREC * L;  // the wave's end (virtual)
        const uint32_t first = (vw & 15u) ? 1u : 0u;
        const uint32_t last = (uint32_t)((((vend - 1) & ~15ull) - xw) >> 4);  // inclusive
        for (uint32_t b = first + lane; b <= last; b += 64)
            st_block_tail(out, xw + 16ull * b - ph, T, stg[b]);
    } else {
#pragma unroll
        for (int m = 0; m < MB; m++) {
            if (delta + 16 * m < (uint32_t)LB) {
                v4u x;
                x.x = alignbyte(A2[4 * m + 1], A2[4 * m], s);
                x.y = alignbyte(A2[4 * m + 2], A2[4 * m + 1], s);
                x.z = alignbyte(A2[4 * m + 3], A2[4 * m + 2], s);
                x.w = alignbyte(A2[4 * m + 4], A2[4 * m + 3], s);
                st_block_tail(out, vj + delta + 16ull * m - ph, T, x);
            }
        }
    }
    // the wave's head: the bytes before its first aligned block
    if (lane == 0 && delta) {
#pragma unroll
        for (int k = 0; k < 15; k++)
            if ((uint32_t)k < delta) out[p0 + k] = (uint8_t)(E[k >> 2] >> (8 * (k & 3)));
    }
}

}  // namespace f64es

__global__ __launch_bounds__(f64es::TPB) void nxg_enc_f64s_kernel(
    const uint64_t* __restrict__ id, const uint64_t* __restrict__ val, uint64_t n,
    uint8_t* __restrict__ out, uint64_t cap, uint32_t flags, DevStatus* __restrict__ st,
    DevStatus* zst) {
    using namespace f64es;
    zero_status(zst);
    __shared__ v4u stage[NXG_ENCS_LDS ? TPB / 64 : 1][NXG_ENCS_LDS ? SBLK : 1];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // the frame, in scalar registers: i0, its length T
    const uint64_t i0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)id[0]) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(id[0] >> 32)) << 32);
    const bool lead = blockIdx.x == 0 && threadIdx.x == 0;
    if (i0 >= (1ull << 35) || n > (1ull << 35) - i0) {  // ids past 35 bits: the tiled encoder
        if (lead) {
            atomicOr(&st->irregular, 4u);
            atomicOr(&st->fast_fail, 1u);
        }
        return;
    }
    const uint64_t T = f64rec16::seq_pos(i0, n);
    if (lead) {
        st->total_bytes = T;
        st->n_rows = n;
        if (T > kMaxBatch) {  // the message holding byte MAX_BATCH (channel.rs:187-191)
            uint64_t lo = 0, hi = n;  // seq_pos(lo) <= kMaxBatch < seq_pos(hi)
            while (hi - lo > 1) {
                const uint64_t mid = (lo + hi) / 2;
                if (f64rec16::seq_pos(i0, mid) <= kMaxBatch) lo = mid;
                else hi = mid;
            }
            st->split_start = f64rec16::seq_pos(i0, lo) + 1;
        }
    }
    // columns too large for `out`: nothing is written, but the ids are still checked, so that a
    // batch that is not a run of consecutive ids (whose real length T does not give) goes to the
    // tiled encoder, which sizes it exactly (fast_fail comes before capacity on the host)
    const bool over = out && T > cap;
    if (over && lead) atomicOr(&st->capacity, 1u);
    uint64_t blk = blockIdx.x;
    if (flags & F_XCD) {  // each XCD streams runs of XRUN consecutive workgroups' records
        const uint64_t full = (uint64_t)gridDim.x / (8 * XRUN) * (8 * XRUN);
        if (blk < full) {
            const uint64_t x = blk % 8, k = blk / 8;
            blk = ((k / XRUN) * 8 + x) * XRUN + k % XRUN;
        }
    }
    const uint64_t k0 = (blk * (TPB / 64) + w) * WREC;
    if (k0 >= n) return;
    const uint32_t nrec = n - k0 < WREC ? (uint32_t)(n - k0) : WREC;
    const uint64_t kl = k0 + (uint64_t)lane * R;  // the lane's first record
    uint64_t ids[R], vals[R];
    bool bad = false;
    if (nrec == WREC) {
#pragma unroll
        for (int r = 0; r < R; r += 2) {
            const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(id + kl + r);
            const ulonglong2 c = *reinterpret_cast<const ulonglong2*>(val + kl + r);
            ids[r] = a.x, ids[r + 1] = a.y;
            vals[r] = c.x, vals[r + 1] = c.y;
        }
    } else {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const bool in = kl + r < n;
            ids[r] = in ? id[kl + r] : i0 + kl + r;
            vals[r] = in ? val[kl + r] : 0;
        }
    }
#pragma unroll
    for (int r = 0; r < R; r++) bad |= ids[r] != i0 + kl + r;
    if (__any(bad)) {  // not a run of consecutive ids: write nothing, the tiled encoder reruns it
        if (lane == 0) {
            atomicOr(&st->irregular, 4u);
            atomicOr(&st->fast_fail, 1u);
        }
        return;
    }
    if (!out || over) return;
    const uint64_t p0 = f64rec16::seq_pos(i0, k0);
    const uint32_t vl = vl64(i0 + k0);
    const uint32_t ph = (uint32_t)((uintptr_t)out & 15u);
    v4u* stg = stage[NXG_ENCS_LDS ? w : 0];
    if (nrec == WREC && vl64(i0 + k0 + WREC - 1) == vl) {
        switch (vl) {
            case 1: emit_fast<1>(ids, vals, out, T, p0, ph, k0, n, i0, val, stg, lane); break;
            case 2: emit_fast<2>(ids, vals, out, T, p0, ph, k0, n, i0, val, stg, lane); break;
            case 3: emit_fast<3>(ids, vals, out, T, p0, ph, k0, n, i0, val, stg, lane); break;
            case 4: emit_fast<4>(ids, vals, out, T, p0, ph, k0, n, i0, val, stg, lane); break;
            default: emit_fast<5>(ids, vals, out, T, p0, ph, k0, n, i0, val, stg, lane); break;
        }
    } else {
        // a width change inside the wave, or the frame's last partial wave: byte stores
        uint64_t o = f64rec16::seq_pos(i0, kl);
#pragma unroll
        for (int r = 0; r < R; r++)
            if (kl + r < n) {
                put_rec_global(out, o, ids[r], vals[r]);
                o += 11 + vl64(ids[r]);
            }
    }
}

uint64_t nxg_enc_f64s_groups(uint64_t n) {
    const uint64_t waves = (n + f64es::WREC - 1) / f64es::WREC;
    return (waves + f64es::TPB / 64 - 1) / (f64es::TPB / 64);
}

hipError_t nxg_launch_enc_f64s(const uint64_t* id, const uint64_t* val, uint64_t n, uint8_t* out,
                               uint64_t cap, DevStatus* st, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t ng = nxg_enc_f64s_groups(n);
    if (ng > 0x7fffffffull) return hipErrorInvalidValue;
    // (the frame's bytes: 12..16 per record; the remap pays past the Infinity Cache)
    const uint32_t flags = 13 * n > f64es::kXcdMin ? f64es::F_XCD : 0u;
    hipLaunchKernelGGL(nxg_enc_f64s_kernel, dim3((uint32_t)ng), dim3(f64es::TPB), 0, s, id, val, n,
                       out, cap, flags, st, nxg_take_zero_slot());
    return hipGetLastError();
}
