// Experiment (probe only, not in the library): // nxg_decode_f64_os.hip -- one-shot homogeneous-f64 decode for gfx950 (record format and merge
// points: nxg_f64_rec.h). Same contract as nxg_decode_f64_1p.hip: replaces the
// receive_batch_fn loop (netidx/src/channel.rs:504-521) for frames in which every message is
// From::Update(Id, F64); anything else raises fast_fail and the host reruns the frame on the
// general decoder.
//
// One workgroup per super-tile s (grid = super-tiles, dispatched in blockIdx order): wave w
// decodes tile 4s + w (tiles start 4032 bytes apart) into its LDS slot, the four counts meet at
// one barrier, wave 0 finds the super-tile's first record index by a decoupled look-back over
// the super-tiles' epoch-tagged counts (lookback_prefix, as the encoders), and every wave writes
// its records to the id / value columns. No scanner and no persistent waves: the workgroup
// holds one tile per wave and retires, so the waves in flight always cover a compact window of
// the frame in dispatch order, and a slow tile holds up only the look-backs that reach it.
#include "../netidx_amd/csrc/nxg_f64_rec.h"

namespace {

#ifndef NXG_OS_NT
#define NXG_OS_NT 0  // nontemporal column stores
#endif
constexpr int TPBO = 256;
constexpr int WAVESO = TPBO / 64;
constexpr int MAXRO = f64dec::STRIDE / 12 + 1;  // records per tile (>= 12 bytes each): 337
constexpr int MAXLO = 6;  // records a lane owns: its span is < 64 + 15 bytes, >= 12 B each
constexpr uint32_t SLOTO = f64dec::IMG + f64dec::HALO;  // image, then its decoded records
constexpr uint32_t VALOFFO = (MAXRO * 4 + 7) & ~7u;     // decoded: u32 ids, then u64 values
static_assert(VALOFFO + MAXRO * 8 <= SLOTO, "decoded records fit the image they replace");

// Records of tile t (LDS image `img`) decoded into the same slot: u32 ids at 0, u64 values at
// VALOFFO, in record order. Returns false (wave-uniform) if the tile is not provably
// homogeneous-f64; `ntile` = its record count.
NXG_DEV bool os_tile_decode(uint8_t* img, uint64_t t, uint64_t W, uint32_t lane,
                            uint32_t& ntile) {
    const uint32_t xa = chunk_merge(img, t, W, lane);
    const uint32_t xb = wave_next(xa);
    const bool owner = lane != 63;  // lane 63's merge point is the next tile's first
    bool bad = (xa == FAIL) | (owner & ((xb == FAIL) | (xa > xb)));
    const uint64_t t0 = t * f64dec::STRIDE;
    // the chain of record starts reads one length byte per step; the records are then loaded
    // together (independent reads) and each is fully checked (its length must be the byte the
    // chain stepped by)
    uint32_t ps[MAXLO];
    uint32_t pos = xa, n = 0;
    const bool walk = owner && !bad;
#pragma unroll
    for (int q = 0; q < MAXLO; q++) {
        ps[q] = walk && pos < xb ? pos : 0u;
        if (walk && pos < xb) {
            const uint32_t Lb = img[pos];
            bad |= Lb - 12u > 3u;
            pos += Lb - 12u > 3u ? 12u : Lb;
            n++;
        }
    }
    bad |= owner && pos != xb;
    uint32_t rid[MAXLO];
    uint64_t rval[MAXLO];
    const uint32_t remt = W - t0 < 0xffffffffull ? (uint32_t)(W - t0) : 0xffffffffu;
#pragma unroll
    for (int q = 0; q < MAXLO; q++) {
        uint32_t e0, e1, e2, e3;
        load16(img, ps[q], e0, e1, e2, e3);
        const uint32_t Lr = rec_check32(e0, e1, remt - ps[q]);
        bad |= (uint32_t)q < n && Lr == 0;
        uint64_t id, val;
        rec_decode(e0, e1, e2, e3, Lr ? Lr : 12u, id, val);
        rid[q] = (uint32_t)id;  // f64 records carry ids < 2^28
        rval[q] = val;
    }
    if (__any(bad)) return false;
    const uint32_t inc = wave_incl_scan(n);
    ntile = wave_last(inc);
    wave_lds_order();  // every lane has read its records before the image is overwritten
    uint32_t* did = reinterpret_cast<uint32_t*>(img);
    uint64_t* dval = reinterpret_cast<uint64_t*>(img + VALOFFO);
    const uint32_t i0 = inc - n;
#pragma unroll
    for (int q = 0; q < MAXLO; q++) {
        if ((uint32_t)q < n) {
            did[i0 + q] = rid[q];
            dval[i0 + q] = rval[q];
        }
    }
    return true;
}

}  // namespace

__global__ __launch_bounds__(TPBO) void nxg_f64_os_kernel(
    const uint8_t* __restrict__ wire, uint64_t W, uint64_t nt, uint64_t* __restrict__ oid,
    uint64_t* __restrict__ oval, uint64_t cap, uint64_t* tstat, uint32_t epoch,
    DevStatus* __restrict__ st, DevStatus* zst) {
    zero_status(zst);
    __shared__ __attribute__((aligned(16))) uint8_t slot[WAVESO][SLOTO];
    __shared__ uint32_t wgc[WAVESO];
    __shared__ uint64_t sh_base;
    __shared__ uint32_t sh_abort;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t s = blockIdx.x;  // super-tile
    const uint64_t ns = (nt + WAVESO - 1) / WAVESO;
    const uint64_t t = s * WAVESO + w;
    const bool has = t < nt;
    const uint64_t nfull = W >= f64dec::IMG + f64dec::HALO
                               ? (W - f64dec::IMG - f64dec::HALO) / f64dec::STRIDE + 1
                               : 0;
    uint8_t* img = slot[w];
    uint32_t ntile = 0;
    bool bad = false;
    if (has) {
        TileRegs R;
        if (t < nfull) tile_load_full<false>(R, wire, t * f64dec::STRIDE, lane, nullptr);
        else tile_load(R, wire, t * f64dec::STRIDE, W, lane, nullptr);
        tile_store(img, R, lane);
        wave_lds_order();
        bad = !os_tile_decode(img, t, W, lane, ntile);
    }
    if (lane == 0) wgc[w] = bad ? 0x80000000u : ntile;
    if (threadIdx.x == 0) sh_abort = 0;
    __syncthreads();
    uint32_t sum = 0, off = 0, anybad = 0;
#pragma unroll
    for (int i = 0; i < WAVESO; i++) {
        const uint32_t c = wgc[i];
        anybad |= c;
        off += (uint32_t)i < w ? c : 0u;
        sum += c;
    }
    if (anybad & 0x80000000u) {  // the whole workgroup
        if (threadIdx.x == 0) atomicOr(&st->fast_fail, 1u);
        return;
    }
    if (w == 0) {
        uint64_t base = 0;
        if (s == 0) {
            if (lane == 0) st_agent(&tstat[0], lb_word(kFlagInc, epoch, sum));
        } else {
            if (lane == 0) st_agent(&tstat[s], lb_word(kFlagAgg, epoch, sum));
            bool give_up;
            base = lookback_prefix<1>(tstat, (uint32_t)s, epoch, &st->fast_fail, give_up);
            if (give_up) {
                if (lane == 0) {
                    if (!ld_agent32(&st->fast_fail)) atomicOr(&st->timeout, 1u);
                    atomicOr(&st->fast_fail, 1u);
                    sh_abort = 1;
                }
            } else if (lane == 0) {
                st_agent(&tstat[s], lb_word(kFlagInc, epoch, base + sum));
            }
        }
        if (lane == 0) sh_base = base;
    }
    __syncthreads();
    if (sh_abort) return;
    const uint64_t base = sh_base + off;
    if (s == ns - 1 && threadIdx.x == 0) {
        st->n_rows = sh_base + sum;
        st->path = 1;
    }
    const uint32_t* sid = reinterpret_cast<const uint32_t*>(img);
    const uint64_t* sval = reinterpret_cast<const uint64_t*>(img + VALOFFO);
    uint32_t lim = ntile;
    if (base + ntile > cap) {
        lim = base < cap ? (uint32_t)(cap - base) : 0u;
        if (lane == 0) atomicOr(&st->capacity, 1u);
    }
    for (uint32_t i = lane; i < lim; i += 64) {
        if (NXG_OS_NT) {
            __builtin_nontemporal_store((uint64_t)sid[i], &oid[base + i]);
            __builtin_nontemporal_store(sval[i], &oval[base + i]);
        } else {
            oid[base + i] = sid[i];  // widened to the u64 column
            oval[base + i] = sval[i];
        }
    }
}

uint64_t nxg_dec_f64_os_blocks(uint64_t W) {
    const uint64_t nt = (W + f64dec::STRIDE - 1) / f64dec::STRIDE;
    return (nt + WAVESO - 1) / WAVESO;
}

hipError_t nxg_launch_dec_f64_os(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                                 uint64_t cap, uint64_t* tstat, uint32_t epoch, DevStatus* st,
                                 hipStream_t s) {
    const uint64_t nt = (W + f64dec::STRIDE - 1) / f64dec::STRIDE;
    const uint64_t nb = (nt + WAVESO - 1) / WAVESO;
    if (nb == 0) return hipSuccess;
    if (nb > 0xffffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(nxg_f64_os_kernel, dim3((uint32_t)nb), dim3(TPBO), 0, s, wire, W, nt, oid,
                       oval, cap, tstat, epoch, st, nxg_take_zero_slot());
    return hipGetLastError();
}
