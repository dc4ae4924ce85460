// nxg_share.hip -- one share of a decoded frame's rows (nxg_decode_share): rows [r0, r1) of a
// whole-frame decode, with the children of their values and the control spans between them,
// copied into a rank's own columns and re-based (child indices from 0, ctl_row from 0).
//
// This is nxg_decode_sharded's fallback for frames the byte-range decoders decline (Maps, nested
// containers, rare control messages, long messages, content errors): every rank decodes the frame
// whole -- the frame is on every rank already -- and keeps its share of the rows, as one subscriber
// decodes any frame as one batch (netidx/src/channel.rs:504-521) and hands the updates on in
// order (netidx/src/subscriber/connection.rs:546-567).
//
// Children are allocated depth-first in row order (include/nxg_codec.h), so the subtrees of rows
// [r0, r1) are one contiguous run of child slots [c0, c1): c0 is the first child slot of the first
// container row at or after r0 (child indices grow with the row), c1 that of the first container
// row at or after r1 (or the frame's child count). Control spans are ordered by ctl_row.
#include "nxg_device.h"
#include "nxg_internal.h"

namespace {

constexpr int TPB = 256;

// Array, Map, Error(Value): `fixed` is the first child slot (include/nxg_codec.h)
NXG_DEV bool container(uint32_t t) { return t == 19 || t == 21 || t == 22; }

NXG_DEV uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o = __shfl_xor(v, d, 64);
        v = o < v ? o : v;
    }
    return v;
}

// b[0] = first child slot of a container row >= r0, b[1] = the same for r1, b[2] = first control
// span with ctl_row >= r0, b[3] = the same for r1 (each ~0 when there is none; the host sets
// ~0 before the launch). One atomic per wave and bound.
__global__ __launch_bounds__(TPB) void nxg_share_bounds_kernel(ColsDesc src, uint64_t r0,
                                                               uint64_t r1,
                                                               unsigned long long* b) {
    uint64_t m[4] = {~0ull, ~0ull, ~0ull, ~0ull};
    const uint64_t n = src.n_rows > src.n_ctl ? src.n_rows : src.n_ctl;
    const uint64_t stride = (uint64_t)gridDim.x * TPB;
#pragma unroll 1
    for (uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += stride) {
        if (src.tag && i < src.n_rows && i >= r0 && container(src.tag[i])) {
            const uint64_t f = src.fixed[i];
            m[0] = f < m[0] ? f : m[0];
            if (i >= r1) m[1] = f < m[1] ? f : m[1];
        }
        if (i < src.n_ctl) {
            const uint64_t row = src.ctl_row[i];
            if (row >= r0) m[2] = i < m[2] ? i : m[2];
            if (row >= r1) m[3] = i < m[3] ? i : m[3];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t w = wave_min_u64(m[k]);
        if ((threadIdx.x & 63) == 0 && w != ~0ull) atomicMin(&b[k], (unsigned long long)w);
    }
}

// rows [r0, r0 + nr), children [c0, c0 + nc), control spans [k0, k0 + nk) of src into dst from 0
// (and the Heartbeats among those control spans into *hb)
__global__ __launch_bounds__(TPB) void nxg_share_copy_kernel(ColsDesc src, ColsDesc dst,
                                                             uint64_t r0, uint64_t nr,
                                                             uint64_t c0, uint64_t nc,
                                                             uint64_t k0, uint64_t nk,
                                                             unsigned long long* hb) {
    const uint64_t n = nr > nc ? (nr > nk ? nr : nk) : (nc > nk ? nc : nk);
    const uint64_t stride = (uint64_t)gridDim.x * TPB;
    uint32_t beats = 0;
#pragma unroll 1
    for (uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x; i < n; i += stride) {
        if (i < nr) {
            const uint64_t j = r0 + i;
            uint64_t f = src.fixed[j];
            dst.id[i] = src.id[j];
            if (src.tag && dst.tag) {
                const uint32_t t = src.tag[j];
                if (container(t)) f -= c0;
                dst.tag[i] = (uint8_t)t;
                dst.aux[i] = src.aux[j];
            }
            dst.fixed[i] = f;
        }
        if (i < nc) {
            const uint64_t j = c0 + i;
            const uint32_t t = src.ctag[j];
            const uint64_t f = src.cfixed[j];
            dst.ctag[i] = (uint8_t)t;
            dst.cfixed[i] = container(t) ? f - c0 : f;
            dst.caux[i] = src.caux[j];
        }
        if (i < nk) {
            const uint64_t j = k0 + i;
            dst.ctl_row[i] = src.ctl_row[j] - r0;
            dst.ctl_off[i] = src.ctl_off[j];
            dst.ctl_len[i] = src.ctl_len[j];
            const uint8_t v = src.ctl_variant[j];
            dst.ctl_variant[i] = v;
            beats += v == 5;  // From::Heartbeat
        }
    }
    const uint32_t w = wave_sum<uint32_t>(beats);
    if ((threadIdx.x & 63) == 0 && w) atomicAdd(hb, (unsigned long long)w);
}

int grid_for(uint64_t n) {
    const uint64_t g = (n + TPB - 1) / TPB;
    return (int)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

}  // namespace

hipError_t nxg_launch_share_bounds(const ColsDesc& src, uint64_t r0, uint64_t r1, uint64_t* b,
                                   hipStream_t s) {
    hipError_t e = hipMemsetAsync(b, 0xff, 4 * sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
    const uint64_t n = src.n_rows > src.n_ctl ? src.n_rows : src.n_ctl;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(nxg_share_bounds_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, src, r0, r1,
                       reinterpret_cast<unsigned long long*>(b));
    return hipGetLastError();
}

hipError_t nxg_launch_share_copy(const ColsDesc& src, const ColsDesc& dst, uint64_t r0,
                                 uint64_t nr, uint64_t c0, uint64_t nc, uint64_t k0, uint64_t nk,
                                 uint64_t* hb, hipStream_t s) {
    hipError_t e = hipMemsetAsync(hb, 0, sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
    const uint64_t n = nr > nc ? (nr > nk ? nr : nk) : (nc > nk ? nc : nk);
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(nxg_share_copy_kernel, dim3(grid_for(n)), dim3(TPB), 0, s, src, dst, r0, nr,
                       c0, nc, k0, nk, reinterpret_cast<unsigned long long*>(hb));
    return hipGetLastError();
}
