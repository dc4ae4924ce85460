// probe_f64.hip -- standalone timing probe for the f64 decode (diagnostics, not product).
// Builds an all-f64 frame on the host, then times with HIP events:
//   dec2p     the two-pass decode (count + emit); outputs are checked on the host
//   dec1p*    the single-pass decode (nxg_decode_f64_1p.hip) and its ablations (no wait for the
//             scanner's prefixes, no column stores), with per-phase cycle counters
//   stream    a plain kernel reading W bytes and writing 16N bytes (practical HBM ceiling)
//   d2d       hipMemcpyDeviceToDevice of the frame
// Usage: probe_f64 [records] [reps]
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "../netidx_amd/csrc/nxg_f64_rec.h"  // once, at global scope

namespace prod {
#include "../netidx_amd/csrc/nxg_decode_f64.hip"
}
namespace p1 {
#define NXG_1P_PROBE
#include "../netidx_amd/csrc/nxg_decode_f64_1p.hip"
#undef NXG_1P_PROBE
}
#undef P1_FLAGS
#undef P1_STAMP
namespace p1n {  // the product build (no stamps)
#include "../netidx_amd/csrc/nxg_decode_f64_1p.hip"
}
#define NXG_1P_LAG 2
namespace p1l3 {  // LAG 2: three LDS slots per wave (three 4-wave workgroups per CU by LDS)
#include "../netidx_amd/csrc/nxg_decode_f64_1p.hip"
}
#undef NXG_1P_LAG
namespace pos {  // one-shot decoder
#include "exp_f64_oneshot.hip"
}
#define NXG_OS_NT 1
namespace posnt {  // one-shot decoder, nontemporal column stores
#include "exp_f64_oneshot.hip"
}
#undef NXG_OS_NT
thread_local DevStatus* nxg_zero_slot = nullptr;
thread_local bool nxg_zero_used = false;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void stream_kernel(const uint4* __restrict__ in, uint64_t nin, uint4* __restrict__ out,
                              uint64_t nout) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nout; i += stride) {
        uint4 v = i < nin ? in[i] : make_uint4(0, 0, 0, 0);
        out[i] = v;
    }
}

// Memory-pattern twins of the two passes (no parsing): same persistent grid and runs, the same
// 5 x 16-byte loads per lane per tile; emit_mem also writes ~TILE/14.8 records per tile as two
// 8-byte column stores per lane.
__global__ __launch_bounds__(256) void count_mem_kernel(const uint8_t* __restrict__ wire,
                                                        uint64_t nt, uint32_t* sink) {
    const uint32_t lane = threadIdx.x & 63, R = gridDim.x * 4;
    const uint32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t acc = 0;
    for (uint64_t t = nt * r / R; t < nt * (r + 1) / R; t++) {
        const uint4* p = reinterpret_cast<const uint4*>(wire + t * 4096);
        uint4 a = p[lane], b = p[64 + lane], c = p[128 + lane], d = p[192 + lane];
        acc += a.x ^ b.y ^ c.z ^ d.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(256) void emit_mem_kernel(const uint8_t* __restrict__ wire,
                                                       uint64_t nt, uint64_t* __restrict__ oid,
                                                       uint64_t* __restrict__ oval, uint64_t N) {
    const uint32_t lane = threadIdx.x & 63, R = gridDim.x * 4;
    const uint32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t b = nt * r / R, e = nt * (r + 1) / R;
    uint64_t base = N * b / nt;
    for (uint64_t t = b; t < e; t++) {
        const uint4* p = reinterpret_cast<const uint4*>(wire + t * 4096);
        uint4 a = p[lane], bb = p[64 + lane], c = p[128 + lane], d = p[192 + lane];
        const uint64_t next = N * (t + 1) / nt;
        const uint32_t n = (uint32_t)(next - base);
        for (uint32_t i = lane; i < n; i += 64) {
            oid[base + i] = a.x + i;
            oval[base + i] = bb.y ^ c.z ^ d.w;
        }
        base = next;
    }
}

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    const uint64_t N = argc > 1 ? strtoull(argv[1], 0, 0) : 10000000ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    std::vector<uint8_t> w;
    std::vector<uint64_t> vals(N);
    w.reserve(N * 15);
    uint64_t seed = 7;
    for (uint64_t i = 0; i < N; i++) {
        uint8_t idb[10];
        int nb = 0;
        uint64_t v = i;
        while (v >= 0x80) { idb[nb++] = (uint8_t)(v | 0x80); v >>= 7; }
        idb[nb++] = (uint8_t)v;
        w.push_back((uint8_t)(11 + nb));
        w.push_back(4);
        for (int k = 0; k < nb; k++) w.push_back(idb[k]);
        w.push_back(9);
        const uint64_t f = vals[i] = splitmix(seed);
        for (int k = 7; k >= 0; k--) w.push_back((uint8_t)(f >> (8 * k)));
    }
    const uint64_t W = w.size();
    uint8_t *dw, *dcopy, *dstream;
    uint64_t *oid, *oval, *scratch;
    uint32_t* tickets;
    DevStatus* st;
    CK(hipMalloc(&dw, W + 64));
    CK(hipMalloc(&dcopy, W + 64));
    CK(hipMalloc(&dstream, N * 16));
    CK(hipMalloc(&oid, N * 8));
    CK(hipMalloc(&oval, N * 8));
    CK(hipMalloc(&scratch, (f64dec::SCRATCH_WORDS + 1) * 8));
    CK(hipMemset(scratch, 0, (f64dec::SCRATCH_WORDS + 1) * 8));
    tickets = reinterpret_cast<uint32_t*>(scratch + f64dec::SCRATCH_WORDS);
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipMalloc(&st, sizeof(DevStatus)));
    CK(hipMemcpy(dw, w.data(), W, hipMemcpyHostToDevice));
    const uint64_t ntiles = (W + 3967) / 3968 + 1;  // >= the 1p kernel's tiles
    uint64_t* tstat;
    const size_t tstat_bytes = (2 * ntiles + 512 * 16) * 8 + 64;  // agg, pre, dummy lines
    CK(hipMalloc(&tstat, tstat_bytes));
    CK(hipMemset(tstat, 0, tstat_bytes));
    uint32_t epoch = 0;
    uint8_t* moff;
    CK(hipMalloc(&moff, 64 * (W / 4032 + 2)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<uint64_t> hid(N), hval(N);
    auto timeit = [&](const char* name, auto fn, bool check) {
        for (int i = 0; i < 3; i++) fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < reps; i++) fn();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        DevStatus h;
        CK(hipMemcpy(&h, st, sizeof h, hipMemcpyDeviceToHost));
        long bad = -1;
        if (check) {
            CK(hipMemcpy(hid.data(), oid, N * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hval.data(), oval, N * 8, hipMemcpyDeviceToHost));
            bad = 0;
            for (uint64_t i = 0; i < N; i++) bad += hid[i] != i || hval[i] != vals[i];
        }
        printf("%-9s %8.4f ms  %7.1f GB/s (W+16N)  rows=%llu fast_fail=%u timeout=%u cap=%u "
               "mismatches=%ld\n",
               name, ms, (W + 16.0 * N) / ms / 1e6, (unsigned long long)h.n_rows, h.fast_fail,
               h.timeout, h.capacity, bad);
        fflush(stdout);
    };
#define LAUNCH(NS) CK(NS::nxg_launch_dec_f64(dw, W, oid, oval, N, scratch, moff, \
                                            NS::nxg_dec_f64_wgs(ncu), st, 0))
    auto dec = [&](int v) {
        return [&, v]() {
            CK(hipMemsetAsync(st, 0, sizeof(DevStatus), 0));
            CK(hipMemsetAsync(oid, 0, 8, 0));
            if (v == 0) LAUNCH(prod);
            if (v == 2) {
                epoch++;
                CK(p1n::nxg_launch_dec_f64_1p(dw, W, oid, oval, N, tstat, epoch,
                                              p1n::nxg_dec_f64_1p_wgs(ncu), st, 0));
            }
            if (v == 7) {
                epoch++;
                CK(pos::nxg_launch_dec_f64_os(dw, W, oid, oval, N, tstat, epoch, st, 0));
            }
            if (v == 8) {
                epoch++;
                CK(posnt::nxg_launch_dec_f64_os(dw, W, oid, oval, N, tstat, epoch, st, 0));
            }
            if (v == 3) {
                epoch++;
                CK(p1l3::nxg_launch_dec_f64_1p(dw, W, oid, oval, N, tstat, epoch,
                                               p1l3::nxg_dec_f64_1p_wgs(ncu), st, 0));
            }
            if (v == 1) {
                epoch++;
                CK(p1::nxg_launch_dec_f64_1p(dw, W, oid, oval, N, tstat, epoch,
                                             p1::nxg_dec_f64_1p_wgs(ncu), st, 0));
            }
        };
    };
    printf("wgs=%d 1p_wgs=%d (probe build) %d (product) %d (lag2)\n", prod::nxg_dec_f64_wgs(ncu),
           p1::nxg_dec_f64_1p_wgs(ncu), p1n::nxg_dec_f64_1p_wgs(ncu), p1l3::nxg_dec_f64_1p_wgs(ncu));
    printf("records=%llu wire=%llu bytes\n", (unsigned long long)N, (unsigned long long)W);
    timeit("dec2p", dec(0), true);
    timeit("dec1p_prod", dec(2), true);
    timeit("dec_oneshot", dec(7), true);
    timeit("dec_oneshot_nt", dec(8), true);
    timeit("dec1p_prod", dec(2), true);
    timeit("dec_oneshot", dec(7), true);
    timeit("dec_oneshot_nt", dec(8), true);
    timeit("dec1p_lag2", dec(3), true);
    const char* names[4] = {"dec1p", "1p_nowait", "1p_nostore", "1p_nowait_nostore"};
    for (uint32_t f = 0; f < 4; f++) {
        CK(hipMemcpyToSymbol(HIP_SYMBOL(p1::g_1p_dbg), &f, sizeof f));
        unsigned long long z[8] = {0};
        CK(hipMemcpyToSymbol(HIP_SYMBOL(p1::g_1p_cyc), z, sizeof z));
        timeit(names[f], dec(1), f == 0);
        unsigned long long c[8];
        CK(hipMemcpyFromSymbol(c, HIP_SYMBOL(p1::g_1p_cyc), sizeof c));
        double tot = 0;
        for (int i = 0; i < 5; i++) tot += (double)c[i];
        printf("   cycles/wave-step share: stage %.1f%% starts %.1f%% decode %.1f%% wait %.1f%% "
               "store %.1f%% (total %.3g)\n", 100 * c[0] / tot, 100 * c[1] / tot,
               100 * c[2] / tot, 100 * c[3] / tot, 100 * c[4] / tot, tot);
    }
    uint32_t* sink;
    CK(hipMalloc(&sink, 64));
    const uint64_t nt_full = W / 4096;
    timeit("count_mem", [&]() {
        hipLaunchKernelGGL(count_mem_kernel, dim3(prod::nxg_dec_f64_wgs(ncu)), dim3(256), 0, 0, dw,
                           nt_full, sink);
    }, false);
    timeit("emit_mem", [&]() {
        hipLaunchKernelGGL(emit_mem_kernel, dim3(prod::nxg_dec_f64_wgs(ncu)), dim3(256), 0, 0, dw,
                           nt_full, oid, oval, N);
    }, false);
    timeit("stream", [&]() {
        hipLaunchKernelGGL(stream_kernel, dim3(8192), dim3(256), 0, 0, (const uint4*)dw, W / 16,
                           (uint4*)dstream, N);
    }, false);
    timeit("d2d", [&]() { CK(hipMemcpyAsync(dcopy, dw, W, hipMemcpyDeviceToDevice, 0)); }, false);
    return 0;
}
