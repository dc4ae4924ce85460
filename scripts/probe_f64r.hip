// probe_f64r.hip -- timing probe for the length-run f64 decode (nxg_decode_f64_run.hip) against
// the persistent single-pass decoder (nxg_decode_f64_1p.hip) and a plain stream kernel.
// Frames (all From::Update(Id, F64)): seq = ids 0..N-1 in order (Id::new order, BASELINE
// configs[1]); x28 = sequential ids straddling 2^28 (4- and 5-byte varints); perm = a random
// permutation of 0..N-1 (record lengths vary record to record); w35 = random ids in [2^28, 2^35).
// Every decode is checked against the generator's columns.
// Usage: probe_f64r [records] [reps]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#include "../netidx_amd/csrc/nxg_f64_rec.h"
#define NXG_F64R_NT 0
#define NXG_F64R_LDS 0
#define NXG_F64R_DPP 0
#define NXG_F64R_R 4

namespace p1n {
#include "../netidx_amd/csrc/nxg_decode_f64_1p.hip"
}
namespace fr {
#include "../netidx_amd/csrc/nxg_decode_f64_run.hip"
}
#undef NXG_F64R_NT
#define NXG_F64R_NT 4
namespace fr8 {  // nontemporal stores for the tile's inner lines
#include "../netidx_amd/csrc/nxg_decode_f64_run.hip"
}
#undef NXG_F64R_NT
#define NXG_F64R_NT 0
#undef NXG_F64R_T
#define NXG_F64R_T 16384
namespace fr4 {  // 16 KiB probe tiles
#include "../netidx_amd/csrc/nxg_decode_f64_run.hip"
}
#undef NXG_F64R_T
#define NXG_F64R_T 32768
#undef NXG_F64R_DPP
#define NXG_F64R_DPP 1
namespace frdn {  // one load per record
#include "../netidx_amd/csrc/nxg_decode_f64_run.hip"
}
#undef NXG_F64R_DPP
#define NXG_F64R_DPP 0
#undef NXG_F64R_DPP
#define NXG_F64R_DPP 1
#undef NXG_F64R_NT
#define NXG_F64R_NT 4
namespace frd {  // one load per record + inner nontemporal stores
#include "../netidx_amd/csrc/nxg_decode_f64_run.hip"
}
#undef NXG_F64R_DPP
#define NXG_F64R_DPP 0
#undef NXG_F64R_NT
#define NXG_F64R_NT 0
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

// the emit's memory pattern without parsing: lane k reads 16 B at 15 k and writes 8 B to each
// of two columns
__global__ void copy2col_kernel(const uint8_t* __restrict__ in, uint64_t N,
                                uint64_t* __restrict__ a, uint64_t* __restrict__ b) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += stride) {
        const uint4 v = *reinterpret_cast<const uint4*>(in + ((15 * i) & ~15ull));
        a[i] = ((uint64_t)v.y << 32) | v.x;
        b[i] = ((uint64_t)v.w << 32) | v.z;
    }
}
typedef uint32_t v4p __attribute__((ext_vector_type(4)));
__global__ void stream_nt_kernel(const v4p* __restrict__ in, uint64_t nin, v4p* __restrict__ out,
                                 uint64_t nout) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nout; i += 4 * stride) {
        v4p v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t j = i + k * stride;
            v[k] = j < nin ? __builtin_nontemporal_load(in + j) : v4p{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t j = i + k * stride;
            if (j < nout) __builtin_nontemporal_store(v[k], out + j);
        }
    }
}

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void build(const std::vector<uint64_t>& ids, std::vector<uint64_t>& vals,
                  std::vector<uint8_t>& w) {
    uint64_t seed = 7;
    w.clear();
    w.reserve(ids.size() * 16);
    vals.resize(ids.size());
    for (size_t i = 0; i < ids.size(); i++) {
        uint8_t idb[10];
        int nb = 0;
        uint64_t v = ids[i];
        while (v >= 0x80) { idb[nb++] = (uint8_t)(v | 0x80); v >>= 7; }
        idb[nb++] = (uint8_t)v;
        w.push_back((uint8_t)(11 + nb));
        w.push_back(4);
        for (int k = 0; k < nb; k++) w.push_back(idb[k]);
        w.push_back(9);
        const uint64_t f = vals[i] = splitmix(seed);
        for (int k = 7; k >= 0; k--) w.push_back((uint8_t)(f >> (8 * k)));
    }
}

int main(int argc, char** argv) {
    const uint64_t N = argc > 1 ? strtoull(argv[1], 0, 0) : 10000000ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    uint64_t *oid, *oval, *tstat;
    uint8_t *dw, *dstream;
    void* desc;
    DevStatus* st;
    const uint64_t Wmax = N * 16 + 64;
    CK(hipMalloc(&dw, Wmax));
    CK(hipMalloc(&dstream, N * 16 + 64));
    CK(hipMalloc(&oid, N * 8));
    CK(hipMalloc(&oval, N * 8));
    CK(hipMalloc(&desc, (Wmax / 4096 + 2) * 16));
    const size_t tsw = 2 * (Wmax / 3968 + 2) + 4096;
    CK(hipMalloc(&tstat, tsw * 8));
    CK(hipMemset(tstat, 0, tsw * 8));
    CK(hipMalloc(&st, sizeof(DevStatus) * 2));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    uint32_t epoch = 0;
    std::vector<uint64_t> hid(N), hval(N);

    auto run = [&](const char* name, const std::vector<uint64_t>& ids,
                   const std::vector<uint64_t>& vals, uint64_t W, int which,
                   uint32_t flags = 0) {
        auto fn = [&]() {
            CK(hipMemsetAsync(st, 0, sizeof(DevStatus), 0));
            epoch++;
            if (which == 0)
                CK(fr::nxg_launch_dec_f64r(dw, W, 0, W, oid, oval, N, desc, tstat, epoch, flags, st, 0));
            else if (which == 8)
                CK(fr8::nxg_launch_dec_f64r(dw, W, 0, W, oid, oval, N, desc, tstat, epoch, flags, st, 0));
            else if (which == 4)
                CK(fr4::nxg_launch_dec_f64r(dw, W, 0, W, oid, oval, N, desc, tstat, epoch, flags, st, 0));
            else if (which == 5)
                CK(frd::nxg_launch_dec_f64r(dw, W, 0, W, oid, oval, N, desc, tstat, epoch, flags, st, 0));
            else if (which == 6)
                CK(frdn::nxg_launch_dec_f64r(dw, W, 0, W, oid, oval, N, desc, tstat, epoch, flags, st, 0));
            else if (which == 20) {  // the probe kernel alone
                const uint64_t nt = fr::nxg_dec_f64r_tiles(W);
                hipLaunchKernelGGL(fr::nxg_f64r_probe_kernel, dim3(fr::nxg_dec_f64r_groups(W)),
                                   dim3(256), 0, 0, dw, W, W, (uint64_t)0, nt,
                                   (fr::f64r::Desc*)desc, tstat, epoch, 12u, st,
                                   (DevStatus*)nullptr);
            } else if (which == 21) {  // the emit kernel alone (descriptors of the last run)
                const uint64_t nt = fr::nxg_dec_f64r_tiles(W);
                hipLaunchKernelGGL(fr::nxg_f64r_emit_kernel, dim3((nt * fr::f64r::ESUB + 3) / 4),
                                   dim3(256), 0, 0, dw, W, W, (uint64_t)0, nt,
                                   (const fr::f64r::Desc*)desc, oid, oval, N, 12u, st);
            }
            else
                CK(p1n::nxg_launch_dec_f64_1p(dw, W, oid, oval, N, tstat, epoch,
                                              p1n::nxg_dec_f64_1p_wgs(ncu), st, 0));
        };
        for (int i = 0; i < 3; i++) fn();
        CK(hipDeviceSynchronize());
        CK(hipMemset(oid, 0xff, N * 8));
        CK(hipMemset(oval, 0xff, N * 8));
        fn();
        CK(hipDeviceSynchronize());
        DevStatus h;
        CK(hipMemcpy(&h, st, sizeof h, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hid.data(), oid, N * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hval.data(), oval, N * 8, hipMemcpyDeviceToHost));
        long bad = 0;
        for (uint64_t i = 0; i < N; i++) bad += hid[i] != ids[i] || hval[i] != vals[i];
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < reps; i++) fn();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        printf("%-14s %-5s %8.4f ms %7.1f GB/s (W+16N) %5.1f%% rows=%llu ff=%u irr=%u to=%u "
               "cap=%u exact_tiles=%llu mismatches=%ld\n",
               which == 1 ? "f64_1p" : which == 8 ? "f64run_ntIn" : which == 4 ? "f64run_T16k"
               : which == 5 ? "f64run_dppntIn" : which == 6 ? "f64run_dpp"
               : which == 20 ? "probe_only" : which == 21 ? "emit_only"
               : (flags & 1 ? "f64run_exact" : flags & 2 ? "f64run_nobail" : "f64run"),
               name, ms, (W + 16.0 * N) / ms / 1e6,
               (W + 16.0 * N) / ms / 1e6 / 8000 * 100, (unsigned long long)h.n_rows, h.fast_fail,
               h.irregular, h.timeout, h.capacity, (unsigned long long)h.diag[0], bad);
        fflush(stdout);
    };

    std::vector<uint64_t> ids(N), vals;
    std::vector<uint8_t> w;
    const char* names[4] = {"seq", "x28", "perm", "w35"};
    for (int f = 0; f < 4; f++) {
        if (f == 0) for (uint64_t i = 0; i < N; i++) ids[i] = i;
        if (f == 1) for (uint64_t i = 0; i < N; i++) ids[i] = (1ull << 28) - N / 2 + i;
        if (f == 2) {
            for (uint64_t i = 0; i < N; i++) ids[i] = i;
            std::mt19937_64 g(11);
            std::shuffle(ids.begin(), ids.end(), g);
        }
        if (f == 3) {
            uint64_t s = 99;
            for (uint64_t i = 0; i < N; i++)
                ids[i] = (1ull << 28) + splitmix(s) % ((1ull << 35) - (1ull << 28));
        }
        build(ids, vals, w);
        const uint64_t W = w.size();
        CK(hipMemcpy(dw, w.data(), W, hipMemcpyHostToDevice));
        printf("frame %s: records=%llu wire=%llu bytes\n", names[f], (unsigned long long)N,
               (unsigned long long)W);
        run(names[f], ids, vals, W, 0);
        if (f != 2) {
            run(names[f], ids, vals, W, 8);
            run(names[f], ids, vals, W, 4);
            run(names[f], ids, vals, W, 5);
            run(names[f], ids, vals, W, 6);
        }
        if (f == 0 || f == 2) run(names[f], ids, vals, W, 1);
        if (f == 2) run(names[f], ids, vals, W, 0, 2);            // two-run search everywhere
        if (f == 0) {
            run(names[f], ids, vals, W, 0);
            run(names[f], ids, vals, W, 20);
            run(names[f], ids, vals, W, 0);
            run(names[f], ids, vals, W, 21);
            run(names[f], ids, vals, W, 1);
            auto tstream = [&](const char* nm, int grid) {
                for (int i = 0; i < 3; i++)
                    hipLaunchKernelGGL(stream_kernel, dim3(grid), dim3(256), 0, 0,
                                       (const uint4*)dw, W / 16, (uint4*)dstream, N);
                CK(hipEventRecord(a, 0));
                for (int i = 0; i < reps; i++)
                    hipLaunchKernelGGL(stream_kernel, dim3(grid), dim3(256), 0, 0,
                                       (const uint4*)dw, W / 16, (uint4*)dstream, N);
                CK(hipEventRecord(b, 0));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                ms /= reps;
                printf("%-14s %-5s %8.4f ms %7.1f GB/s (W+16N) %5.1f%%\n", nm, "seq", ms,
                       (W + 16.0 * N) / ms / 1e6, (W + 16.0 * N) / ms / 1e6 / 80);
            };
            tstream("stream_8192", 8192);
            {
                auto t2 = [&](const char* nm, auto launch) {
                    for (int i = 0; i < 3; i++) launch();
                    CK(hipEventRecord(a, 0));
                    for (int i = 0; i < reps; i++) launch();
                    CK(hipEventRecord(b, 0));
                    CK(hipEventSynchronize(b));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, a, b));
                    ms /= reps;
                    printf("%-14s %-5s %8.4f ms %7.1f GB/s (W+16N) %5.1f%%\n", nm, "seq", ms,
                           (W + 16.0 * N) / ms / 1e6, (W + 16.0 * N) / ms / 1e6 / 80);
                };
                t2("copy2col", [&]() {
                    hipLaunchKernelGGL(copy2col_kernel, dim3(8192), dim3(256), 0, 0, dw, N, oid,
                                       oval);
                });
                t2("stream_nt", [&]() {
                    hipLaunchKernelGGL(stream_nt_kernel, dim3(2048), dim3(256), 0, 0,
                                       (const v4p*)dw, W / 16, (v4p*)dstream, N);
                });
            }
            tstream("stream_2048", 2048);
        }
    }
    return 0;
}
