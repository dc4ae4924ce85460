// probe_copy.hip -- diagnostics: the practical HBM ceiling for the f64 decode's traffic shape
// (read W wire bytes, write 16N column bytes as two 8N arrays), by copy kernels of several
// shapes. Usage: probe_copy <N>   (W = 14.98 N bytes, as config 2/5)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <functional>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ inline uint4 ntld(const uint4* p) {
    const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ inline void ntst(uint4 v, uint4* p) {
    v4u x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(p));
}

// A: one 16-B load + store per iteration (the old probe's stream kernel)
__global__ void copy_a(const uint4* __restrict__ in, uint64_t nin, uint4* __restrict__ out,
                       uint64_t nout) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nout; i += stride)
        out[i] = i < nin ? in[i] : make_uint4(0, 0, 0, 0);
}

// B: U loads in flight per lane, then U stores; blocks own contiguous chunks of U*TPB*16 B
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_b(const uint4* __restrict__ in, uint64_t nin,
                                              uint4* __restrict__ out, uint64_t nout) {
    const uint64_t per = (uint64_t)U * 256;
    for (uint64_t b = (uint64_t)blockIdx.x * per; b < nout; b += (uint64_t)gridDim.x * per) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = b + u * 256 + threadIdx.x;
            if (NT) v[u] = i < nin ? ntld(in + i) : make_uint4(0, 0, 0, 0);
            else v[u] = i < nin ? in[i] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = b + u * 256 + threadIdx.x;
            if (i < nout) {
                if (NT) ntst(v[u], out + i);
                else out[i] = v[u];
            }
        }
    }
}

// C: the decoder's shape: a wave reads a 4 KiB tile (4 x 16 B per lane), writes the tile's
// ~272 records as two u64 arrays (8 B per lane per store); persistent grid, contiguous runs
template <bool NT>
__global__ __launch_bounds__(256) void copy_c(const uint8_t* __restrict__ wire, uint64_t W,
                                              uint64_t* __restrict__ oid, uint64_t* __restrict__ oval,
                                              uint64_t N) {
    const uint32_t lane = threadIdx.x & 63, R = gridDim.x * 4;
    const uint32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t nt = (W + 4031) / 4032;
    const uint64_t tb = nt * r / R, te = nt * (r + 1) / R;
    for (uint64_t t = tb; t < te; t++) {
        const uint4* p = reinterpret_cast<const uint4*>(wire + t * 4032);
        uint4 a[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t off = t * 4032 + (u * 64 + lane) * 16;
            a[u] = off + 16 <= W ? (NT ? ntld(p + u * 64 + lane) : p[u * 64 + lane])
                                 : make_uint4(0, 0, 0, 0);
        }
        const uint64_t r0 = N * t / nt, r1 = N * (t + 1) / nt;
        uint64_t x = (uint64_t)(a[0].x ^ a[1].y) << 32 | (a[2].z ^ a[3].w);
        for (uint64_t i = r0 + lane; i < r1; i += 64) {
            if (NT) {
                __builtin_nontemporal_store(x, oid + i);
                __builtin_nontemporal_store(x + 1, oval + i);
            } else {
                oid[i] = x;
                oval[i] = x + 1;
            }
        }
    }
}


// D: interleaved tiles (t = k*V + v) with the next tile prefetched into registers while the
// current one is "stored": SW = 8 (one record per lane per store, two u64 arrays) or 16 (two
// records per lane: aligned uint4 stores of id pairs / value pairs, edges by 8-B stores)
template <int SW>
__global__ __launch_bounds__(256) void copy_d(const uint8_t* __restrict__ wire, uint64_t W,
                                              uint64_t* __restrict__ oid, uint64_t* __restrict__ oval,
                                              uint64_t N) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t V = (uint64_t)gridDim.x * 4, v = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t nt = (W + 4031) / 4032;
    uint4 a[4];
    auto ld = [&](uint64_t t) {
        const uint4* p = reinterpret_cast<const uint4*>(wire + t * 4032);
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t off = t * 4032 + (u * 64 + lane) * 16;
            a[u] = off + 16 <= W ? p[u * 64 + lane] : make_uint4(0, 0, 0, 0);
        }
    };
    if (v < nt) ld(v);
    for (uint64_t t = v; t < nt; t += V) {
        uint64_t x = (uint64_t)(a[0].x ^ a[1].y) << 32 | (a[2].z ^ a[3].w);
        if (t + V < nt) ld(t + V);
        const uint64_t r0 = N * t / nt, r1 = N * (t + 1) / nt;
        if (SW == 8) {
            for (uint64_t i = r0 + lane; i < r1; i += 64) {
                oid[i] = x;
                oval[i] = x + 1;
            }
        } else {
            const uint64_t a0 = (r0 + 1) & ~1ull, a1 = r1 & ~1ull;  // aligned pair range
            if (lane == 0 && r0 < a0) { oid[r0] = x; oval[r0] = x; }
            if (lane == 1 && a1 < r1 && a1 >= a0) { oid[a1] = x; oval[a1] = x; }
            for (uint64_t i = a0 + 2 * lane; i < a1; i += 128) {
                *reinterpret_cast<uint4*>(oid + i) = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)x, 0);
                *reinterpret_cast<uint4*>(oval + i) = make_uint4((uint32_t)x, 1, (uint32_t)x, 2);
            }
        }
    }
}

int main(int argc, char** argv) {
    const uint64_t N = argc > 1 ? strtoull(argv[1], 0, 10) : 100000000ull;
    const uint64_t W = N * 1498 / 100;
    uint8_t* dw;
    uint64_t *oid, *oval;
    CK(hipMalloc(&dw, W + 64));
    CK(hipMalloc(&oid, N * 16));
    oval = oid + N;
    CK(hipMemset(dw, 0x5a, W + 64));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)W + 16.0 * N;
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    auto timeit = [&](const char* name, std::function<void()> f) {
        for (int i = 0; i < 3; i++) f();
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int i = 0; i < 20; i++) {
            CK(hipEventRecord(e0, 0));
            f();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%-28s %8.4f ms  %7.1f GB/s (W+16N)\n", name, ts[10], bytes / ts[10] / 1e6);
        fflush(stdout);
    };
    const uint64_t nin = W / 16, nout = N;  // 16N bytes out as uint4
    timeit("A 8192x256", [&] { hipLaunchKernelGGL(copy_a, dim3(8192), dim3(256), 0, 0, (const uint4*)dw, nin, (uint4*)oid, nout); });
    for (int g : {ncu * 4, ncu * 8, ncu * 16, 8192, 32768}) {
        char nm[64];
        snprintf(nm, sizeof nm, "B U4 g%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL((copy_b<4, false>), dim3(g), dim3(256), 0, 0, (const uint4*)dw, nin, (uint4*)oid, nout); });
        snprintf(nm, sizeof nm, "B U8 g%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL((copy_b<8, false>), dim3(g), dim3(256), 0, 0, (const uint4*)dw, nin, (uint4*)oid, nout); });
        snprintf(nm, sizeof nm, "B U4 nt g%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL((copy_b<4, true>), dim3(g), dim3(256), 0, 0, (const uint4*)dw, nin, (uint4*)oid, nout); });
    }
    {
        const uint64_t nblk = (nout + 1023) / 1024;
        timeit("B U4 one-shot", [&] { hipLaunchKernelGGL((copy_b<4, false>), dim3((uint32_t)nblk), dim3(256), 0, 0, (const uint4*)dw, nin, (uint4*)oid, nout); });
        timeit("B U4 nt one-shot", [&] { hipLaunchKernelGGL((copy_b<4, true>), dim3((uint32_t)nblk), dim3(256), 0, 0, (const uint4*)dw, nin, (uint4*)oid, nout); });
    }
    for (int occ : {2, 4, 8}) {
        char nm[64];
        snprintf(nm, sizeof nm, "C tiles occ%d", occ);
        timeit(nm, [&] { hipLaunchKernelGGL((copy_c<false>), dim3(ncu * occ), dim3(256), 0, 0, dw, W, oid, oval, N); });
        snprintf(nm, sizeof nm, "C tiles nt occ%d", occ);
        timeit(nm, [&] { hipLaunchKernelGGL((copy_c<true>), dim3(ncu * occ), dim3(256), 0, 0, dw, W, oid, oval, N); });
    }
    for (int occ : {2, 4, 8}) {
        char nm[64];
        snprintf(nm, sizeof nm, "D8 interleaved occ%d", occ);
        timeit(nm, [&] { hipLaunchKernelGGL((copy_d<8>), dim3(ncu * occ), dim3(256), 0, 0, dw, W, oid, oval, N); });
        snprintf(nm, sizeof nm, "D16 interleaved occ%d", occ);
        timeit(nm, [&] { hipLaunchKernelGGL((copy_d<16>), dim3(ncu * occ), dim3(256), 0, 0, dw, W, oid, oval, N); });
    }
    {
        const uint32_t g = (uint32_t)(((W + 4031) / 4032 + 3) / 4);
        timeit("D8 one-shot", [&] { hipLaunchKernelGGL((copy_d<8>), dim3(g), dim3(256), 0, 0, dw, W, oid, oval, N); });
        timeit("D16 one-shot", [&] { hipLaunchKernelGGL((copy_d<16>), dim3(g), dim3(256), 0, 0, dw, W, oid, oval, N); });
    }
    return 0;
}
