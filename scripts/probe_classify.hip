// probe_classify.hip -- diagnostics: runs the general decoder's emit-pass classification
// (nxg_decode_gen.hip: classify + the wire-order scans) over tile 0 of a frame file with one
// wave and prints each message's class, child-slot count and child base.
// Usage: probe_classify <frame file>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "../netidx_amd/csrc/nxg_decode_gen.hip"
thread_local DevStatus* nxg_zero_slot = nullptr;
thread_local bool nxg_zero_used = false;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)


__device__ void classify_dbg(const Src& s, uint64_t p) {
    const LdsSrc ls{s.lds, s.t0};
    uint64_t q = p, L;
    uint32_t e0 = dvar(ls, q, s.W, L);
    const uint64_t take = L - vl64(L);
    const uint64_t lim = take < s.W - q ? q + take : s.W;
    printf("p=%llu e0=%u L=%llu q=%llu lim=%llu nlds=%u\n", (unsigned long long)p, e0,
           (unsigned long long)L, (unsigned long long)q, (unsigned long long)lim, s.nlds);
    const uint32_t variant = ls.byte(q++);
    uint64_t id;
    uint32_t e1 = dvar(ls, q, lim, id);
    const uint32_t t = ls.byte(q++);
    uint64_t cnt = 777;
    uint32_t e2 = dvar(ls, q, lim, cnt);
    printf("variant=%u e1=%u id=%llu t=%u e2=%u cnt=%llu q=%llu w=%08x %08x\n", variant, e1,
           (unsigned long long)id, t, e2, (unsigned long long)cnt, (unsigned long long)q,
           ls.word(q - 1), ls.word(q + 3));
    const uint32_t cw = classify(s, p);
    printf("classify k=%u kids=%u\n", cw & 15u, cw >> 8);
}

__global__ void classify_kernel(const uint8_t* wire, uint64_t W, uint32_t* out, uint32_t nmax) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[gdec2::IMG + 16];
    const uint32_t lane = threadIdx.x;
    GRegs g;
    g_load(g, wire, 0, W, lane);
    g_stage(buf, g, lane);
    const Src s = g_src(buf, wire, 0, W);
    // message starts by a sequential walk (one lane), then classify in parallel
    __shared__ uint32_t mpos[2048];
    __shared__ uint32_t nm;
    if (lane == 0) {
        uint64_t p = 0;
        uint32_t k = 0;
        while (p < W && p < 4096 && k < 2048) {
            mpos[k++] = (uint32_t)p;
            uint64_t q = p, L = 1;
            nxgmsg::dvar(nxgmsg::GlbSrc{s.g}, q, W, L);
            const uint64_t take = L - vl64(L);
            p = take < W - q ? q + take : W;
        }
        nm = k;
    }
    __syncthreads();
    uint32_t ccar = 0;
    for (uint32_t m0 = 0; m0 < nm; m0 += 64) {
        const uint32_t m = m0 + lane;
        if (m0 == 64 && lane == 62) classify_dbg(s, mpos[m]);
        const uint32_t cw = m < nm ? classify(s, mpos[m]) : 99u;
        uint32_t kids = cw >> 8, k = cw & 15u;
        bool upd = cw & C_UPD;
        const bool in = m < nm;
        const uint32_t ci = wave_incl_scan(in ? kids : 0u);
        if (in && m < nmax) {
            out[m * 4 + 0] = mpos[m];
            out[m * 4 + 1] = k | (upd ? 0x80u : 0u);
            out[m * 4 + 2] = kids;
            out[m * 4 + 3] = ccar + ci - kids;
        }
        ccar += __shfl(ci, 63, 64);
    }
}

int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    std::vector<uint8_t> w(1 << 20);
    const size_t W = fread(w.data(), 1, w.size(), f);
    fclose(f);
    uint8_t* dw;
    uint32_t* out;
    CK(hipMalloc(&dw, W + 64));
    CK(hipMemcpy(dw, w.data(), W, hipMemcpyHostToDevice));
    const uint32_t nmax = 2048;
    CK(hipMalloc(&out, nmax * 16));
    CK(hipMemset(out, 0xff, nmax * 16));
    hipLaunchKernelGGL(classify_kernel, dim3(1), dim3(64), 0, 0, dw, (uint64_t)W, out, nmax);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> h(nmax * 4);
    CK(hipMemcpy(h.data(), out, nmax * 16, hipMemcpyDeviceToHost));
    for (uint32_t m = 0; m < nmax && h[m * 4] != 0xffffffffu; m++)
        printf("%u pos=%u cls=%u upd=%u kids=%u cb=%u\n", m, h[m * 4], h[m * 4 + 1] & 0x7f,
               h[m * 4 + 1] >> 7, h[m * 4 + 2], h[m * 4 + 3]);
    return 0;
}
