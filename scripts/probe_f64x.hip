// probe_f64x.hip -- diagnostics for the single-pass f64 decoder (nxg_decode_f64_x.hip): decodes
// frames of From::Update(Id, F64) records (sequential ids 0..n-1, or a random permutation) and
// prints the status plus, for the first chunks whose start-mask check fails, the masks the lane
// computed. Usage: probe_f64x [records] [perm 0/1]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <vector>

#include <hip/hip_runtime.h>

struct DiagRec {
    unsigned long long v[8];
};
__device__ DiagRec g_diag[64];
__device__ unsigned int g_ndiag;
__device__ void nxg_f64x_diag(unsigned long long fp, unsigned long long S, unsigned long long slo,
                              unsigned long long sin, unsigned long long shi,
                              unsigned long long Snx, unsigned long long wlo,
                              unsigned long long whi) {
    const unsigned k = atomicAdd(&g_ndiag, 1u);
    if (k < 64) g_diag[k] = DiagRec{{fp, S, slo, sin, shi, Snx, wlo, whi}};
}
#define NXG_F64X_DIAG 1
#include "../netidx_amd/csrc/nxg_decode_f64_x.hip"

thread_local DevStatus* nxg_zero_slot = nullptr;
thread_local bool nxg_zero_used = false;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

static void put_varint(std::vector<uint8_t>& o, uint64_t v) {
    while (v >= 0x80) {
        o.push_back((uint8_t)(v | 0x80));
        v >>= 7;
    }
    o.push_back((uint8_t)v);
}

int main(int argc, char** argv) {
    setvbuf(stdout, nullptr, _IONBF, 0);
    printf("start\n");
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : 1000;
    const int perm = argc > 2 ? atoi(argv[2]) : 0;
    std::vector<uint64_t> ids(n), vals(n);
    for (uint64_t i = 0; i < n; i++) ids[i] = i;
    if (perm) std::shuffle(ids.begin(), ids.end(), std::mt19937_64(7));
    std::mt19937_64 rng(11);
    std::vector<uint8_t> w;
    for (uint64_t i = 0; i < n; i++) {
        double d = (double)(rng() % 1000000) * 0.25;
        memcpy(&vals[i], &d, 8);
        std::vector<uint8_t> body;
        body.push_back(4);
        put_varint(body, ids[i]);
        body.push_back(9);
        for (int b = 7; b >= 0; b--) body.push_back((uint8_t)(vals[i] >> (8 * b)));
        w.push_back((uint8_t)(body.size() + 1));  // encoded_len: the whole message (pack.rs:533)
        w.insert(w.end(), body.begin(), body.end());
    }
    if (argc > 3) {  // a frame from a file (sequential / permuted ids are then unknown: no row check)
        FILE* f = fopen(argv[3], "rb");
        if (!f) { perror(argv[3]); return 1; }
        fseek(f, 0, SEEK_END);
        const long sz = ftell(f);
        fseek(f, 0, SEEK_SET);
        w.resize(sz);
        if (fread(w.data(), 1, sz, f) != (size_t)sz) return 1;
        fclose(f);
    }
    const uint64_t W = w.size();
    uint8_t* dw;
    uint64_t *oid, *oval, *tstat;
    DevStatus* st;
    CK(hipMalloc(&dw, W + 64));
    CK(hipMemcpy(dw, w.data(), W, hipMemcpyHostToDevice));
    CK(hipMalloc(&oid, n * 8 + 8));
    CK(hipMalloc(&oval, n * 8 + 8));
    const uint64_t ng = nxg_dec_f64x_groups(W);
    CK(hipMalloc(&tstat, (ng + 1) * 8));
    CK(hipMemset(tstat, 0, (ng + 1) * 8));
    CK(hipMalloc(&st, 2 * sizeof(DevStatus)));
    CK(hipMemset(st, 0, 2 * sizeof(DevStatus)));
    nxg_zero_slot = st + 1;
    printf("launch W=%llu\n", (unsigned long long)W);
    CK(nxg_launch_dec_f64x(dw, W, oid, oval, n, tstat, 1, st, 0));
    CK(hipDeviceSynchronize());
    printf("done\n");
    DevStatus h;
    CK(hipMemcpy(&h, st, sizeof h, hipMemcpyDeviceToHost));
    unsigned nd = 0;
    CK(hipMemcpyFromSymbol(&nd, HIP_SYMBOL(g_ndiag), 4));
    std::vector<DiagRec> dr(64);
    CK(hipMemcpyFromSymbol(dr.data(), HIP_SYMBOL(g_diag), sizeof(DiagRec) * 64));
    std::vector<uint64_t> gi(n), gv(n);
    CK(hipMemcpy(gi.data(), oid, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gv.data(), oval, n * 8, hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; i++) bad += gi[i] != ids[i] || gv[i] != vals[i];
    printf("n=%llu W=%llu groups=%llu: fast_fail %u timeout %u path %u rows %llu capacity %u; "
           "rows differing %llu; failing chunks %u\n",
           (unsigned long long)n, (unsigned long long)W, (unsigned long long)ng, h.fast_fail,
           h.timeout, h.path, (unsigned long long)h.n_rows, h.capacity, (unsigned long long)bad,
           nd);
    // the true starts, for comparison
    std::vector<uint8_t> isstart(W + 1, 0);
    for (uint64_t p = 0; p < W; p += w[p]) isstart[p] = 1;
    for (unsigned k = 0; k < std::min(nd, 12u); k++) {
        const DiagRec& r = dr[k];
        const uint64_t fp = r.v[0];
        uint64_t truth = 0;
        for (int i = 0; i < 64; i++)
            if (fp + i < W && isstart[fp + i]) truth |= 1ull << i;
        printf("fp %llu: S %016llx true %016llx slo %016llx sin %016llx shi %016llx Snx %016llx "
               "wlo %llx whi %llx\n",
               r.v[0], r.v[1], (unsigned long long)truth, r.v[2], r.v[3], r.v[4], r.v[5], r.v[6],
               r.v[7]);
    }
    return 0;
}
