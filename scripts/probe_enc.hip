// probe_enc.hip -- standalone timing probe for the f64 encode (diagnostics, not product).
// Variants of nxg_encode_f64.hip (records per thread, staging bytes per record, nontemporal loads/stores)
// timed with HIP events on the same box, each checked byte for byte against a host encoding:
// sequential ids (config 4) and, at 10^6 records, random 64-bit ids (every varint width, and
// tiles past the 16-byte staging take the byte-by-byte global path).
// Usage: probe_enc [records] [reps]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../netidx_amd/csrc/nxg_device.h"
thread_local DevStatus* nxg_zero_slot = nullptr;
thread_local bool nxg_zero_used = false;

#define NXG_ENC_RPT 4
#define NXG_ENC_STGB 21
#define NXG_ENC_NT 0
namespace e0 {  // the r01e encode
#include "../netidx_amd/csrc/nxg_encode_f64.hip"
}
#undef NXG_ENC_RPT
#undef NXG_ENC_STGB
#define NXG_ENC_RPT 8
#define NXG_ENC_STGB 15
namespace e1 {
#include "../netidx_amd/csrc/nxg_encode_f64.hip"
}
#undef NXG_ENC_NT
#define NXG_ENC_NT 1
namespace e2 {
#include "../netidx_amd/csrc/nxg_encode_f64.hip"
}
#undef NXG_ENC_NT
#undef NXG_ENC_RPT
#undef NXG_ENC_STGB
namespace e3 {  // the product defaults (8 records per thread, 15-byte staging, nt stores)
#include "../netidx_amd/csrc/nxg_encode_f64.hip"
}
#undef NXG_ENC_NT
#define NXG_ENC_NT 3
namespace e4 {
#include "../netidx_amd/csrc/nxg_encode_f64.hip"
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void host_encode(const std::vector<uint64_t>& id, const std::vector<uint64_t>& v,
                        std::vector<uint8_t>& w) {
    w.clear();
    for (size_t i = 0; i < id.size(); i++) {
        uint8_t b[10];
        int nb = 0;
        uint64_t x = id[i];
        while (x >= 0x80) { b[nb++] = (uint8_t)(x | 0x80); x >>= 7; }
        b[nb++] = (uint8_t)x;
        w.push_back((uint8_t)(11 + nb));
        w.push_back(4);
        for (int k = 0; k < nb; k++) w.push_back(b[k]);
        w.push_back(9);
        for (int k = 7; k >= 0; k--) w.push_back((uint8_t)(v[i] >> (8 * k)));
    }
}

int main(int argc, char** argv) {
    const uint64_t N = argc > 1 ? strtoull(argv[1], 0, 0) : 10000000ull;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const uint64_t NR = 1000000;  // random-id check
    std::vector<uint64_t> id(N), val(N), rid(NR), rval(NR);
    uint64_t seed = 11;
    for (uint64_t i = 0; i < N; i++) { id[i] = i; val[i] = splitmix(seed); }
    for (uint64_t i = 0; i < NR; i++) {
        const uint64_t r = splitmix(seed);
        rid[i] = r >> (r & 63);  // every varint width
        rval[i] = splitmix(seed);
    }
    std::vector<uint8_t> ref, rref;
    host_encode(id, val, ref);
    host_encode(rid, rval, rref);
    const uint64_t W = ref.size(), RW = rref.size();
    uint64_t *did, *dval, *drid, *drval, *tstat;
    uint8_t* out;
    DevStatus* st;
    CK(hipMalloc(&did, N * 8));
    CK(hipMalloc(&dval, N * 8));
    CK(hipMalloc(&drid, NR * 8));
    CK(hipMalloc(&drval, NR * 8));
    const uint64_t cap = (W > RW ? W : RW) + 64;
    CK(hipMalloc(&out, cap));
    CK(hipMalloc(&tstat, (N / 256 + 64) * 8));
    CK(hipMemset(tstat, 0, (N / 256 + 64) * 8));
    CK(hipMalloc(&st, sizeof(DevStatus)));
    CK(hipMemcpy(did, id.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dval, val.data(), N * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(drid, rid.data(), NR * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(drval, rval.data(), NR * 8, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    uint32_t epoch = 0;
    std::vector<uint8_t> h(cap);
    printf("records=%llu wire=%llu bytes (random-id check: %llu records, %llu bytes)\n",
           (unsigned long long)N, (unsigned long long)W, (unsigned long long)NR,
           (unsigned long long)RW);
#define RUN(NS, I, V, NN) CK(NS::nxg_launch_enc_f64(I, V, NN, out, cap, tstat, ++epoch, st, 0, 0))
    auto variant = [&](const char* name, auto launch) {
        // correctness: random ids, then sequential ids
        CK(hipMemset(st, 0, sizeof(DevStatus)));
        launch(drid, drval, NR);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), out, RW, hipMemcpyDeviceToHost));
        DevStatus hs;
        CK(hipMemcpy(&hs, st, sizeof hs, hipMemcpyDeviceToHost));
        const bool rok = memcmp(h.data(), rref.data(), RW) == 0 && hs.total_bytes == RW;
        for (int i = 0; i < 3; i++) launch(did, dval, N);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < reps; i++) launch(did, dval, N);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        ms /= reps;
        CK(hipMemcpy(h.data(), out, W, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&hs, st, sizeof hs, hipMemcpyDeviceToHost));
        const bool ok = memcmp(h.data(), ref.data(), W) == 0 && hs.total_bytes == W;
        printf("%-22s %8.4f ms  %7.1f GB/s (16N+W)  seq_ok=%d random_ok=%d timeout=%u cap=%u\n",
               name, ms, (W + 16.0 * N) / ms / 1e6, ok, rok, hs.timeout, hs.capacity);
        fflush(stdout);
    };
    for (int pass = 0; pass < 2; pass++) {
        variant("r01e_rpt4_stg21", [&](uint64_t* I, uint64_t* V, uint64_t n) { RUN(e0, I, V, n); });
        variant("rpt8_stg15", [&](uint64_t* I, uint64_t* V, uint64_t n) { RUN(e1, I, V, n); });
        variant("rpt8_nt_loads", [&](uint64_t* I, uint64_t* V, uint64_t n) { RUN(e2, I, V, n); });
        variant("product_rpt8_nt_stores", [&](uint64_t* I, uint64_t* V, uint64_t n) { RUN(e3, I, V, n); });
        variant("rpt8_nt_both", [&](uint64_t* I, uint64_t* V, uint64_t n) { RUN(e4, I, V, n); });
    }
    return 0;
}
