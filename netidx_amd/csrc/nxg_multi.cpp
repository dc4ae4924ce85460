// nxg_multi.cpp -- multi-GPU calls of the C ABI (include/nxg_codec.h): an RCCL communicator over
// xGMI, the sharded encode of BASELINE configs[4] (shards encoded into their final offsets, then
// grouped send/recv: SURVEY.md H5) and the byte-range sharded decode.
//
// Only the public ABI and librccl are used here. librccl is opened at nxg_comm_init with dlopen
// (RTLD_GLOBAL, soname librccl.so.1): the codec loads on a machine without RCCL, and inside a
// process that already has RCCL (PyTorch's torch.distributed) the same library is shared.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/nxg_codec.h"

namespace {

void set_err(NetidxError* err, const char* fmt, ...) {
    if (!err) return;
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    free(err->msg);
    err->msg = strdup(buf);
}

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t,
                         hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

bool rccl(Rccl** out, NetidxError* err) {
    static Rccl r;
    static bool tried = false, ok = false;
    if (!tried) {
        tried = true;
        r.h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!r.h) r.h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (r.h) {
            auto sym = [&](const char* n) { return dlsym(r.h, n); };
            r.GetUniqueId = (decltype(r.GetUniqueId))sym("ncclGetUniqueId");
            r.CommInitRank = (decltype(r.CommInitRank))sym("ncclCommInitRank");
            r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
            r.AllGather = (decltype(r.AllGather))sym("ncclAllGather");
            r.Send = (decltype(r.Send))sym("ncclSend");
            r.Recv = (decltype(r.Recv))sym("ncclRecv");
            r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
            r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
            r.GetErrorString = (decltype(r.GetErrorString))sym("ncclGetErrorString");
            ok = r.GetUniqueId && r.CommInitRank && r.CommDestroy && r.AllGather && r.Send &&
                 r.Recv && r.GroupStart && r.GroupEnd && r.GetErrorString;
        }
    }
    if (!ok) {
        set_err(err, "librccl is not available (dlopen librccl.so.1: %s)",
                r.h ? "missing symbols" : dlerror());
        return false;
    }
    *out = &r;
    return true;
}

}  // namespace

struct NxgComm {
    Rccl* r = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0;
    hipStream_t stream = nullptr;  // the ctx's stream at init
    uint64_t* dscratch = nullptr;  // per-rank exchange slots (sizes, range summaries)
};

#define NCCLCHK(expr)                                                                         \
    do {                                                                                      \
        ncclResult_t r_ = (expr);                                                             \
        if (r_ != ncclSuccess) {                                                              \
            set_err(err, "%s failed: %s", #expr, comm->r->GetErrorString(r_));                \
            return false;                                                                     \
        }                                                                                     \
    } while (0)
#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) {                                                               \
            set_err(err, "%s failed: %s", #expr, hipGetErrorString(e_));                      \
            return false;                                                                     \
        }                                                                                     \
    } while (0)

namespace {
constexpr int kSlotWords = 8;  // one rank's exchange slot: 64 bytes (an NxgRange fits)
static_assert(sizeof(NxgRange) <= kSlotWords * 8, "range summary fits a slot");

// all-gather of one 64-byte slot per rank: mine -> all[0 .. nranks)
bool gather_slots(NxgComm* comm, const void* mine, void* all, NetidxError* err) {
    uint64_t* d = comm->dscratch;  // [nranks + 1] slots: gathered, then the local one
    uint64_t* local = d + (size_t)comm->nranks * kSlotWords;
    HIPCHK(hipMemcpyAsync(local, mine, kSlotWords * 8, hipMemcpyHostToDevice, comm->stream));
    NCCLCHK(comm->r->AllGather(local, d, kSlotWords * 8, ncclUint8, comm->comm, comm->stream));
    HIPCHK(hipMemcpyAsync(all, d, (size_t)comm->nranks * kSlotWords * 8, hipMemcpyDeviceToHost,
                          comm->stream));
    HIPCHK(hipStreamSynchronize(comm->stream));
    return true;
}
}  // namespace

extern "C" {

bool nxg_comm_unique_id(uint8_t id[128], NetidxError* err) {
    Rccl* r;
    if (!id || !rccl(&r, err)) {
        if (!id) set_err(err, "null argument");
        return false;
    }
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id is 128 bytes");
    ncclUniqueId u;
    const ncclResult_t e = r->GetUniqueId(&u);
    if (e != ncclSuccess) {
        set_err(err, "ncclGetUniqueId failed: %s", r->GetErrorString(e));
        return false;
    }
    memcpy(id, &u, 128);
    return true;
}

NxgComm* nxg_comm_init(NxgCtx* ctx, int nranks, int rank, const uint8_t id[128],
                       NetidxError* err) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks) {
        set_err(err, "bad argument (nranks %d, rank %d)", nranks, rank);
        return nullptr;
    }
    NxgComm* comm = new NxgComm();
    if (!rccl(&comm->r, err)) {
        delete comm;
        return nullptr;
    }
    comm->nranks = nranks;
    comm->rank = rank;
    comm->stream = (hipStream_t)nxg_ctx_stream(ctx);
    ncclUniqueId u;
    memcpy(&u, id, 128);
    ncclResult_t e = comm->r->CommInitRank(&comm->comm, nranks, u, rank);
    if (e != ncclSuccess) {
        set_err(err, "ncclCommInitRank failed: %s", comm->r->GetErrorString(e));
        delete comm;
        return nullptr;
    }
    if (hipMalloc(&comm->dscratch, (size_t)(nranks + 1) * kSlotWords * 8) != hipSuccess) {
        set_err(err, "hipMalloc of the exchange slots failed");
        comm->r->CommDestroy(comm->comm);
        delete comm;
        return nullptr;
    }
    return comm;
}

void nxg_comm_destroy(NxgComm* comm) {
    if (!comm) return;
    if (comm->stream) (void)hipStreamSynchronize(comm->stream);
    if (comm->comm) comm->r->CommDestroy(comm->comm);
    if (comm->dscratch) (void)hipFree(comm->dscratch);
    delete comm;
}

bool nxg_encode_allgather(NxgCtx* ctx, NxgComm* comm, const NxgColumns* din, const uint8_t* dheap,
                          uint8_t* dout, uint64_t cap, uint64_t* len_out, uint64_t* shard_off,
                          NetidxError* err) {
    if (!ctx || !comm || !din || !dout) {
        set_err(err, "null argument");
        return false;
    }
    comm->stream = (hipStream_t)nxg_ctx_stream(ctx);
    // 1. this shard's encoded size, then every shard's (8 bytes per rank)
    uint64_t mine[kSlotWords] = {0};
    if (!nxg_encoded_len(ctx, din, dheap, &mine[0], err)) return false;
    std::vector<uint64_t> all((size_t)comm->nranks * kSlotWords);
    if (!gather_slots(comm, mine, all.data(), err)) return false;
    std::vector<uint64_t> off(comm->nranks + 1, 0);
    for (int i = 0; i < comm->nranks; i++) off[i + 1] = off[i] + all[(size_t)i * kSlotWords];
    const uint64_t total = off[comm->nranks];
    if (total > cap) {
        set_err(err, "output buffer too small: the frame has %llu bytes, capacity %llu",
                (unsigned long long)total, (unsigned long long)cap);
        return false;
    }
    // 2. the shard straight into its final place
    const uint64_t my_off = off[comm->rank], my_len = mine[0];
    uint64_t wrote = 0;
    if (my_len &&
        !nxg_encode_updates(ctx, din, dheap, dout + my_off, cap - my_off, &wrote, err))
        return false;
    if (wrote != my_len) {
        set_err(err, "shard encoded to %llu bytes, sized at %llu", (unsigned long long)wrote,
                (unsigned long long)my_len);
        return false;
    }
    // 3. every shard to every rank, at the same offsets (grouped point-to-point over xGMI)
    NCCLCHK(comm->r->GroupStart());
    for (int p = 0; p < comm->nranks; p++) {
        if (p == comm->rank) continue;
        const uint64_t plen = off[p + 1] - off[p];
        if (my_len) NCCLCHK(comm->r->Send(dout + my_off, my_len, ncclUint8, p, comm->comm,
                                          comm->stream));
        if (plen) NCCLCHK(comm->r->Recv(dout + off[p], plen, ncclUint8, p, comm->comm,
                                        comm->stream));
    }
    NCCLCHK(comm->r->GroupEnd());
    HIPCHK(hipStreamSynchronize(comm->stream));
    if (len_out) *len_out = total;
    if (shard_off)
        for (int i = 0; i < comm->nranks; i++) shard_off[i] = off[i];
    return true;
}

bool nxg_decode_sharded(NxgCtx* ctx, NxgComm* comm, const uint8_t* dframe, uint64_t frame_len,
                        NxgColumns* dout, uint64_t* row_off, NxgRange* rng, NetidxError* err) {
    if (!ctx || !comm || !dout || (!dframe && frame_len)) {
        set_err(err, "null argument");
        return false;
    }
    comm->stream = (hipStream_t)nxg_ctx_stream(ctx);
    const int n = comm->nranks, r = comm->rank;
    const uint64_t b = frame_len * (uint64_t)r / (uint64_t)n;
    const uint64_t e = frame_len * (uint64_t)(r + 1) / (uint64_t)n;
    NxgRange mine;
    if (!nxg_decode_range(ctx, dframe, frame_len, b, e, dout, &mine, err)) return false;
    std::vector<NxgRange> all(n);
    std::vector<uint64_t> offs(n);
    std::vector<uint64_t> buf((size_t)n * kSlotWords);
    // link; a range whose entry is off the chain (a false record start guessed at its head)
    // decodes again from its predecessor's exit, which is a true start: at most n rounds
    for (int round = 0; round <= n; round++) {
        uint64_t slot[kSlotWords] = {0};
        memcpy(slot, &mine, sizeof mine);
        if (!gather_slots(comm, slot, buf.data(), err)) return false;
        for (int i = 0; i < n; i++) memcpy(&all[i], &buf[(size_t)i * kSlotWords], sizeof(NxgRange));
        for (int i = 0; i < n; i++)
            if (!all[i].ok) {
                set_err(err, "range %d is not a homogeneous-f64 range: decode the whole frame "
                             "with nxg_decode_updates", i);
                return false;
            }
        uint32_t bad = 0;
        NetidxError e2{nullptr};
        const bool linked = nxg_range_link(all.data(), (uint32_t)n, frame_len, offs.data(), &bad,
                                           &e2);
        nxg_error_free(&e2);
        if (linked) break;
        if (round == n) {
            set_err(err, "the byte ranges of the frame do not link into one chain");
            return false;
        }
        // the first broken range re-decodes from its predecessor's exit (every rank agrees on
        // `bad`: they all see the same summaries)
        if ((int)bad == r && r > 0) {
            uint64_t at = 0;  // the chain's position entering range r
            for (int i = 0; i < r; i++)
                if (all[i].begin != all[i].end) at = all[i].exit;
            if (at < b || at > frame_len) {
                set_err(err, "range %d: predecessor exit %llu outside the range", r,
                        (unsigned long long)at);
                return false;
            }
            NxgRange again;
            if (!nxg_decode_range(ctx, dframe, frame_len, at < e ? at : e, e, dout, &again, err))
                return false;
            again.begin = b;  // the same range, now entered on the chain
            if (at >= e) {    // no message starts in the range: the chain passes through
                again.entry = again.exit = at;
                again.n_rows = 0;
            }
            mine = again;
        } else if ((int)bad == r && r == 0) {
            set_err(err, "the frame does not start with a message");
            return false;
        }
    }
    if (row_off) *row_off = offs[r];
    if (rng) *rng = mine;
    return true;
}

}  // extern "C"
