// nxg_multi.cpp -- multi-GPU calls of the C ABI (include/nxg_codec.h): an RCCL communicator over
// xGMI, the sharded encode of BASELINE configs[4] (shards encoded into their final offsets, then
// grouped send/recv: SURVEY.md H5) and the byte-range sharded decode.
//
// The protocols are written once against a transport (RCCL, or a caller's NxgCommOps) and a
// local codec (the ctx's kernels, or the ops' hooks), so the code that runs on an 8-GPU node is
// the code the multi-process tests run. Every collective step carries each rank's status word:
// a rank that fails tells the others in the next exchange and they all return false at the same
// step (a rank that returned early would leave its peers waiting in a collective forever).
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
    Rccl* r = nullptr;  // RCCL transport, or
    bool use_ops = false;
    NxgCommOps ops{};   // the caller's transport (and codec)
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0;
    NxgCtx* ctx = nullptr;
    hipStream_t stream = nullptr;  // the ctx's stream at the last call
    uint64_t* dscratch = nullptr;  // RCCL: per-rank exchange slots (sizes, range summaries)
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
constexpr int kSlotWords = 8;  // one rank's exchange slot: 64 bytes
constexpr int kStatusWord = 7; // the slot's last word: 0 = this rank is fine, else failed
static_assert(sizeof(NxgRange) <= (kSlotWords - 1) * 8, "range summary fits a slot");

// ---- transport ------------------------------------------------------------------------------
// all-gather of one 64-byte slot per rank (host memory): mine -> all[0 .. nranks). A transport
// failure cannot be agreed on (the transport is what broke): it is returned as is.
bool gather_slots(NxgComm* comm, const uint64_t* mine, uint64_t* all, NetidxError* err) {
    if (comm->use_ops) {
        if (!comm->ops.allgather(comm->ops.user, mine, all, kSlotWords * 8)) {
            set_err(err, "rank %d: the transport's all-gather failed", comm->rank);
            return false;
        }
        return true;
    }
    uint64_t* d = comm->dscratch;  // [nranks + 1] slots: gathered, then the local one
    uint64_t* local = d + (size_t)comm->nranks * kSlotWords;
    HIPCHK(hipMemcpyAsync(local, mine, kSlotWords * 8, hipMemcpyHostToDevice, comm->stream));
    NCCLCHK(comm->r->AllGather(local, d, kSlotWords * 8, ncclUint8, comm->comm, comm->stream));
    HIPCHK(hipMemcpyAsync(all, d, (size_t)comm->nranks * kSlotWords * 8, hipMemcpyDeviceToHost,
                          comm->stream));
    HIPCHK(hipStreamSynchronize(comm->stream));
    return true;
}

// every shard [off[p], off[p+1]) of `buf` to every rank, at the same offsets
bool exchange_shards(NxgComm* comm, uint8_t* buf, const std::vector<uint64_t>& off,
                     NetidxError* err) {
    if (comm->use_ops) {
        if (!comm->ops.allgatherv(comm->ops.user, buf, off.data(), (uint32_t)comm->nranks,
                                  (uint32_t)comm->rank)) {
            set_err(err, "rank %d: the transport's shard exchange failed", comm->rank);
            return false;
        }
        return true;
    }
    // grouped point-to-point over xGMI: no padding to the largest shard, no compaction
    const uint64_t my_off = off[comm->rank], my_len = off[comm->rank + 1] - my_off;
    NCCLCHK(comm->r->GroupStart());
    for (int p = 0; p < comm->nranks; p++) {
        if (p == comm->rank) continue;
        const uint64_t plen = off[p + 1] - off[p];
        if (my_len) NCCLCHK(comm->r->Send(buf + my_off, my_len, ncclUint8, p, comm->comm,
                                          comm->stream));
        if (plen) NCCLCHK(comm->r->Recv(buf + off[p], plen, ncclUint8, p, comm->comm,
                                        comm->stream));
    }
    NCCLCHK(comm->r->GroupEnd());
    HIPCHK(hipStreamSynchronize(comm->stream));
    return true;
}

// ---- local codec ----------------------------------------------------------------------------
bool has_codec_hooks(const NxgComm* comm) { return comm->use_ops && comm->ops.decode_range; }

bool local_encoded_len(NxgComm* comm, const NxgColumns* in, const uint8_t* heap, uint64_t* len,
                       NetidxError* err) {
    if (has_codec_hooks(comm)) {
        if (!comm->ops.encoded_len(comm->ops.user, in, heap, len)) {
            set_err(err, "rank %d: encoded_len failed", comm->rank);
            return false;
        }
        return true;
    }
    return nxg_encoded_len(comm->ctx, in, heap, len, err);
}
bool local_encode(NxgComm* comm, const NxgColumns* in, const uint8_t* heap, uint8_t* out,
                  uint64_t cap, uint64_t* len, NetidxError* err) {
    if (has_codec_hooks(comm)) {
        if (!comm->ops.encode(comm->ops.user, in, heap, out, cap, len)) {
            set_err(err, "rank %d: encode failed", comm->rank);
            return false;
        }
        return true;
    }
    return nxg_encode_updates(comm->ctx, in, heap, out, cap, len, err);
}
bool local_decode_range(NxgComm* comm, const uint8_t* f, uint64_t W, uint64_t b, uint64_t e,
                        NxgColumns* out, NxgRange* rng, NetidxError* err) {
    if (has_codec_hooks(comm)) {
        if (!comm->ops.decode_range(comm->ops.user, f, W, b, e, out, rng)) {
            set_err(err, "rank %d: decode_range failed", comm->rank);
            return false;
        }
        return true;
    }
    return nxg_decode_range(comm->ctx, f, W, b, e, out, rng, err);
}

bool local_decode_share(NxgComm* comm, const uint8_t* f, uint64_t W, NxgColumns* out,
                        uint64_t* row_off, NxgStatus* st, NetidxError* err) {
    if (has_codec_hooks(comm)) {
        if (!comm->ops.decode_share) {
            set_err(err, "rank %d: a byte range was declined and the ops carry no decode_share",
                    comm->rank);
            return false;
        }
        if (!comm->ops.decode_share(comm->ops.user, f, W, (uint32_t)comm->rank,
                                    (uint32_t)comm->nranks, out, row_off, st)) {
            set_err(err, "rank %d: decode_share failed", comm->rank);
            return false;
        }
        return true;
    }
    return nxg_decode_share(comm->ctx, f, W, (uint32_t)comm->rank, (uint32_t)comm->nranks, out,
                            row_off, st, err);
}

// After a gather: the first rank whose status word is set, or -1.
int first_failed(const NxgComm* comm, const std::vector<uint64_t>& all) {
    for (int i = 0; i < comm->nranks; i++)
        if (all[(size_t)i * kSlotWords + kStatusWord]) return i;
    return -1;
}
// The agreed failure: this rank keeps its own message if it is the one that failed.
bool fail_together(NxgComm* comm, int who, const char* what, NetidxError* err) {
    if (who != comm->rank || !err || !err->msg) set_err(err, "rank %d failed %s", who, what);
    return false;
}

bool comm_ready(NxgCtx* ctx, NxgComm* comm, NetidxError* err) {
    if (!comm || (!ctx && !has_codec_hooks(comm))) {
        set_err(err, "null argument");
        return false;
    }
    if (ctx) comm->ctx = ctx;
    comm->stream = ctx ? (hipStream_t)nxg_ctx_stream(ctx) : nullptr;
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
    comm->ctx = ctx;
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

NxgComm* nxg_comm_init_ops(NxgCtx* ctx, int nranks, int rank, const NxgCommOps* ops,
                           NetidxError* err) {
    if (!ops || !ops->allgather || !ops->allgatherv || nranks < 1 || rank < 0 || rank >= nranks) {
        set_err(err, "bad argument (nranks %d, rank %d, ops %p)", nranks, rank, (const void*)ops);
        return nullptr;
    }
    const int hooks = !!ops->encoded_len + !!ops->encode + !!ops->decode_range;
    if (hooks != 0 && hooks != 3) {
        set_err(err, "the local codec hooks come all three or none");
        return nullptr;
    }
    if (!ctx && hooks == 0) {
        set_err(err, "a ctx is needed unless the ops carry the local codec");
        return nullptr;
    }
    NxgComm* comm = new NxgComm();
    comm->use_ops = true;
    comm->ops = *ops;
    comm->nranks = nranks;
    comm->rank = rank;
    comm->ctx = ctx;
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
    if (!comm_ready(ctx, comm, err)) return false;
    const int n = comm->nranks;
    std::vector<uint64_t> all((size_t)n * kSlotWords);
    // 1. every shard's encoded size (and whether it could be sized)
    uint64_t mine[kSlotWords] = {0};
    if (!din || !dout) {
        set_err(err, "null argument");
        mine[kStatusWord] = 1;
    } else if (!local_encoded_len(comm, din, dheap, &mine[0], err)) {
        mine[kStatusWord] = 1;
    }
    if (!gather_slots(comm, mine, all.data(), err)) return false;
    int bad = first_failed(comm, all);
    if (bad >= 0) return fail_together(comm, bad, "to size its shard", err);
    std::vector<uint64_t> off(n + 1, 0);
    for (int i = 0; i < n; i++) off[i + 1] = off[i] + all[(size_t)i * kSlotWords];
    const uint64_t total = off[n];
    // 2. the shard straight into its final place; then agree that every rank managed
    const uint64_t my_off = off[comm->rank], my_len = mine[0];
    uint64_t st[kSlotWords] = {0};
    if (total > cap) {
        set_err(err, "output buffer too small: the frame has %llu bytes, capacity %llu",
                (unsigned long long)total, (unsigned long long)cap);
        st[kStatusWord] = 1;
    } else if (my_len) {
        uint64_t wrote = 0;
        if (!local_encode(comm, din, dheap, dout + my_off, cap - my_off, &wrote, err)) {
            st[kStatusWord] = 1;
        } else if (wrote != my_len) {
            set_err(err, "shard encoded to %llu bytes, sized at %llu", (unsigned long long)wrote,
                    (unsigned long long)my_len);
            st[kStatusWord] = 1;
        }
    }
    if (!gather_slots(comm, st, all.data(), err)) return false;
    bad = first_failed(comm, all);
    if (bad >= 0) return fail_together(comm, bad, "to encode its shard", err);
    // 3. every shard to every rank, at the same offsets
    if (!exchange_shards(comm, dout, off, err)) return false;
    if (len_out) *len_out = total;
    if (shard_off)
        for (int i = 0; i < n; i++) shard_off[i] = off[i];
    return true;
}

// nxg_decode_sharded's fallback: rank r keeps row share r of the whole frame's decode; the ranks
// agree on any local failure in one more exchange. Every rank decodes the same frame with the
// same decoders, so the frame's error (if any) is the same on every rank.
static bool share_fallback(NxgComm* comm, const uint8_t* dframe, uint64_t W, uint64_t b,
                           uint64_t e, NxgColumns* dout, uint64_t* row_off, NxgRange* rng,
                           NetidxError* err) {
    NxgStatus s{};
    uint64_t off = 0;
    uint64_t slot[kSlotWords] = {0};
    if (!local_decode_share(comm, dframe, W, dout, &off, &s, err)) {
        slot[kStatusWord] = 1;
    } else if (s.err_kind == NXG_CAPACITY || s.err_kind == NXG_NOT_F64) {
        // this rank's share does not fit its columns: a local failure, agreed by every rank (the
        // frame's own errors are the same on every rank and stay in rng)
        set_err(err, "rank %d: its row share does not fit its columns (%s)", comm->rank,
                s.err_kind == NXG_CAPACITY ? "capacity" : "f64-only columns for mixed rows");
        slot[kStatusWord] = 1;
    }
    std::vector<uint64_t> buf((size_t)comm->nranks * kSlotWords);
    if (!gather_slots(comm, slot, buf.data(), err)) return false;
    const int who = first_failed(comm, buf);
    if (who >= 0) return fail_together(comm, who, "to decode its row share", err);
    if (row_off) *row_off = off;
    if (rng) {
        NxgRange m{};
        m.begin = b;
        m.end = e;
        m.entry = m.exit = ~0ull;
        m.n_rows = s.n_rows;
        m.ok = 2;
        m.err_kind = (uint32_t)s.err_kind;
        m.err_offset = s.err_offset;
        *rng = m;
    }
    return true;
}

bool nxg_decode_sharded(NxgCtx* ctx, NxgComm* comm, const uint8_t* dframe, uint64_t frame_len,
                        NxgColumns* dout, uint64_t* row_off, NxgRange* rng, NetidxError* err) {
    if (!comm_ready(ctx, comm, err)) return false;
    const int n = comm->nranks, r = comm->rank;
    const uint64_t b = frame_len * (uint64_t)r / (uint64_t)n;
    const uint64_t e = frame_len * (uint64_t)(r + 1) / (uint64_t)n;
    NxgRange mine{};
    bool failed = false;
    if (!dout || (!dframe && frame_len)) {
        set_err(err, "null argument");
        failed = true;
    } else if (!local_decode_range(comm, dframe, frame_len, b, e, dout, &mine, err)) {
        failed = true;
    }
    std::vector<NxgRange> all(n);
    std::vector<uint64_t> offs(n);
    std::vector<uint64_t> buf((size_t)n * kSlotWords);
    // link; a range whose entry is off the chain (a false record start guessed at its head)
    // decodes again from its predecessor's exit, which is a true start: at most n rounds. Every
    // rank sees the same summaries, so every decision below is the same on every rank.
    for (int round = 0;; round++) {
        uint64_t slot[kSlotWords] = {0};
        memcpy(slot, &mine, sizeof mine);
        slot[kStatusWord] = failed ? 1 : 0;
        if (!gather_slots(comm, slot, buf.data(), err)) return false;
        const int who = first_failed(comm, buf);
        if (who >= 0) return fail_together(comm, who, "to decode its byte range", err);
        for (int i = 0; i < n; i++) memcpy(&all[i], &buf[(size_t)i * kSlotWords], sizeof(NxgRange));
        int declined = -1;
        for (int i = 0; i < n; i++) {
            if (all[i].ok) continue;
            if (all[i].err_kind == NXG_CAPACITY) {
                set_err(err, "range %d: the columns of rank %d are too small for its rows", i, i);
                return false;
            }
            if (declined < 0) declined = i;
        }
        // content the byte-range decoders do not take: every rank saw it in this exchange, so
        // every rank takes the row-share fallback (the frame decoded whole, rows in shares)
        if (declined >= 0) return share_fallback(comm, dframe, frame_len, b, e, dout, row_off, rng,
                                                 err);
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
        if (bad == 0) {
            set_err(err, "the frame does not start with a message");
            return false;
        }
        // the first broken range re-decodes from its predecessor's exit
        if ((int)bad == r) {
            uint64_t at = 0;  // the chain's position entering range r
            for (int i = 0; i < r; i++)
                if (all[i].begin != all[i].end) at = all[i].exit;
            if (at < b || at > frame_len) {
                set_err(err, "range %d: predecessor exit %llu outside the range", r,
                        (unsigned long long)at);
                failed = true;
                continue;
            }
            NxgRange again{};
            if (!local_decode_range(comm, dframe, frame_len, at < e ? at : e, e, dout, &again,
                                    err)) {
                failed = true;
                continue;
            }
            again.begin = b;  // the same range, now entered on the chain
            if (at >= e) {    // no message starts in the range: the chain passes through
                again.entry = again.exit = at;
                again.n_rows = 0;
            }
            mine = again;
        }
    }
    if (row_off) *row_off = offs[r];
    if (rng) *rng = mine;
    return true;
}

}  // extern "C"
