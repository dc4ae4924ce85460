// nxg_api.cpp -- the C ABI (include/nxg_codec.h): contexts, column allocation, dispatch of the
// gfx950 kernels, host staging for host-resident frames/columns, and host framing.
//
// Error convention follows netidx-ffi (netidx-ffi/src/error.rs:19-29): fallible calls return
// bool and fill NetidxError.msg with a heap string released by nxg_error_free.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/nxg_codec.h"
#include "nxg_internal.h"

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

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            set_err(err, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__,  \
                    __LINE__);                                                             \
            return false;                                                                  \
        }                                                                                  \
    } while (0)

constexpr int kStatusRing = 1024;  // at most kStatusRing/2 async calls in flight

}  // namespace

thread_local uint32_t nxg_patience = 128;  // the calling ctx's, set by begin_call
thread_local DevStatus* nxg_zero_slot = nullptr;
thread_local bool nxg_zero_used = false;

struct NxgCtx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    int ncu = 0;
    int grid_enc_f64 = 0, grid_enc_gen = 0;
    // status ring: one DevStatus per call, the whole ring re-zeroed once per lap
    DevStatus* dst = nullptr;
    DevStatus* hst = nullptr;  // pinned mirror
    uint32_t calls = 0;
    uint32_t epoch = 0;
    uint64_t* tstat = nullptr;
    size_t tstat_words = 0;
    uint32_t* glws = nullptr;      // general decode: lane words, 256 B per tile
    size_t glws_cap = 0;
    uint64_t* gruns = nullptr;     // general decode: run summaries + bases
    bool no_fa = false;            // NXG_ARCH_PATH=exact: archive batches on the exact decoder only
    uint8_t* dscratch = nullptr;   // dispatch: counters, offsets, block sums, unmatched count
    size_t dscratch_cap = 0;
    int wgs_dec_gen = 0;
    // f64 decoder choice: the length-run decoder (nxg_decode_f64_run.hip) unless the frames of
    // this connection have record lengths that vary record to record; then the single-pass
    // decoder of any f64 frame (nxg_decode_f64_x.hip) for the next kIrregularCalls calls
    // (NXG_F64_PATH=x forces it)
    uint8_t* rdesc = nullptr;  // length-run decoder: 16-byte tile descriptors
    size_t rdesc_cap = 0;
    uint32_t irregular_left = 0;
    bool force_x = false;
    // before both: the one-launch decoder of frames whose ids count up by one
    // (nxg_decode_f64_seq.hip), unless it rejected a recent frame of this connection: then it is
    // skipped for the next kSeqSkipCalls calls (NXG_F64_PATH=run skips it always)
    uint32_t seq_left = 0;
    bool no_seq = false;
    // the sequential-id f64 encoder (nxg_encode_f64_seq.hip): after it declines a batch (ids not
    // counting up by one) it is skipped for the next kSeqSkipCalls f64 encodes; NXG_F64_ENC=tile
    // skips it always
    uint8_t* pscratch = nullptr;  // the type-partitioned view's counts and offsets
    size_t pscratch_cap = 0;
    uint32_t enc_seq_left = 0;
    uint32_t last_enc_kernel = 0;  // the last f64 encode: 1 sequential-id kernel, 2 tiled (debug)
    bool no_enc_seq = false;
    // mixed decode: the fast decoder (nxg_decode_mixed.hip) unless it rejected a recent frame of
    // this connection; then the general decoder for the next kMixFailCalls calls
    // (NXG_MIXED_PATH=general: always the general decoder)
    uint32_t mix_left = 0;
    bool no_fmx = false;
    // the fast mixed decoder's count pass: lean (one-byte-prefix Update candidates only, then the
    // tiles where that found no chain recounted from every kind) while this connection's last
    // decoded frame had at most 1 tile in 32 holding a Heartbeat or a two-byte prefix
    // (DevStatus.diag[0], from the resolve pass), else every candidate kind (NXG_FMX_COUNT=full
    // always, =lean always)
    bool fmx_full = false;
    int fmx_count_mode = 0;  // 0 adaptive, 1 full, 2 lean
    int wgs_fmx[2] = {0, 0};
    uint32_t f64r_flags = 0;  // NXG_F64R_FLAGS (tests): 1 every tile exact, 2 never hand over
    uint32_t patience = 128;  // NXG_LOOKBACK_PATIENCE: look-back polls before self-help
    uint8_t* dframe = nullptr;
    size_t dframe_cap = 0;
    uint64_t* escratch = nullptr;
    size_t escratch_words = 0;
    NxgColumns dcols{};  // device staging columns for host-resident outputs/inputs
    bool dcols_valid = false;
    uint8_t* dheap = nullptr;
    size_t dheap_cap = 0;
    // in-flight async operations (completed in order by nxg_ctx_sync)
    struct Pending {
        int kind;  // 1 decode, 2 encode
        int fast;
        const uint8_t* frame;
        uint64_t len;
        NxgColumns* cols;
        uint64_t* len_out;
        uint64_t cap;  // encode: the output capacity
        DevStatus* st;
        uint32_t slot;
        uint32_t flags = 0;            // decode: the caller's NXG_DECODE_* flags
        const uint8_t* heap = nullptr;  // encode: the heap and the output buffer
        uint8_t* out = nullptr;
    };
    std::vector<Pending> pending;
    // zstd (compressed archive records): predefined tables, literal buffers, descriptors
    void* zdefs = nullptr;
    uint8_t* zlit = nullptr;
    int zgrid = 0;
    void* zrecs = nullptr;
    size_t zrecs_cap = 0;
    DevStatus last{};  // last completed decode's device status (diagnostics)
    uint64_t fa_last[8] = {};  // the last fast archive attempt's FaHead (diagnostics)
    uint64_t last_split = 0;  // last completed encode's DevStatus.split_start
};

namespace {

bool set_device(NxgCtx* c, NetidxError* err) {
    HIPCHK(hipSetDevice(c->device));
    return true;
}

// Next status slot + epoch for one call. Slot k is zeroed by the call that used slot
// k - kStatusRing/2 (nxg_zero_slot: block 0 of its kernel, or end_call when it launched none), so
// at most kStatusRing/2 calls may be in flight. Every begin_call is paired with an end_call.
bool begin_call(NxgCtx* c, DevStatus** st, uint32_t* slot, NetidxError* err) {
    *slot = c->calls % kStatusRing;
    *st = c->dst + *slot;
    nxg_patience = c->patience;
    nxg_zero_slot = c->dst + (c->calls + kStatusRing / 2) % kStatusRing;
    nxg_zero_used = false;
    c->calls++;
    c->epoch++;
    if (c->epoch > kEpochMax) {  // wrap: stale words could alias epoch 1 again
        c->epoch = 1;
        if (c->tstat) HIPCHK(hipMemsetAsync(c->tstat, 0, c->tstat_words * 8, c->stream));
    }
    return true;
}

// After a call's launches (or a failure to launch): if no kernel took the zero-ahead slot (an
// empty frame or batch launches nothing), clear it here, so that the call kStatusRing/2 later
// does not inherit this ring lap's status bits.
bool end_call(NxgCtx* c, NetidxError* err) {
    if (nxg_zero_used) return true;
    nxg_zero_used = true;
    HIPCHK(hipMemsetAsync(nxg_zero_slot, 0, sizeof(DevStatus), c->stream));
    return true;
}

bool ensure_tstat(NxgCtx* c, size_t words, NetidxError* err) {
    if (words <= c->tstat_words) return true;
    size_t n = std::max(words, c->tstat_words * 2);
    n = std::max<size_t>(n, 4096);
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->tstat) HIPCHK(hipFree(c->tstat));
    c->tstat = nullptr;
    HIPCHK(hipMalloc(&c->tstat, n * 8));
    HIPCHK(hipMemsetAsync(c->tstat, 0, n * 8, c->stream));
    c->tstat_words = n;
    return true;
}

bool ensure_escratch(NxgCtx* c, size_t words, NetidxError* err) {
    if (words <= c->escratch_words) return true;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->escratch) HIPCHK(hipFree(c->escratch));
    c->escratch = nullptr;
    size_t n = std::max<size_t>(words, 1024);
    HIPCHK(hipMalloc(&c->escratch, n * 8));
    c->escratch_words = n;
    return true;
}

bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

ColsDesc desc_of(const NxgColumns* c) {
    ColsDesc d{};
    d.cap_rows = c->cap_rows;
    d.cap_children = c->cap_children;
    d.cap_ctl = c->cap_ctl;
    d.n_rows = c->n_rows;
    d.n_children = c->n_children;
    d.n_ctl = c->n_ctl;
    d.id = c->id;
    d.tag = c->tag;
    d.fixed = c->fixed;
    d.aux = c->aux;
    d.ctag = c->ctag;
    d.cfixed = c->cfixed;
    d.caux = c->caux;
    d.ctl_row = c->ctl_row;
    d.ctl_off = c->ctl_off;
    d.ctl_len = c->ctl_len;
    d.ctl_variant = c->ctl_variant;
    return d;
}

bool cols_alloc_impl(uint32_t layout, uint64_t cr, uint64_t cc, uint64_t ck, uint32_t mem,
                     NxgColumns* o, NetidxError* err) {
    memset(o, 0, sizeof *o);
    o->layout = layout;
    o->mem = mem;
    o->cap_rows = cr;
    o->cap_children = cc;
    o->cap_ctl = ck;
    auto alloc = [&](void** p, size_t bytes) -> bool {
        bytes = std::max<size_t>(bytes, 16);
        hipError_t e = mem == NXG_MEM_DEVICE ? hipMalloc(p, bytes)
                                             : hipHostMalloc(p, bytes, hipHostMallocDefault);
        if (e != hipSuccess) {
            set_err(err, "column allocation of %zu bytes failed: %s", bytes, hipGetErrorString(e));
            return false;
        }
        return true;
    };
    if (!alloc((void**)&o->id, cr * 8) || !alloc((void**)&o->fixed, cr * 8)) return false;
    if (layout == NXG_LAYOUT_MIXED) {
        if (!alloc((void**)&o->tag, cr) || !alloc((void**)&o->aux, cr * 4) ||
            !alloc((void**)&o->ctag, cc) || !alloc((void**)&o->cfixed, cc * 8) ||
            !alloc((void**)&o->caux, cc * 4) || !alloc((void**)&o->ctl_row, ck * 8) ||
            !alloc((void**)&o->ctl_off, ck * 8) || !alloc((void**)&o->ctl_len, ck * 4) ||
            !alloc((void**)&o->ctl_variant, ck))
            return false;
    }
    return true;
}

void cols_free_impl(NxgColumns* c) {
    void* ps[] = {c->id, c->tag, c->fixed, c->aux, c->ctag, c->cfixed, c->caux,
                  c->ctl_row, c->ctl_off, c->ctl_len, c->ctl_variant};
    for (void* p : ps) {
        if (!p) continue;
        if (c->mem == NXG_MEM_DEVICE) (void)hipFree(p);
        else (void)hipHostFree(p);
    }
    memset(c, 0, sizeof *c);
}

// device staging columns shaped like `like` (grown on demand)
bool mixed_capable(const NxgColumns* c) {
    return c->tag && c->aux && c->ctag && c->cfixed && c->caux && c->ctl_row && c->ctl_off &&
           c->ctl_len && c->ctl_variant;
}

bool ensure_dcols(NxgCtx* c, const NxgColumns* like, NetidxError* err) {
    const bool mixed = mixed_capable(like);
    if (c->dcols_valid && c->dcols.cap_rows >= like->cap_rows &&
        c->dcols.cap_children >= like->cap_children && c->dcols.cap_ctl >= like->cap_ctl &&
        (c->dcols.layout == NXG_LAYOUT_MIXED || !mixed))
        return true;
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->dcols_valid) cols_free_impl(&c->dcols);
    c->dcols_valid = false;
    if (!cols_alloc_impl(mixed ? NXG_LAYOUT_MIXED : NXG_LAYOUT_F64, like->cap_rows,
                         like->cap_children, like->cap_ctl, NXG_MEM_DEVICE, &c->dcols, err))
        return false;
    c->dcols_valid = true;
    return true;
}

// view of the device staging columns restricted to `like`'s layout and capacities
NxgColumns staged_view(NxgCtx* c, const NxgColumns* like) {
    NxgColumns v = c->dcols;
    v.layout = like->layout;
    v.cap_rows = like->cap_rows;
    v.cap_children = like->cap_children;
    v.cap_ctl = like->cap_ctl;
    if (!mixed_capable(like)) {
        v.tag = nullptr;
        v.aux = nullptr;
        v.ctag = nullptr;
        v.cfixed = nullptr;
        v.caux = nullptr;
        v.ctl_row = nullptr;
        v.ctl_off = nullptr;
        v.ctl_len = nullptr;
        v.ctl_variant = nullptr;
    }
    return v;
}

constexpr uint32_t kIrregularCalls = 64;
constexpr uint32_t kMixFailCalls = 16;
constexpr uint32_t kSeqSkipCalls = 64;

// path codes of a fast attempt (Pending::fast): homogeneous f64 (SEQ, RUN, X) or mixed (MIX)
enum { FAST_NONE = 0, FAST_RUN = 1, FAST_X = 2, FAST_MIX = 3, FAST_SEQ = 4 };

bool seq_active(const NxgCtx* c) {
    return !c->no_seq && !c->force_x && c->seq_left == 0 && c->irregular_left == 0;
}

bool ensure_rdesc(NxgCtx* c, size_t bytes, NetidxError* err) {
    if (bytes <= c->rdesc_cap) return true;
    size_t n = std::max(bytes, c->rdesc_cap * 2);
    n = std::max<size_t>(n, 1 << 16);
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->rdesc) HIPCHK(hipFree(c->rdesc));
    c->rdesc = nullptr;
    HIPCHK(hipMalloc(&c->rdesc, n));
    c->rdesc_cap = n;
    return true;
}

// the single-pass decoder of any f64 frame
bool enqueue_dec_x(NxgCtx* c, const uint8_t* f, uint64_t len, NxgColumns* out, DevStatus* st,
                   NetidxError* err) {
    if (!ensure_tstat(c, nxg_dec_f64x_groups(len), err)) return false;
    HIPCHK(nxg_launch_dec_f64x(f, len, out->id, out->fixed, out->cap_rows, c->tstat, c->epoch, st,
                               c->stream));
    return true;
}

// Homogeneous-f64 attempt; *path receives the FAST_* code of the decoder that was enqueued.
// try_seq: the sequential-id decoder may be tried first (not on a rerun after it declined).
bool enqueue_dec_fast(NxgCtx* c, const uint8_t* f, uint64_t len, NxgColumns* out, DevStatus* st,
                      int* path, NetidxError* err, bool try_seq = true) {
    if (try_seq && len > 0 && seq_active(c)) {
        *path = FAST_SEQ;
        HIPCHK(nxg_launch_dec_f64s(f, len, out->id, out->fixed, out->cap_rows, st,
                                   nxg_take_zero_slot(), c->stream));
        return true;
    }
    // (a rerun right after the sequential-id decoder declined does not count: the skip lasts
    // kSeqSkipCalls calls after the one that declined)
    if (try_seq && c->seq_left) c->seq_left--;
    if (!c->force_x && c->irregular_left == 0) {
        *path = FAST_RUN;
        if (!ensure_tstat(c, nxg_dec_f64r_groups(len), err)) return false;
        if (!ensure_rdesc(c, 16 * nxg_dec_f64r_tiles(len), err)) return false;
        HIPCHK(nxg_launch_dec_f64r(f, len, 0, len, out->id, out->fixed, out->cap_rows, c->rdesc,
                                   c->tstat, c->epoch, c->f64r_flags, st, c->stream));
        return true;
    }
    if (c->irregular_left) c->irregular_left--;
    *path = FAST_X;
    return enqueue_dec_x(c, f, len, out, st, err);
}

bool ensure_glws(NxgCtx* c, size_t bytes, NetidxError* err) {
    if (bytes <= c->glws_cap) return true;
    size_t n = std::max(bytes, c->glws_cap * 2);
    n = std::max<size_t>(n, 1 << 16);
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->glws) HIPCHK(hipFree(c->glws));
    c->glws = nullptr;
    HIPCHK(hipMalloc(&c->glws, n));
    c->glws_cap = n;
    return true;
}

bool enqueue_dec_general(NxgCtx* c, const uint8_t* f, uint64_t len, NxgColumns* out,
                         DevStatus* st, NetidxError* err) {
    if (!ensure_glws(c, nxg_dec_gen_scratch_bytes(len), err)) return false;
    const ColsDesc d = desc_of(out);
    HIPCHK(nxg_launch_dec_gen(f, len, d, c->glws, c->gruns,
                              c->gruns + (size_t)gdec2::MAX_RUNS * gdec2::RUN_WORDS,
                              c->wgs_dec_gen, st, c->stream));
    return true;
}

// Mixed decode: the fast decoder for frames of short Update messages (it raises fast_fail on
// anything else and finish_decode reruns the frame on the general decoder).
bool enqueue_dec_mixed(NxgCtx* c, const uint8_t* f, uint64_t len, NxgColumns* out, DevStatus* st,
                       int* path, NetidxError* err) {
    const ColsDesc d = desc_of(out);
    // (frames of 4 GiB or more: the general decoder; the fast path keeps per-tile counts in 32 bits)
    if (len > 0 && len < (1ull << 32) && d.tag && d.ctag && !c->no_fmx && c->mix_left == 0) {
        *path = FAST_MIX;
        // one buffer for both, so that a fallback does not reallocate
        const uint64_t need = std::max(nxg_fmx_scratch_bytes(len), nxg_dec_gen_scratch_bytes(len));
        if (!ensure_glws(c, need, err)) return false;
        const bool lean = c->fmx_count_mode == 2 || (c->fmx_count_mode == 0 && !c->fmx_full);
        HIPCHK(nxg_launch_dec_fmx(f, len, d, reinterpret_cast<uint8_t*>(c->glws), c->wgs_fmx, st,
                                  c->stream, lean));
        return true;
    }
    if (c->mix_left) c->mix_left--;
    *path = FAST_NONE;
    return enqueue_dec_general(c, f, len, out, st, err);
}

// finish a device decode: read status, fall back to the general kernel if the f64 kernel
// rejected the frame, fill the user-visible status
// `fetched`: the caller has already copied the status ring to c->hst after the stream drained.
// `redone` (optional) is set when a fallback decoder rewrote the columns here, i.e. after every
// call enqueued behind this one had already run.
bool finish_decode(NxgCtx* c, const uint8_t* f, uint64_t len, NxgColumns* out, int tried_fast,
                   DevStatus* st, uint32_t slot, NxgStatus* ust, NetidxError* err,
                   bool fetched = false, bool* redone = nullptr) {
    if (redone) *redone = false;
    if (!fetched) {
        HIPCHK(hipMemcpyAsync(c->hst + slot, st, sizeof(DevStatus), hipMemcpyDeviceToHost,
                              c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    DevStatus h = c->hst[slot];
    if (tried_fast == FAST_SEQ && len > 0 && h.fast_fail) {
        if (h.irregular & 2u) {
            // not an f64 frame at all: on to the mixed decoders (as after the length-run probe)
            tried_fast = FAST_RUN;
        } else {
            // an f64 frame whose ids do not count up by one: the length-run (or single-pass)
            // decoder, and this one skipped for the next kSeqSkipCalls calls
            c->seq_left = kSeqSkipCalls;
            DevStatus* st2;
            uint32_t slot2;
            if (!begin_call(c, &st2, &slot2, err)) return false;
            const bool ok = enqueue_dec_fast(c, f, len, out, st2, &tried_fast, err, false);
            if (!end_call(c, err) || !ok) return false;
            if (redone) *redone = true;
            HIPCHK(hipMemcpyAsync(c->hst + slot2, st2, sizeof(DevStatus), hipMemcpyDeviceToHost,
                                  c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            h = c->hst[slot2];
        }
    }
    // (irregular bit 1: not an f64 frame at all -- straight on to the mixed decoders)
    if (tried_fast == FAST_RUN && len > 0 && h.fast_fail && (h.irregular & 3u) == 1u) {
        // record lengths vary record to record: the single-pass decoder of any f64 frame, for
        // this frame and the next kIrregularCalls ones
        c->irregular_left = kIrregularCalls;
        DevStatus* st2;
        uint32_t slot2;
        if (!begin_call(c, &st2, &slot2, err)) return false;
        const bool ok = enqueue_dec_x(c, f, len, out, st2, err);
        if (!end_call(c, err) || !ok) return false;
        if (redone) *redone = true;
        HIPCHK(hipMemcpyAsync(c->hst + slot2, st2, sizeof(DevStatus), hipMemcpyDeviceToHost,
                              c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        h = c->hst[slot2];
    }
    // a rejected frame: after the f64 decoders the mixed fast path (mixed columns), after that
    // the general decoder
    while (tried_fast && len > 0 && h.fast_fail) {
        if (tried_fast == FAST_MIX) {
            c->mix_left = kMixFailCalls;
            c->fmx_full = true;  // its next attempt with every candidate kind
        }
        DevStatus* st2;
        uint32_t slot2;
        if (!begin_call(c, &st2, &slot2, err)) return false;
        int next = FAST_NONE;
        const bool ok = tried_fast == FAST_MIX
                            ? enqueue_dec_general(c, f, len, out, st2, err)
                            : enqueue_dec_mixed(c, f, len, out, st2, &next, err);
        if (!end_call(c, err) || !ok) return false;
        if (redone) *redone = true;
        HIPCHK(hipMemcpyAsync(c->hst + slot2, st2, sizeof(DevStatus), hipMemcpyDeviceToHost,
                              c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        h = c->hst[slot2];
        tried_fast = next;
    }
    // the next fast mixed decode's count pass from this frame's mix of tiles
    if (h.path == 4 && len > 0) c->fmx_full = h.diag[0] * 32 > (len + 4095) / 4096;
    if (h.err_key) {  // general decode: the earliest (offset, kind) on the true chain
        h.err_kind = (uint32_t)(~h.err_key & 0xffu);
        h.err_offset = ~h.err_key >> 8;
    }
    c->last = h;
    if (h.timeout || h.err_kind == NXG_TIMEOUT) {
        set_err(err, "device look-back watchdog expired");
        return false;
    }
    NxgStatus s{};
    s.n_rows = h.n_rows;
    s.n_children = h.n_children;
    s.n_ctl = h.n_ctl;
    s.n_heartbeat = h.n_heartbeat;
    s.err_kind = (int32_t)h.err_kind;
    s.err_offset = h.err_offset;
    s.path = len == 0 ? 1 : h.path;
    if (!s.err_kind && h.capacity) s.err_kind = NXG_CAPACITY;
    if (!s.err_kind && !mixed_capable(out) && (h.nonf64 || s.n_ctl || s.n_children))
        s.err_kind = NXG_NOT_F64;
    if (ust) *ust = s;
    out->n_rows = s.n_rows;
    out->n_children = s.n_children;
    out->n_ctl = s.n_ctl;
    out->n_heartbeat = s.n_heartbeat;
    return true;
}

bool copy_cols_d2h(NxgCtx* c, const NxgColumns* d, NxgColumns* h, NetidxError* err) {
    const uint64_t nr = std::min(d->n_rows, h->cap_rows);
    HIPCHK(hipMemcpyAsync(h->id, d->id, nr * 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(h->fixed, d->fixed, nr * 8, hipMemcpyDeviceToHost, c->stream));
    if (mixed_capable(h) && d->tag) {
        const uint64_t nc = std::min(d->n_children, h->cap_children);
        const uint64_t nk = std::min(d->n_ctl, h->cap_ctl);
        HIPCHK(hipMemcpyAsync(h->tag, d->tag, nr, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(h->aux, d->aux, nr * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(h->ctag, d->ctag, nc, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(h->cfixed, d->cfixed, nc * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(h->caux, d->caux, nc * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(h->ctl_row, d->ctl_row, nk * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(h->ctl_off, d->ctl_off, nk * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(h->ctl_len, d->ctl_len, nk * 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(h->ctl_variant, d->ctl_variant, nk, hipMemcpyDeviceToHost,
                              c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return true;
}

bool copy_cols_h2d(NxgCtx* c, const NxgColumns* h, NxgColumns* d, NetidxError* err) {
    const uint64_t nr = h->n_rows, nc = h->n_children, nk = h->n_ctl;
    HIPCHK(hipMemcpyAsync(d->id, h->id, nr * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d->fixed, h->fixed, nr * 8, hipMemcpyHostToDevice, c->stream));
    if (h->layout == NXG_LAYOUT_MIXED) {
        HIPCHK(hipMemcpyAsync(d->tag, h->tag, nr, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(d->aux, h->aux, nr * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(d->ctag, h->ctag, nc, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(d->cfixed, h->cfixed, nc * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(d->caux, h->caux, nc * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(d->ctl_row, h->ctl_row, nk * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(d->ctl_off, h->ctl_off, nk * 8, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(d->ctl_len, h->ctl_len, nk * 4, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(d->ctl_variant, h->ctl_variant, nk, hipMemcpyHostToDevice,
                              c->stream));
    }
    d->n_rows = nr;
    d->n_children = nc;
    d->n_ctl = nk;
    return true;
}

bool frame_to_device(NxgCtx* c, const uint8_t* frame, uint64_t len, const uint8_t** df,
                     NetidxError* err) {
    const bool dev = is_device_ptr(frame);
    if (dev && ((uintptr_t)frame & 15) == 0) {
        *df = frame;
        return true;
    }
    if (c->dframe_cap < len + 16) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->dframe) HIPCHK(hipFree(c->dframe));
        c->dframe = nullptr;
        size_t n = std::max<size_t>(len + 16, 1 << 20);
        HIPCHK(hipMalloc(&c->dframe, n));
        c->dframe_cap = n;
    }
    if (len)
        HIPCHK(hipMemcpyAsync(c->dframe, frame, len,
                              dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
    *df = c->dframe;
    return true;
}

// *fast = 1 when the sequential-id f64 encoder was launched (finish_encode then reruns a batch it
// declines on the tiled encoder); allow_seq = false forces the tiled encoder.
bool enqueue_encode(NxgCtx* c, const NxgColumns* in, const uint8_t* heap, uint8_t* out,
                    uint64_t cap, DevStatus* st, NetidxError* err, int* fast = nullptr,
                    bool allow_seq = true) {
    if (fast) *fast = 0;
    if (in->layout == NXG_LAYOUT_F64) {
        const bool try_seq = allow_seq && !c->no_enc_seq && in->n_rows > 0;
        if (try_seq && c->enc_seq_left == 0) {
            HIPCHK(nxg_launch_enc_f64s(in->id, in->fixed, in->n_rows, out, cap, st, c->stream));
            if (fast) *fast = 1;
            return true;
        }
        if (try_seq) c->enc_seq_left--;
        const uint64_t nt = nxg_enc_f64_tiles(in->n_rows);
        if (!ensure_tstat(c, nt, err)) return false;
        HIPCHK(nxg_launch_enc_f64(in->id, in->fixed, in->n_rows, out, cap, c->tstat, c->epoch, st,
                                  c->grid_enc_f64, c->stream));
        return true;
    }
    const uint64_t nt = nxg_enc_general_tiles(in->n_rows);
    if (!ensure_tstat(c, nt, err)) return false;
    if (!ensure_escratch(c, in->n_ctl ? in->n_ctl + 1 + in->n_rows : 1, err)) return false;
    const ColsDesc d = desc_of(in);
    HIPCHK(nxg_launch_enc_general(d, heap, out, cap, c->escratch, c->tstat, c->epoch, st,
                                  c->grid_enc_gen, c->stream));
    return true;
}

bool finish_encode(NxgCtx* c, const NxgColumns* in, DevStatus* st, uint32_t slot,
                   uint64_t* len_out, uint64_t cap, bool wrote, NetidxError* err,
                   bool fetched = false, int fast = 0, const uint8_t* heap = nullptr,
                   uint8_t* out = nullptr, bool* redone = nullptr) {
    if (redone) *redone = false;
    if (!fetched)
        HIPCHK(hipMemcpyAsync(c->hst + slot, st, sizeof(DevStatus), hipMemcpyDeviceToHost,
                              c->stream));
    uint64_t ctl_total = 0;
    if (in->layout == NXG_LAYOUT_MIXED && in->n_ctl)
        HIPCHK(hipMemcpyAsync(&ctl_total, c->escratch + in->n_ctl, 8, hipMemcpyDeviceToHost,
                              c->stream));
    if (!fetched || (in->layout == NXG_LAYOUT_MIXED && in->n_ctl))
        HIPCHK(hipStreamSynchronize(c->stream));
    DevStatus h = c->hst[slot];
    if (fast && h.fast_fail) {
        // the sequential-id encoder declined (ids that do not count up by one, or past 35 bits):
        // the tiled encoder, and the sequential one skipped for the next kSeqSkipCalls encodes
        c->enc_seq_left = kSeqSkipCalls;
        DevStatus* st2;
        uint32_t slot2;
        if (!begin_call(c, &st2, &slot2, err)) return false;
        const bool ok = enqueue_encode(c, in, heap, out, cap, st2, err, nullptr, false);
        if (!end_call(c, err) || !ok) return false;
        if (redone) *redone = true;
        HIPCHK(hipMemcpyAsync(c->hst + slot2, st2, sizeof(DevStatus), hipMemcpyDeviceToHost,
                              c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        h = c->hst[slot2];
    }
    c->last_split = h.split_start;
    if (in->layout == NXG_LAYOUT_F64) c->last_enc_kernel = fast && !h.fast_fail ? 1u : 2u;
    if (h.timeout) {
        set_err(err, "device look-back watchdog expired");
        return false;
    }
    if (h.err_kind) {
        if (h.err_kind == NXG_TOO_BIG)
            set_err(err, "encode failed: a message exceeds MAX_BATCH (%llu bytes) or a size "
                         "guard (PackError::TooBig)", (unsigned long long)kMaxBatch);
        else
            set_err(err, "encode failed: PackError kind %u", h.err_kind);
        return false;
    }
    const uint64_t total = h.total_bytes + ctl_total;
    if (len_out) *len_out = total;
    if (wrote && (h.capacity || total > cap)) {
        set_err(err, "output buffer too small: need %llu bytes, have %llu",
                (unsigned long long)total, (unsigned long long)cap);
        return false;
    }
    return true;
}


// ---- memory touched by a call (nxg_ctx_sync's ordering of late fallbacks) ---------------------
struct Span {
    uintptr_t lo, hi;
};

Span span_of(const void* p, uint64_t bytes) {
    const uintptr_t a = (uintptr_t)p;
    return Span{a, p ? a + bytes : a};
}

// every column array of `c`, sized by its capacity (or its count, if larger)
void cols_spans(const NxgColumns* c, std::vector<Span>* v) {
    const uint64_t r = std::max(c->cap_rows, c->n_rows);
    const uint64_t k = std::max(c->cap_children, c->n_children);
    const uint64_t q = std::max(c->cap_ctl, c->n_ctl);
    const std::pair<const void*, uint64_t> a[] = {
        {c->id, r * 8},      {c->fixed, r * 8},   {c->tag, r},         {c->aux, r * 4},
        {c->ctag, k},        {c->cfixed, k * 8},  {c->caux, k * 4},    {c->ctl_row, q * 8},
        {c->ctl_off, q * 8}, {c->ctl_len, q * 4}, {c->ctl_variant, q}};
    for (const auto& x : a)
        if (x.first && x.second) v->push_back(span_of(x.first, x.second));
}

bool overlaps(const std::vector<Span>& a, const std::vector<Span>& b) {
    for (const Span& x : a)
        for (const Span& y : b)
            if (x.lo < y.hi && y.lo < x.hi) return true;
    return false;
}

// a pending decode done again from the start, synchronously (its first attempt's columns were
// overwritten by an earlier frame's late fallback)
bool redo_decode(NxgCtx* c, const NxgCtx::Pending& p, NxgStatus* s, NetidxError* err) {
    DevStatus* st;
    uint32_t slot;
    if (!begin_call(c, &st, &slot, err)) return false;
    int fast = FAST_NONE;
    const bool ok = !(p.flags & NXG_DECODE_HINT_MIXED)
                        ? enqueue_dec_fast(c, p.frame, p.len, p.cols, st, &fast, err)
                        : enqueue_dec_mixed(c, p.frame, p.len, p.cols, st, &fast, err);
    if (!end_call(c, err) || !ok) return false;
    return finish_decode(c, p.frame, p.len, p.cols, fast, st, slot, s, err);
}

// a pending encode done again, synchronously (its input columns were rewritten after it ran)
bool redo_encode(NxgCtx* c, const NxgCtx::Pending& p, const NxgColumns* in, NetidxError* err) {
    DevStatus* st;
    uint32_t slot;
    if (!begin_call(c, &st, &slot, err)) return false;
    int fast = 0;
    const bool ok = enqueue_encode(c, in, p.heap, p.out, p.cap, st, err, &fast);
    if (!end_call(c, err) || !ok) return false;
    return finish_encode(c, in, st, slot, p.len_out, p.cap, true, err, false, fast, p.heap, p.out);
}

}  // namespace

extern "C" {

const char* nxg_version(void) { return "nxg 0.1.0 gfx950"; }

// Not part of the ABI: the last decode's kernel diagnostics (DevStatus::diag), for profiling.
void nxg_debug_status(NxgCtx* c, unsigned long long out[6]) {
    const DevStatus z{};
    const DevStatus& h = c ? c->last : z;
    out[0] = h.fast_fail;
    out[1] = h.irregular;
    out[2] = h.path;
    out[3] = h.n_rows;
    out[4] = h.err_kind;
    out[5] = h.timeout;
}
// Not part of the ABI: which f64 encoder wrote the last f64 encode (1 sequential-id, 2 tiled).
unsigned nxg_debug_enc_kernel(NxgCtx* c) { return c ? c->last_enc_kernel : 0u; }
void nxg_debug_diag(NxgCtx* c, unsigned long long out[8]) {
    for (int i = 0; i < 8; i++) out[i] = c ? c->last.diag[i] : 0;
}

// Not part of the ABI: the last fast archive attempt's FaHead (fast_fail | arrived << 32, end,
// end_children, items, kids, recounts, decline reasons, 1 + the last declining tile).
void nxg_debug_fa(NxgCtx* c, unsigned long long out[8]) {
    for (int i = 0; i < 8; i++) out[i] = c ? c->fa_last[i] : 0;
}

void nxg_error_free(NetidxError* err) {
    if (!err) return;
    free(err->msg);
    err->msg = nullptr;
}

NxgCtx* nxg_ctx_new(int device, NetidxError* err) {
    NxgCtx* c = new NxgCtx();
    c->device = device;
    auto fail = [&](const char* what, hipError_t e) -> NxgCtx* {
        set_err(err, "%s: %s", what, hipGetErrorString(e));
        delete c;
        return nullptr;
    };
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess)
        return fail("hipGetDeviceProperties", e);
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_err(err, "nxg codec is built for gfx950 (MI355X); device %d is %s", device,
                prop.gcnArchName);
        delete c;
        return nullptr;
    }
    c->ncu = prop.multiProcessorCount;
    if ((e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking)) != hipSuccess)
        return fail("hipStreamCreate", e);
    c->stream = c->own;
    // Default schedule for the look-back (encode) kernels: one workgroup per tile in blockIdx
    // order (grid 0), so the look-back always finds recent inclusive prefixes. NXG_PERSISTENT=1
    // selects a persistent grid instead: every workgroup co-resident, with one block of margin
    // under the occupancy answer (MI355X_MICROARCH.md residency notes).
    auto grid = [&](int occ) { return c->ncu * std::max(1, occ > 2 ? occ - 1 : occ); };
    const char* pe = getenv("NXG_PERSISTENT");
    const bool persist = pe && pe[0] == '1';
    c->grid_enc_f64 = persist ? grid(nxg_occupancy_enc_f64()) : 0;
    c->grid_enc_gen = persist ? grid(nxg_occupancy_enc_general()) : 0;
    if ((e = hipMalloc(&c->dst, sizeof(DevStatus) * kStatusRing)) != hipSuccess)
        return fail("hipMalloc(status)", e);
    if ((e = hipMemset(c->dst, 0, sizeof(DevStatus) * kStatusRing)) != hipSuccess)
        return fail("hipMemset(status)", e);
    // (one slot more: the fast archive decoder's FaHead)
    if ((e = hipHostMalloc(&c->hst, sizeof(DevStatus) * (kStatusRing + 1), hipHostMallocDefault)) !=
        hipSuccess)
        return fail("hipHostMalloc(status)", e);
    // general decode: run summaries + bases (no initialisation needed)
    const size_t gw = (size_t)gdec2::MAX_RUNS * (gdec2::RUN_WORDS + 4);
    if ((e = hipMalloc(&c->gruns, gw * 8)) != hipSuccess) return fail("hipMalloc(gruns)", e);
    c->wgs_dec_gen = nxg_dec_gen_wgs(c->ncu);
    nxg_fmx_wgs(c->ncu, c->wgs_fmx);
    const char* fp = getenv("NXG_F64_PATH");
    c->force_x = fp && strcmp(fp, "x") == 0;
    c->no_seq = fp && (strcmp(fp, "run") == 0 || strcmp(fp, "x") == 0);
    const char* fe = getenv("NXG_F64_ENC");
    c->no_enc_seq = fe && strcmp(fe, "tile") == 0;
    const char* mp = getenv("NXG_MIXED_PATH");
    c->no_fmx = mp && strcmp(mp, "general") == 0;
    const char* fc = getenv("NXG_FMX_COUNT");
    c->fmx_count_mode = fc && strcmp(fc, "full") == 0 ? 1 : (fc && strcmp(fc, "lean") == 0 ? 2 : 0);
    const char* ap = getenv("NXG_ARCH_PATH");
    c->no_fa = ap && strcmp(ap, "exact") == 0;
    // (per context: a test context with patience 0 leaves every other context's alone)
    const char* lp = getenv("NXG_LOOKBACK_PATIENCE");
    c->patience = lp ? (uint32_t)strtoul(lp, nullptr, 0) : 128u;
    const char* ff = getenv("NXG_F64R_FLAGS");
    c->f64r_flags = ff ? (uint32_t)strtoul(ff, nullptr, 0) : 0u;
    return c;
}

void nxg_ctx_destroy(NxgCtx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->dcols_valid) cols_free_impl(&c->dcols);
    if (c->tstat) (void)hipFree(c->tstat);
    if (c->glws) (void)hipFree(c->glws);
    if (c->gruns) (void)hipFree(c->gruns);
    if (c->dscratch) (void)hipFree(c->dscratch);
    if (c->pscratch) (void)hipFree(c->pscratch);
    if (c->dframe) (void)hipFree(c->dframe);
    if (c->escratch) (void)hipFree(c->escratch);
    if (c->rdesc) (void)hipFree(c->rdesc);
    if (c->zdefs) (void)hipFree(c->zdefs);
    if (c->zlit) (void)hipFree(c->zlit);
    if (c->zrecs) (void)hipFree(c->zrecs);
    if (c->dheap) (void)hipFree(c->dheap);
    if (c->dst) (void)hipFree(c->dst);
    if (c->hst) (void)hipHostFree(c->hst);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

bool nxg_ctx_set_stream(NxgCtx* c, void* s, NetidxError* err) {
    if (!c) {
        set_err(err, "null ctx");
        return false;
    }
    if (!set_device(c, err)) return false;
    HIPCHK(hipStreamSynchronize(c->stream));
    c->stream = s ? (hipStream_t)s : c->own;
    return true;
}

void* nxg_ctx_stream(NxgCtx* c) { return c ? (void*)c->stream : nullptr; }

bool nxg_columns_alloc(NxgCtx* c, uint32_t layout, uint64_t cap_rows, uint64_t cap_children,
                       uint64_t cap_ctl, uint32_t mem, NxgColumns* out, NetidxError* err) {
    if (!c || !out) {
        set_err(err, "null argument");
        return false;
    }
    if (layout != NXG_LAYOUT_F64 && layout != NXG_LAYOUT_MIXED) {
        set_err(err, "unknown layout %u", layout);
        return false;
    }
    if (mem != NXG_MEM_DEVICE && mem != NXG_MEM_HOST) {
        set_err(err, "unknown memory kind %u", mem);
        return false;
    }
    if (!set_device(c, err)) return false;
    if (!cols_alloc_impl(layout, cap_rows, cap_children, cap_ctl, mem, out, err)) {
        cols_free_impl(out);
        return false;
    }
    return true;
}

void nxg_columns_free(NxgCtx* c, NxgColumns* cols) {
    if (!cols) return;
    if (c) (void)hipSetDevice(c->device);
    cols_free_impl(cols);
}

bool nxg_decode_updates(NxgCtx* c, const uint8_t* frame, uint64_t len, NxgColumns* out,
                        uint32_t flags, NxgStatus* ust, NetidxError* err) {
    if (!c || !out || (!frame && len)) {
        set_err(err, "null argument");
        return false;
    }
    if (!c->pending.empty()) {
        set_err(err, "an async operation is pending on this ctx; call nxg_ctx_sync first");
        return false;
    }
    if (len >= (1ull << 40)) {
        set_err(err, "frame too large (%llu bytes)", (unsigned long long)len);
        return false;
    }
    if (!set_device(c, err)) return false;
    const uint8_t* df;
    if (!frame_to_device(c, frame, len, &df, err)) return false;
    NxgColumns* target = out;
    NxgColumns view;
    const bool host_out = out->mem == NXG_MEM_HOST;
    if (host_out) {
        if (!ensure_dcols(c, out, err)) return false;
        view = staged_view(c, out);
        target = &view;
    }
    DevStatus* st;
    uint32_t slot;
    if (!begin_call(c, &st, &slot, err)) return false;
    int fast = FAST_NONE;
    const bool ok = !(flags & NXG_DECODE_HINT_MIXED)
                        ? enqueue_dec_fast(c, df, len, target, st, &fast, err)
                        : enqueue_dec_mixed(c, df, len, target, st, &fast, err);
    if (!end_call(c, err) || !ok) return false;
    NxgStatus s;
    if (!finish_decode(c, df, len, target, fast, st, slot, &s, err)) return false;
    // result layout: F64 when the homogeneous kernel produced it (tag/aux not written)
    out->layout = (!mixed_capable(out) || s.path == 1) ? NXG_LAYOUT_F64 : NXG_LAYOUT_MIXED;
    if (host_out) {
        target->n_rows = s.n_rows;
        target->n_children = s.n_children;
        target->n_ctl = s.n_ctl;
        if (s.err_kind == 0) {
            NxgColumns hv = *out;
            if (s.path == 1) hv.tag = nullptr;  // only id/fixed were produced
            if (!copy_cols_d2h(c, target, &hv, err)) return false;
        }
    }
    out->n_rows = s.n_rows;
    out->n_children = s.n_children;
    out->n_ctl = s.n_ctl;
    out->n_heartbeat = s.n_heartbeat;
    if (ust) *ust = s;
    return true;
}

bool nxg_decode_updates_async(NxgCtx* c, const uint8_t* dframe, uint64_t len, NxgColumns* dout,
                              uint32_t flags, NetidxError* err) {
    if (!c || !dout || (!dframe && len)) {
        set_err(err, "null argument");
        return false;
    }
    if (c->pending.size() >= kStatusRing / 2) {
        set_err(err, "too many in-flight async calls (max %d); call nxg_ctx_sync", kStatusRing / 2);
        return false;
    }
    if (dout->mem != NXG_MEM_DEVICE || ((uintptr_t)dframe & 15)) {
        set_err(err, "async decode needs device columns and a 16-byte aligned device frame");
        return false;
    }
    DevStatus* st;
    uint32_t slot;
    if (!begin_call(c, &st, &slot, err)) return false;
    int fast = FAST_NONE;
    const bool ok = !(flags & NXG_DECODE_HINT_MIXED)
                        ? enqueue_dec_fast(c, dframe, len, dout, st, &fast, err)
                        : enqueue_dec_mixed(c, dframe, len, dout, st, &fast, err);
    if (!end_call(c, err) || !ok) return false;
    c->pending.push_back({1, fast, dframe, len, dout, nullptr, 0, st, slot, flags});
    return true;
}

bool nxg_decode_frames_async(NxgCtx* c, uint32_t n, const uint8_t* const* dframes,
                             const uint64_t* lens, NxgColumns* const* douts, uint32_t flags,
                             NetidxError* err) {
    if (!c || (n && (!dframes || !lens || !douts))) {
        set_err(err, "null argument");
        return false;
    }
    if (c->pending.size() + n > kStatusRing / 2) {
        set_err(err, "too many in-flight async calls (max %d); call nxg_ctx_sync", kStatusRing / 2);
        return false;
    }
    uint64_t max_len = 0;
    for (uint32_t j = 0; j < n; j++) {
        if (!douts[j] || (!dframes[j] && lens[j])) {
            set_err(err, "null frame or columns at %u", j);
            return false;
        }
        if (douts[j]->mem != NXG_MEM_DEVICE || ((uintptr_t)dframes[j] & 15)) {
            set_err(err, "async decode needs device columns and 16-byte aligned device frames");
            return false;
        }
        max_len = std::max(max_len, lens[j]);
    }
    const bool run_path = !(flags & NXG_DECODE_HINT_MIXED) && !c->force_x &&
                          c->irregular_left == 0 && n > 1 && !seq_active(c);
    if (!run_path) {
        for (uint32_t j = 0; j < n; j++)
            if (!nxg_decode_updates_async(c, dframes[j], lens[j], douts[j], flags, err))
                return false;
        return true;
    }
    if (!set_device(c, err)) return false;
    // two descriptor arrays: frame j's probe runs beside frame j - 1's emit
    const size_t half = (16 * nxg_dec_f64r_tiles(max_len) + 255) & ~(size_t)255;
    if (!ensure_tstat(c, nxg_dec_f64r_groups(max_len), err)) return false;
    if (!ensure_rdesc(c, 2 * half, err)) return false;
    std::vector<NxgF64rFrame> fr(n);
    std::vector<NxgCtx::Pending> pend;
    pend.reserve(n);
    uint32_t nonempty = 0;  // descriptor arrays alternate over the frames that launch
    for (uint32_t j = 0; j < n; j++) {
        DevStatus* st;
        uint32_t slot;
        if (!begin_call(c, &st, &slot, err)) return false;
        NxgF64rFrame& f = fr[j];
        f.wire = dframes[j];
        f.W = lens[j];
        f.oid = douts[j]->id;
        f.oval = douts[j]->fixed;
        f.cap = douts[j]->cap_rows;
        f.desc = c->rdesc + (nonempty & 1) * half;
        if (lens[j]) nonempty++;
        f.epoch = c->epoch;
        f.st = st;
        f.zst = nxg_take_zero_slot();
        // an empty frame launches nothing: its zero-ahead slot is cleared here
        if (lens[j] == 0) HIPCHK(hipMemsetAsync(f.zst, 0, sizeof(DevStatus), c->stream));
        pend.push_back({1, FAST_RUN, dframes[j], lens[j], douts[j], nullptr, 0, st, slot});
    }
    // (the frames become pending only once their launches are enqueued: a failed launch leaves
    // no call behind whose status slot no kernel wrote)
    HIPCHK(nxg_launch_dec_f64r_stream(fr.data(), n, c->tstat, c->f64r_flags, c->stream));
    // (these frames skipped the sequential-id decoder: they count toward its skip)
    c->seq_left = c->seq_left > n ? c->seq_left - n : 0;
    c->pending.insert(c->pending.end(), pend.begin(), pend.end());
    return true;
}

// Completes every in-flight call in order (every one, even after a failure, so that each decode
// gets its fallback and each encode its length); the status returned is the last call's, or the
// first failing call's, and the first error is the one reported.
//
// A decode that falls back here rewrites its columns after every later call of the backlog has
// run. Later calls that touched the same memory are therefore done again, in order: a decode
// whose columns (or frame) overlap what was rewritten, and an encode whose input columns do; what
// those rewrite joins the set. (nxg_codec.h allows a backlog to reuse columns, the later frame's
// rows being the ones left.)
bool nxg_ctx_sync(NxgCtx* c, NxgStatus* ust, NetidxError* err) {
    if (!c) {
        set_err(err, "null ctx");
        return false;
    }
    if (!set_device(c, err)) return false;
    std::vector<NxgCtx::Pending> ps;
    ps.swap(c->pending);
    HIPCHK(hipStreamSynchronize(c->stream));
    // the in-flight calls used consecutive ring slots: at most two copies cover them
    std::vector<DevStatus> hs(ps.size());
    if (!ps.empty()) {
        const uint32_t s0 = ps.front().slot, s1 = ps.back().slot;
        if (s0 <= s1) {
            HIPCHK(hipMemcpyAsync(c->hst + s0, c->dst + s0, sizeof(DevStatus) * (s1 - s0 + 1),
                                  hipMemcpyDeviceToHost, c->stream));
        } else {
            HIPCHK(hipMemcpyAsync(c->hst + s0, c->dst + s0, sizeof(DevStatus) * (kStatusRing - s0),
                                  hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipMemcpyAsync(c->hst, c->dst, sizeof(DevStatus) * (s1 + 1),
                                  hipMemcpyDeviceToHost, c->stream));
        }
        HIPCHK(hipStreamSynchronize(c->stream));
        // (kept aside: the fallbacks below take ring slots of their own, which may wrap)
        for (size_t i = 0; i < ps.size(); i++) hs[i] = c->hst[ps[i].slot];
    }
    if (ust) memset(ust, 0, sizeof *ust);
    bool reported = false, ok = true;
    std::vector<Span> dirty;  // memory rewritten by a call completed out of order
    for (size_t i = 0; i < ps.size(); i++) {
        auto& p = ps[i];
        c->hst[p.slot] = hs[i];
        NetidxError e{nullptr};
        bool r;
        if (p.kind == 1) {
            std::vector<Span> w;
            cols_spans(p.cols, &w);
            const bool stale =
                !dirty.empty() && (overlaps(dirty, w) || overlaps(dirty, {span_of(p.frame, p.len)}));
            NxgStatus s;
            bool redone = false;
            // write-after-read: a fallback re-reads the frame after every later call has run; if
            // a later call wrote into the frame (stream-ordered reuse of the buffer as an encode
            // output or as columns), those bytes are gone -- fail loudly instead of decoding them
            if (!stale && hs[i].fast_fail && p.len > 0 && p.fast) {
                const std::vector<Span> fr = {span_of(p.frame, p.len)};
                bool clobbered = false;
                for (size_t j = i + 1; j < ps.size() && !clobbered; j++) {
                    std::vector<Span> wj;
                    if (ps[j].kind == 1) cols_spans(ps[j].cols, &wj);
                    else wj.push_back(span_of(ps[j].out, ps[j].cap));
                    clobbered = overlaps(fr, wj);
                }
                if (clobbered) {
                    if (ok) {
                        ok = false;
                        set_err(err, "decode of async call %zu needs its frame again (fallback), "
                                     "but a later call in the backlog wrote into that frame "
                                     "buffer; keep a frame unchanged until nxg_ctx_sync",
                                i);
                    }
                    continue;
                }
            }
            if (stale) {
                r = redo_decode(c, p, &s, &e);
                redone = true;
            } else {
                r = finish_decode(c, p.frame, p.len, p.cols, p.fast, p.st, p.slot, &s, &e, true,
                                  &redone);
            }
            if (redone) dirty.insert(dirty.end(), w.begin(), w.end());
            if (r) {
                p.cols->layout =
                    (!mixed_capable(p.cols) || s.path == 1) ? NXG_LAYOUT_F64 : NXG_LAYOUT_MIXED;
                if (ust && !reported) *ust = s;
                if (s.err_kind) reported = true;
            }
        } else {
            NxgColumns dummy{};
            dummy.layout = NXG_LAYOUT_F64;
            const NxgColumns* in = p.cols ? p.cols : &dummy;
            std::vector<Span> rd;
            cols_spans(in, &rd);
            bool clobbered = false;
            if (p.fast && hs[i].fast_fail && (dirty.empty() || !overlaps(dirty, rd))) {
                // write-after-read: the fallback re-reads the input columns after every later
                // call ran; a later call that wrote into them leaves nothing to encode
                for (size_t j = i + 1; j < ps.size() && !clobbered; j++) {
                    std::vector<Span> wj;
                    if (ps[j].kind == 1) cols_spans(ps[j].cols, &wj);
                    else wj.push_back(span_of(ps[j].out, ps[j].cap));
                    clobbered = overlaps(rd, wj);
                }
            }
            if (clobbered) {
                r = false;
                set_err(&e, "encode of async call %zu needs its columns again (fallback), but a "
                            "later call in the backlog wrote into them; keep them unchanged until "
                            "nxg_ctx_sync", i);
            } else if (!dirty.empty() && overlaps(dirty, rd)) {
                // its input columns were rewritten after it ran: encode again
                r = redo_encode(c, p, in, &e);
                dirty.push_back(span_of(p.out, p.cap));
            } else {
                bool redone = false;
                r = finish_encode(c, in, p.st, p.slot, p.len_out, p.cap, true, &e, true, p.fast,
                                  p.heap, p.out, &redone);
                if (redone) dirty.push_back(span_of(p.out, p.cap));
            }
        }
        if (!r && ok) {
            ok = false;
            set_err(err, "%s", e.msg ? e.msg : "async call failed");
        }
        nxg_error_free(&e);
    }
    return ok;
}

static bool encode_impl(NxgCtx* c, const NxgColumns* in, const uint8_t* heap, uint8_t* out,
                        uint64_t cap, uint64_t* len_out, NetidxError* err) {
    if (!c || !in) {
        set_err(err, "null argument");
        return false;
    }
    if (!c->pending.empty()) {
        set_err(err, "an async operation is pending on this ctx; call nxg_ctx_sync first");
        return false;
    }
    if (!set_device(c, err)) return false;
    const bool host = in->mem == NXG_MEM_HOST || !is_device_ptr(in->id);
    const NxgColumns* din = in;
    NxgColumns view;
    const uint8_t* dheap = heap;
    uint8_t* dout = out;
    uint64_t heap_len = 0;
    if (host) {
        if (!ensure_dcols(c, in, err)) return false;
        view = staged_view(c, in);
        if (!copy_cols_h2d(c, in, &view, err)) return false;
        din = &view;
        // the heap extent: everything referenced by offsets; callers pass the frame/heap whose
        // length is not part of the ABI, so stage the maximum referenced byte
        if (heap && in->layout == NXG_LAYOUT_MIXED) {
            uint64_t hi = 0;
            auto upd = [&](uint8_t t, uint64_t f, uint32_t a) {
                if (t == 12 || t == 13 || t == 18 || t == 27) hi = std::max<uint64_t>(hi, f + a);
                if (t == 20) hi = std::max<uint64_t>(hi, f + 16);
            };
            for (uint64_t i = 0; i < in->n_rows; i++) upd(in->tag[i], in->fixed[i], in->aux[i]);
            for (uint64_t i = 0; i < in->n_children; i++)
                upd(in->ctag[i], in->cfixed[i], in->caux[i]);
            for (uint64_t i = 0; i < in->n_ctl; i++)
                hi = std::max<uint64_t>(hi, in->ctl_off[i] + in->ctl_len[i]);
            heap_len = hi;
            if (c->dheap_cap < heap_len + 16) {
                HIPCHK(hipStreamSynchronize(c->stream));
                if (c->dheap) HIPCHK(hipFree(c->dheap));
                c->dheap = nullptr;
                size_t n = std::max<size_t>(heap_len + 16, 1 << 20);
                HIPCHK(hipMalloc(&c->dheap, n));
                c->dheap_cap = n;
            }
            if (heap_len)
                HIPCHK(hipMemcpyAsync(c->dheap, heap, heap_len, hipMemcpyHostToDevice, c->stream));
            dheap = c->dheap;
        }
        dout = nullptr;
    }
    DevStatus* st;
    uint32_t slot;
    uint64_t total = 0;
    // pass 1 (sizing) when writing to a host buffer; a device buffer is written directly
    if (host && out) {
        if (!begin_call(c, &st, &slot, err)) return false;
        int fast = 0;
        const bool ok = enqueue_encode(c, din, dheap, nullptr, 0, st, err, &fast);
        if (!end_call(c, err) || !ok) return false;
        if (!finish_encode(c, din, st, slot, &total, 0, false, err, false, fast, dheap, nullptr))
            return false;
        if (total > cap) {
            set_err(err, "output buffer too small: need %llu bytes, have %llu",
                    (unsigned long long)total, (unsigned long long)cap);
            return false;
        }
        if (c->dframe_cap < total + 16) {
            HIPCHK(hipStreamSynchronize(c->stream));
            if (c->dframe) HIPCHK(hipFree(c->dframe));
            c->dframe = nullptr;
            size_t n = std::max<size_t>(total + 16, 1 << 20);
            HIPCHK(hipMalloc(&c->dframe, n));
            c->dframe_cap = n;
        }
        dout = c->dframe;
        cap = total;
    }
    if (!begin_call(c, &st, &slot, err)) return false;
    int fast = 0;
    const bool ok = enqueue_encode(c, din, dheap, dout, out ? cap : 0, st, err, &fast);
    if (!end_call(c, err) || !ok) return false;
    if (!finish_encode(c, din, st, slot, &total, cap, dout != nullptr, err, false, fast, dheap,
                       dout))
        return false;
    if (host && out && total) {
        HIPCHK(hipMemcpyAsync(out, dout, total, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    if (len_out) *len_out = total;
    return true;
}

// ---- archive batches (netidx-archive logfile/mod.rs:150-205) ---------------------------------
// <Vec<BatchItem> as Pack>::encode (pack.rs:941-952): the count varint here, the items by the
// general encoder's rows kernel in archive mode
bool nxg_encode_archive_batch(NxgCtx* c, const NxgColumns* in, const uint8_t* heap, uint8_t* out,
                              uint64_t cap, uint64_t* len_out, NetidxError* err) {
    if (!c || !in) {
        set_err(err, "null argument");
        return false;
    }
    if (!c->pending.empty()) {
        set_err(err, "an async operation is pending on this ctx; call nxg_ctx_sync first");
        return false;
    }
    if (in->mem != NXG_MEM_DEVICE || !mixed_capable(in) || in->n_ctl ||
        (in->n_rows && (!in->id || !is_device_ptr(in->id)))) {
        set_err(err, "archive batches encode from device MIXED-layout columns without control "
                     "messages");
        return false;
    }
    if (in->n_rows > kMaxVecBytes / kBatchItemSize) {  // Vec::encode's guard (pack.rs:943-945)
        set_err(err, "encode failed: %llu items exceed MAX_VEC (PackError::TooBig)",
                (unsigned long long)in->n_rows);
        return false;
    }
    if (!set_device(c, err)) return false;
    uint8_t hdr[10];
    uint32_t hl = 0;
    for (uint64_t v = in->n_rows;; v >>= 7) {
        if (v < 0x80) {
            hdr[hl++] = (uint8_t)v;
            break;
        }
        hdr[hl++] = (uint8_t)((v & 0x7f) | 0x80);
    }
    if (out && cap < hl) {
        set_err(err, "output buffer too small: need at least %u bytes", hl);
        return false;
    }
    if (out) HIPCHK(hipMemcpyAsync(out, hdr, hl, hipMemcpyHostToDevice, c->stream));
    const uint64_t nt = nxg_enc_general_tiles(in->n_rows);
    if (!ensure_tstat(c, nt, err) || !ensure_escratch(c, 1, err)) return false;
    DevStatus* st;
    uint32_t slot;
    if (!begin_call(c, &st, &slot, err)) return false;
    const hipError_t le = nxg_launch_enc_general(desc_of(in), heap, out, out ? cap : 0, c->escratch,
                                                 c->tstat, c->epoch, st, c->grid_enc_gen,
                                                 c->stream, hl);
    if (!end_call(c, err)) return false;
    HIPCHK(le);
    uint64_t total = 0;
    if (!finish_encode(c, in, st, slot, &total, cap, out != nullptr, err)) return false;
    if (in->n_rows == 0) total = hl;
    if (len_out) *len_out = total;
    return true;
}

struct NxgZstdDict {
    int device;
    void* ddev = nullptr;       // NxzDictDev
    uint8_t* content = nullptr;  // the dictionary's content (history before every frame)
};

NxgZstdDict* nxg_zstd_dict_new(NxgCtx* c, const uint8_t* dict, uint64_t len, NetidxError* err) {
    if (!c || (!dict && len)) {
        set_err(err, "null argument");
        return nullptr;
    }
    if (!set_device(c, err)) return nullptr;
    std::vector<uint8_t> host(nxg_zstd_dict_dev_bytes());
    NxzDictDev* hd = reinterpret_cast<NxzDictDev*>(host.data());
    uint64_t coff = 0;
    if (!nxg_zstd_build_dict(dict, len, hd, &coff)) {
        set_err(err, "not a valid zstd dictionary");
        return nullptr;
    }
    NxgZstdDict* d = new NxgZstdDict();
    d->device = c->device;
    const uint64_t clen = len - coff;
    auto fail = [&](hipError_t e) -> NxgZstdDict* {
        set_err(err, "zstd dictionary upload: %s", hipGetErrorString(e));
        nxg_zstd_dict_free(d);
        return nullptr;
    };
    hipError_t e;
    if ((e = hipMalloc(&d->content, std::max<uint64_t>(clen, 1))) != hipSuccess) return fail(e);
    if (clen && (e = hipMemcpy(d->content, dict + coff, clen, hipMemcpyHostToDevice)) != hipSuccess)
        return fail(e);
    nxg_zstd_set_content(hd, d->content);
    if ((e = hipMalloc(&d->ddev, host.size())) != hipSuccess) return fail(e);
    if ((e = hipMemcpy(d->ddev, host.data(), host.size(), hipMemcpyHostToDevice)) != hipSuccess)
        return fail(e);
    return d;
}

void nxg_zstd_dict_free(NxgZstdDict* d) {
    if (!d) return;
    (void)hipSetDevice(d->device);
    if (d->ddev) (void)hipFree(d->ddev);
    if (d->content) (void)hipFree(d->content);
    delete d;
}

bool nxg_archive_decompress(NxgCtx* c, const NxgZstdDict* dict, const uint8_t* src,
                            uint64_t src_len, NxgArchiveRecord* recs, uint32_t n, bool indexed,
                            uint8_t* dout, uint64_t cap, uint64_t* need, NetidxError* err) {
    if (!c || (n && (!recs || !src))) {
        set_err(err, "null argument");
        return false;
    }
    if (!c->pending.empty()) {
        set_err(err, "an async operation is pending on this ctx; call nxg_ctx_sync first");
        return false;
    }
    if (is_device_ptr(src)) {
        set_err(err, "the records must be in host memory (the archive's mmap)");
        return false;
    }
    // the records' headers on the host (reader.rs:453-466): the uncompressed length sizes each
    // output slot, the index is skipped
    struct Rec {
        uint64_t frame_off, frame_len, out_off, out_cap;
    };
    std::vector<Rec> rd(n);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        NxgArchiveRecord& r = recs[i];
        r.out_len = 0;
        r.err = 0;
        r.out_off = total;
        Rec& x = rd[i];
        x = Rec{0, 0, total, 0};
        if (r.off > src_len || r.len > src_len - r.off || r.len < 4) {
            r.err = 7;
            continue;
        }
        const uint8_t* p = src + r.off;
        const uint64_t uncomp = ((uint64_t)p[0] << 24) | ((uint64_t)p[1] << 16) |
                                ((uint64_t)p[2] << 8) | p[3];
        uint64_t pos = 4;
        if (indexed) {  // decode_varint (pack.rs:504-520): the index's length, prefix included
            uint64_t v = 0;
            uint32_t k = 0;
            bool ok = false;
            for (; k < 10 && pos + k < r.len; k++) {
                v |= (uint64_t)(p[pos + k] & 0x7f) << (7 * k);
                if (p[pos + k] < 0x80) {
                    ok = true;
                    break;
                }
            }
            if (!ok || v > r.len - pos) {
                r.err = 7;
                continue;
            }
            pos += v;
        }
        x.frame_off = r.off + pos;
        x.frame_len = r.len - pos;
        x.out_cap = uncomp;
        total += uncomp;
    }
    if (need) *need = total;
    if (!dout) return true;
    if (total > cap) {
        set_err(err, "output buffer too small: the records need %llu bytes, capacity %llu",
                (unsigned long long)total, (unsigned long long)cap);
        return false;
    }
    if (n == 0) return true;
    if (!set_device(c, err)) return false;
    if (!c->zdefs) {
        std::vector<uint8_t> h(nxg_zstd_defaults_bytes());
        if (!nxg_zstd_build_defaults(reinterpret_cast<NxzDefaults*>(h.data()))) {
            set_err(err, "predefined zstd tables");
            return false;
        }
        HIPCHK(hipMalloc(&c->zdefs, h.size()));
        HIPCHK(hipMemcpy(c->zdefs, h.data(), h.size(), hipMemcpyHostToDevice));
        c->zgrid = nxg_zstd_grid(c->ncu);
        HIPCHK(hipMalloc(&c->zlit, (size_t)c->zgrid * nxg_zstd_litbuf_bytes()));
    }
    const size_t rb = nxg_zstd_rec_bytes(), sb = nxg_zstd_res_bytes();
    static_assert(sizeof(Rec) == 32, "NxzRec layout");
    if (c->zrecs_cap < (size_t)n * (rb + sb)) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->zrecs) HIPCHK(hipFree(c->zrecs));
        c->zrecs = nullptr;
        c->zrecs_cap = std::max<size_t>((size_t)n * (rb + sb), 1 << 16);
        HIPCHK(hipMalloc(&c->zrecs, c->zrecs_cap));
    }
    uint8_t* drecs = static_cast<uint8_t*>(c->zrecs);
    uint8_t* dres = drecs + (size_t)n * rb;
    const uint8_t* dsrc;
    if (!frame_to_device(c, src, src_len, &dsrc, err)) return false;
    HIPCHK(hipMemcpyAsync(drecs, rd.data(), (size_t)n * rb, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(dres, 0, (size_t)n * sb, c->stream));
    HIPCHK(nxg_launch_zstd(dsrc, drecs, n, dict ? dict->ddev : nullptr, c->zdefs, dout, c->zlit,
                           dres, c->zgrid, c->stream));
    struct Res {
        uint64_t out_len;
        uint32_t err, pad;
    };
    std::vector<Res> hr(n);
    HIPCHK(hipMemcpyAsync(hr.data(), dres, (size_t)n * sb, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (uint32_t i = 0; i < n; i++) {
        if (recs[i].err) continue;  // rejected on the host
        recs[i].out_len = hr[i].out_len;
        recs[i].err = hr[i].err;
        if (recs[i].err) recs[i].out_len = 0;
    }
    return true;
}

// the fast archive decoder's device results (nxg_archive_fast.hip FaHead)
struct FaHeadHost {
    uint32_t fast_fail, arrived;
    uint64_t end, end_children, items, ticket, recounts, why, why_tile;
};
static_assert(sizeof(FaHeadHost) == 64 && sizeof(FaHeadHost) <= sizeof(DevStatus), "FaHead");

// The batch header on the host: the count varint (decode_varint, pack.rs:504-520: at most 10
// bytes, bits past 64 dropped) and its length; false when it is not a complete varint (the exact
// decoder reports that) or check_sz! would refuse it (pack.rs:919-925)
static bool arch_header(NxgCtx* c, const uint8_t* buf, uint64_t len, uint64_t* count, uint32_t* p0,
                        NetidxError* err) {
    uint8_t h[10] = {0};
    const uint64_t n = std::min<uint64_t>(len, 10);
    if (n == 0) return false;
    if (is_device_ptr(buf)) {
        if (hipMemcpyAsync(h, buf, n, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            return false;
    } else {
        memcpy(h, buf, n);
    }
    (void)err;
    uint64_t v = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t b = h[i];
        v |= i < 9 ? (b & 0x7f) << (7 * i) : (b & 1) << 63;
        if (b < 0x80) {
            *count = v;
            *p0 = i + 1;
            const uint64_t sz = v > ~0ull / 24 ? ~0ull : v * 24;  // size_of::<BatchItem>()
            return sz <= kMaxVecBytes && sz <= ((len - (i + 1)) << 8);
        }
    }
    return false;
}

bool nxg_decode_archive_batch(NxgCtx* c, const uint8_t* buf, uint64_t len, NxgColumns* out,
                              NxgStatus* ust, uint64_t* consumed, NetidxError* err) {
    if (!c || !out || (!buf && len)) {
        set_err(err, "null argument");
        return false;
    }
    if (!c->pending.empty()) {
        set_err(err, "an async operation is pending on this ctx; call nxg_ctx_sync first");
        return false;
    }
    if (len >= (1ull << 40)) {
        set_err(err, "batch too large (%llu bytes)", (unsigned long long)len);
        return false;
    }
    if (out->mem != NXG_MEM_DEVICE || !mixed_capable(out) || !out->id) {
        set_err(err, "archive batches decode into device MIXED-layout columns");
        return false;
    }
    if (!set_device(c, err)) return false;
    const uint8_t* df;
    // the fast path (nxg_archive_fast.hip) over a window of the buffer that grows until the batch
    // fits; anything it declines goes to the exact decoder below over the whole buffer
    uint64_t count = 0;
    uint32_t p0 = 0;
    if (!c->no_fa && arch_header(c, buf, len, &count, &p0, err) && count >= 1 &&
        count <= out->cap_rows && count < (1ull << 31) && out->tag && out->ctag) {
        const uint64_t wmax = std::min<uint64_t>(len, 0xfff00000ull);
        uint64_t W = std::min<uint64_t>(wmax, p0 + count * 24 + 65536);
        FaHeadHost* hh = reinterpret_cast<FaHeadHost*>(c->hst + kStatusRing);
#pragma unroll 1
        for (;;) {
            if (!frame_to_device(c, buf, W, &df, err)) return false;
            const size_t need = nxg_fa_scratch_bytes(W);
            if (need > c->dscratch_cap) {
                HIPCHK(hipStreamSynchronize(c->stream));
                if (c->dscratch) HIPCHK(hipFree(c->dscratch));
                c->dscratch = nullptr;
                const size_t sz = std::max(need, c->dscratch_cap * 2);
                HIPCHK(hipMalloc(&c->dscratch, sz));
                c->dscratch_cap = sz;
            }
            HIPCHK(nxg_launch_dec_fa(df, W, p0, count, desc_of(out), c->dscratch, hh, nullptr,
                                     c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            memcpy(c->fa_last, hh, sizeof c->fa_last);
            if (!hh->fast_fail && hh->end) {
                NxgStatus s{};
                s.n_rows = count;
                s.n_children = hh->end_children;
                s.path = NXG_PATH_ARCHIVE_FAST;
                out->n_rows = count;
                out->n_children = hh->end_children;
                out->n_ctl = 0;
                out->layout = NXG_LAYOUT_MIXED;
                if (ust) *ust = s;
                if (consumed) *consumed = hh->end - 1;
                return true;
            }
            // a larger window helps only a chain that ran out of window (decline reasons 1 and
            // 2: a broken or mismatched chain); a decode error or a declined value goes straight
            // to the exact decoder
            if (W >= wmax || (hh->why & ~3ull)) break;
            W = std::min(wmax, 2 * W);
        }
    }
    if (!frame_to_device(c, buf, len, &df, err)) return false;
    const size_t need = 64 + nxg_arch_scratch_bytes(len);
    if (need > c->dscratch_cap) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->dscratch) HIPCHK(hipFree(c->dscratch));
        c->dscratch = nullptr;
        const size_t sz = std::max(need, c->dscratch_cap * 2);
        HIPCHK(hipMalloc(&c->dscratch, sz));
        c->dscratch_cap = sz;
    }
    uint32_t* cap_flag = reinterpret_cast<uint32_t*>(c->dscratch);
    HIPCHK(hipMemsetAsync(cap_flag, 0, 4, c->stream));
    NxgArchResult r{};
    HIPCHK(nxg_arch_decode(df, len, desc_of(out), c->dscratch + 64, cap_flag, 8, &r, c->stream));
    NxgStatus s{};
    s.n_rows = r.n_rows;
    s.n_children = r.n_children;
    s.err_kind = (int32_t)r.err_kind;
    s.err_offset = r.err_offset;
    s.path = NXG_PATH_ARCHIVE;
    out->n_rows = r.n_rows;
    out->n_children = r.n_children;
    out->n_ctl = 0;
    out->layout = NXG_LAYOUT_MIXED;
    if (ust) *ust = s;
    if (consumed) *consumed = r.consumed;
    return true;
}

// ---- type-partitioned view ------------------------------------------------------
bool nxg_partition_by_tag(NxgCtx* c, const NxgColumns* cols, NxgTagView* out, NetidxError* err) {
    if (!c || !cols || !out) {
        set_err(err, "null argument");
        return false;
    }
    const uint64_t n = cols->n_rows;
    if (cols->layout != NXG_LAYOUT_MIXED || !cols->tag || !cols->fixed || !cols->aux) {
        set_err(err, "the type-partitioned view needs mixed-layout columns (a tag column)");
        return false;
    }
    if (n && (!out->rank || !out->row_of || !out->fixed || !out->aux)) {
        set_err(err, "null output array");
        return false;
    }
    if (n > out->cap_rows || n > 0xffffffffull) {
        set_err(err, "%llu rows: the view's capacity is %llu (and rows must be < 2^32)",
                (unsigned long long)n, (unsigned long long)out->cap_rows);
        return false;
    }
    if (n && (!is_device_ptr(cols->tag) || !is_device_ptr(out->rank))) {
        set_err(err, "the type-partitioned view needs device columns and device outputs");
        return false;
    }
    if (!c->pending.empty()) {
        set_err(err, "an async operation is pending on this ctx; call nxg_ctx_sync first");
        return false;
    }
    if (!set_device(c, err)) return false;
    const size_t need = nxg_part_scratch_bytes(n);
    if (need > c->pscratch_cap) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->pscratch) HIPCHK(hipFree(c->pscratch));
        c->pscratch = nullptr;
        const size_t m = std::max(need, c->pscratch_cap * 2);
        HIPCHK(hipMalloc(&c->pscratch, m));
        c->pscratch_cap = m;
    }
    uint64_t* doff = nullptr;
    HIPCHK(nxg_launch_partition(cols->tag, cols->fixed, cols->aux, n, c->pscratch, out->rank,
                                out->row_of, out->fixed, out->aux, &doff, c->stream));
    HIPCHK(hipMemcpyAsync(out->off, doff, sizeof(uint64_t) * (NXG_TAG_BINS + 1),
                          hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int t = 0; t < NXG_TAG_BINS; t++) out->count[t] = out->off[t + 1] - out->off[t];
    out->n_rows = n;
    return true;
}

// ---- dispatch (connection.rs:546-567) --------------------------------------------------------
bool nxg_dispatch_updates(NxgCtx* c, const NxgSubTable* tab, const uint64_t* id, uint64_t n_rows,
                          NxgDispatch* out, NetidxError* err) {
    if (!c || !tab || !out || (n_rows && !id) || !out->chan_off) {
        set_err(err, "null argument");
        return false;
    }
    if ((tab->n_ids && !tab->slot_of_id) ||
        (tab->n_slots && (!tab->slot_sub_id || !tab->slot_stream_off || !tab->slot_has_last ||
                          !out->last_row)) ||
        (out->cap_entries && (!out->ent_sub || !out->ent_row))) {
        set_err(err, "null table or output array");
        return false;
    }
    if (n_rows && tab->n_slots && !tab->stream_chan && tab->n_chans) {
        set_err(err, "null stream_chan");
        return false;
    }
    HIPCHK(hipSetDevice(c->device));
    const size_t need = 64 + nxg_disp_scratch_bytes(n_rows, tab->n_chans);
    if (need > c->dscratch_cap) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->dscratch) HIPCHK(hipFree(c->dscratch));
        c->dscratch = nullptr;
        const size_t n = std::max(need, c->dscratch_cap * 2);
        HIPCHK(hipMalloc(&c->dscratch, n));
        c->dscratch_cap = n;
    }
    uint64_t* um = reinterpret_cast<uint64_t*>(c->dscratch);
    HIPCHK(nxg_launch_dispatch(*tab, id, n_rows, c->dscratch + 64, out->chan_off, out->ent_sub,
                               out->ent_row, out->cap_entries, out->last_row, um, c->ncu,
                               c->stream));
    uint64_t res[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(&res[0], out->chan_off + tab->n_chans, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(&res[1], um, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    out->n_entries = res[0];
    out->n_unmatched = res[1];
    if (res[0] > out->cap_entries) {
        set_err(err, "dispatch needs %llu entries, capacity is %llu", (unsigned long long)res[0],
                (unsigned long long)out->cap_entries);
        return false;
    }
    return true;
}

// ---- publisher commit (publisher/mod.rs:776-845) -----------------------------------------------
bool nxg_publish_commit(NxgCtx* c, const NxgPubTable* tab, const NxgColumns* batch,
                        const uint8_t* heap, const uint8_t* kind, const uint32_t* to_client,
                        NxgDispatch* out, NetidxError* err) {
    if (!c || !tab || !batch || !out || !out->chan_off) {
        set_err(err, "null argument");
        return false;
    }
    const uint64_t n = batch->n_rows;
    if (n && (!batch->id || !batch->fixed || !kind || !to_client)) {
        set_err(err, "null batch column, kind or to_client");
        return false;
    }
    if ((tab->n_ids && !tab->slot_of_id) ||
        (tab->n_slots && (!tab->slot_client_off || !tab->cur_fixed || !out->last_row)) ||
        (out->cap_entries && (!out->ent_sub || !out->ent_row))) {
        set_err(err, "null table or output array");
        return false;
    }
    if (n >= 0xffffffffull) {
        set_err(err, "publish batches are limited to 2^32 - 1 rows");
        return false;
    }
    HIPCHK(hipSetDevice(c->device));
    const size_t pub = (nxg_pub_scratch_bytes(n, tab->n_slots) + 255) & ~size_t(255);
    const size_t need = pub + 64 + nxg_disp_scratch_bytes(n, tab->n_clients);
    if (need > c->dscratch_cap) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->dscratch) HIPCHK(hipFree(c->dscratch));
        c->dscratch = nullptr;
        const size_t sz = std::max(need, c->dscratch_cap * 2);
        HIPCHK(hipMalloc(&c->dscratch, sz));
        c->dscratch_cap = sz;
    }
    const NxgPubBatch b{batch->id,    batch->tag,   batch->fixed, batch->aux, batch->ctag,
                        batch->cfixed, batch->caux, heap,         kind,       n};
    HIPCHK(nxg_launch_pub_stage1(*tab, b, c->dscratch, c->ncu, c->stream));
    uint32_t flags[4] = {0, 0, 0, 0};
    HIPCHK(hipMemcpyAsync(flags, nxg_pub_flags(c->dscratch), 12, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const uint8_t* mode = nullptr;
    HIPCHK(nxg_launch_pub_stage2(*tab, b, c->dscratch, flags[0] != 0, flags[1] != 0, c->ncu,
                                 c->stream, &mode));
    if (flags[1]) {
        uint32_t f23[2] = {0, 0};
        HIPCHK(hipMemcpyAsync(f23, nxg_pub_flags(c->dscratch) + 2, 8, hipMemcpyDeviceToHost,
                              c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (f23[1]) {  // Decimal / container / Abstract comparisons: the stack-walk kernel
            const uint32_t* prev =
                flags[0] ? nxg_pub_prev(c->dscratch, n, tab->n_slots) : nullptr;
            HIPCHK(nxg_launch_pub_deep(*tab, b, c->dscratch, prev, c->ncu, c->stream));
            HIPCHK(hipMemcpyAsync(f23, nxg_pub_flags(c->dscratch) + 2, 4, hipMemcpyDeviceToHost,
                                  c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
        }
        flags[2] = f23[0];
        if (flags[2]) {
            set_err(err, "NXG_UNSUPPORTED: an UpdateChanged compares values nested deeper than "
                         "%d levels, or a container whose columns have no children",
                    NXG_MAX_DEPTH);
            return false;
        }
    } else {
        mode = kind;  // Update(None) = 0 and Update(Some(cl)) = 2 route as they are
    }
    // the client fan-out is the subscriber dispatch with per-row routing: clients as channels,
    // entries tagged with the row's Id, every slot tracking `current`
    const NxgSubTable st{tab->n_ids, tab->slot_of_id, tab->n_slots, nullptr, tab->slot_client_off,
                         tab->client, nullptr, tab->n_clients};
    uint8_t* ds = c->dscratch + pub;
    uint64_t* um = reinterpret_cast<uint64_t*>(ds);
    HIPCHK(nxg_launch_dispatch(st, batch->id, n, ds + 64, out->chan_off, out->ent_sub, out->ent_row,
                               out->cap_entries, out->last_row, um, c->ncu, c->stream, mode,
                               to_client));
    uint64_t res[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(&res[0], out->chan_off + tab->n_clients, 8, hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipMemcpyAsync(&res[1], um, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    out->n_entries = res[0];
    out->n_unmatched = res[1];
    if (res[0] > out->cap_entries) {
        set_err(err, "publish needs %llu entries, capacity is %llu", (unsigned long long)res[0],
                (unsigned long long)out->cap_entries);
        return false;
    }
    return true;
}

// the commit's unsubscribes (publisher/mod.rs:820-832): every pair routes to its client (row
// mode 2 of the dispatch), so each client's list keeps queue order
bool nxg_publish_unsubscribes(NxgCtx* c, const uint64_t* id, const uint32_t* client, uint64_t n,
                              uint32_t n_clients, NxgDispatch* out, NetidxError* err) {
    if (!c || !out || !out->chan_off || (n && (!id || !client)) ||
        (out->cap_entries && (!out->ent_sub || !out->ent_row))) {
        set_err(err, "null argument");
        return false;
    }
    if (n >= 0xffffffffull) {
        set_err(err, "unsubscribe lists are limited to 2^32 - 1 pairs");
        return false;
    }
    HIPCHK(hipSetDevice(c->device));
    const size_t mode_bytes = (n + 255) & ~uint64_t(255);
    const size_t need = mode_bytes + 64 + nxg_disp_scratch_bytes(n, n_clients);
    if (need > c->dscratch_cap) {
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->dscratch) HIPCHK(hipFree(c->dscratch));
        c->dscratch = nullptr;
        const size_t sz = std::max(need, c->dscratch_cap * 2);
        HIPCHK(hipMalloc(&c->dscratch, sz));
        c->dscratch_cap = sz;
    }
    uint8_t* mode = c->dscratch;
    if (n) HIPCHK(hipMemsetAsync(mode, 2, n, c->stream));
    const NxgSubTable st{0, nullptr, 0, nullptr, nullptr, nullptr, nullptr, n_clients};
    uint8_t* ds = c->dscratch + mode_bytes;
    uint64_t* um = reinterpret_cast<uint64_t*>(ds);
    HIPCHK(nxg_launch_dispatch(st, id, n, ds + 64, out->chan_off, out->ent_sub, out->ent_row,
                               out->cap_entries, nullptr, um, c->ncu, c->stream, mode, client));
    uint64_t total = 0;
    HIPCHK(hipMemcpyAsync(&total, out->chan_off + n_clients, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    out->n_entries = total;
    out->n_unmatched = 0;
    if (total > out->cap_entries) {
        set_err(err, "unsubscribes need %llu entries, capacity is %llu", (unsigned long long)total,
                (unsigned long long)out->cap_entries);
        return false;
    }
    return true;
}

bool nxg_encoded_len(NxgCtx* c, const NxgColumns* in, const uint8_t* heap, uint64_t* len_out,
                     NetidxError* err) {
    return encode_impl(c, in, heap, nullptr, 0, len_out, err);
}

bool nxg_encode_updates(NxgCtx* c, const NxgColumns* in, const uint8_t* heap, uint8_t* out,
                        uint64_t cap, uint64_t* len_out, NetidxError* err) {
    if (!out) {
        set_err(err, "null output buffer");
        return false;
    }
    return encode_impl(c, in, heap, out, cap, len_out, err);
}

bool nxg_encode_updates_async(NxgCtx* c, const NxgColumns* din, const uint8_t* dheap,
                              uint8_t* dout, uint64_t cap, uint64_t* len_out, NetidxError* err) {
    if (!c || !din || !dout) {
        set_err(err, "null argument");
        return false;
    }
    if (c->pending.size() >= kStatusRing / 2) {
        set_err(err, "too many in-flight async calls (max %d); call nxg_ctx_sync", kStatusRing / 2);
        return false;
    }
    // the control-span prefix lives in shared ctx scratch: one such encode in flight at a time
    for (auto& p : c->pending)
        if (p.kind == 2 && din->layout == NXG_LAYOUT_MIXED && din->n_ctl) {
            set_err(err, "sync the previous encode before an async encode with control spans");
            return false;
        }
    DevStatus* st;
    uint32_t slot;
    if (!begin_call(c, &st, &slot, err)) return false;
    int fast = 0;
    const bool ok = enqueue_encode(c, din, dheap, dout, cap, st, err, &fast);
    if (!end_call(c, err) || !ok) return false;
    c->pending.push_back({2, fast, nullptr, 0, const_cast<NxgColumns*>(din), len_out, cap, st,
                          slot, 0, dheap, dout});
    return true;
}

bool nxg_encode_frames(NxgCtx* c, const NxgColumns* in, const uint8_t* heap, uint8_t* out,
                       uint64_t cap, uint64_t* len_out, uint64_t* chunk_len_out,
                       uint64_t cap_chunks, uint64_t* n_chunks, NetidxError* err) {
    if (!out || !n_chunks || (cap_chunks && !chunk_len_out)) {
        set_err(err, "null argument");
        return false;
    }
    uint64_t total = 0;
    if (!encode_impl(c, in, heap, out, cap, &total, err)) return false;
    if (len_out) *len_out = total;
    uint64_t ch[2];
    uint64_t k = 0;
    if (total == 0) {
        k = 0;
    } else if (total <= kMaxBatch) {
        ch[k++] = total;
    } else {
        if (!c->last_split) {
            set_err(err, "frame split: the encoder recorded no boundary for a %llu-byte batch",
                    (unsigned long long)total);
            return false;
        }
        const uint64_t c1 = c->last_split - 1;
        // the next cut is before the first message ending past MAX_BATCH + c1 (channel.rs:187)
        if (total > kMaxBatch + c1) {
            set_err(err, "frame split: a %llu-byte batch needs more than one cut (the reference "
                         "then cuts before every message); split the batch or use "
                         "nxg_frame_split with the message lengths", (unsigned long long)total);
            return false;
        }
        ch[k++] = c1;
        ch[k++] = total - c1;
    }
    if (k > cap_chunks) {
        set_err(err, "frame split: %llu frames, capacity %llu", (unsigned long long)k,
                (unsigned long long)cap_chunks);
        return false;
    }
    for (uint64_t i = 0; i < k; i++) chunk_len_out[i] = ch[i];
    *n_chunks = k;
    return true;
}

// ---- byte-range decode (multi-GPU) ---------------------------------------------------------------
bool nxg_decode_range(NxgCtx* c, const uint8_t* dframe, uint64_t W, uint64_t begin, uint64_t end,
                      NxgColumns* out, NxgRange* rng, NetidxError* err) {
    if (!c || !out || !rng || (!dframe && W)) {
        set_err(err, "null argument");
        return false;
    }
    if (begin > end || end > W) {
        set_err(err, "bad range [%llu, %llu) of a %llu-byte frame", (unsigned long long)begin,
                (unsigned long long)end, (unsigned long long)W);
        return false;
    }
    if (!c->pending.empty()) {
        set_err(err, "an async operation is pending on this ctx; call nxg_ctx_sync first");
        return false;
    }
    if (out->mem != NXG_MEM_DEVICE || !is_device_ptr(dframe)) {
        set_err(err, "range decode needs a device frame and device columns");
        return false;
    }
    if (!set_device(c, err)) return false;
    memset(rng, 0, sizeof *rng);
    rng->begin = begin;
    rng->end = end;
    if (begin == end) {  // an empty range: the chain passes through; linked as identity
        rng->entry = rng->exit = ~0ull;
        rng->ok = 1;
        return true;
    }
    const uint64_t R = end - begin;
    DevStatus* st;
    uint32_t slot;
    if (!begin_call(c, &st, &slot, err)) return false;
    bool ok = ensure_tstat(c, nxg_dec_f64r_groups(R), err) &&
              ensure_rdesc(c, 16 * nxg_dec_f64r_tiles(R), err);
    if (ok) {
        const hipError_t e = nxg_launch_dec_f64r(dframe, W, begin, end, out->id, out->fixed,
                                                 out->cap_rows, c->rdesc, c->tstat, c->epoch,
                                                 c->f64r_flags, st, c->stream);
        if (e != hipSuccess) {
            set_err(err, "range decode launch: %s", hipGetErrorString(e));
            ok = false;
        }
    }
    if (!end_call(c, err) || !ok) return false;
    const uint64_t nt = nxg_dec_f64r_tiles(R);
    uint8_t d0[16], dl[16];
    HIPCHK(hipMemcpyAsync(c->hst + slot, st, sizeof(DevStatus), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(d0, c->rdesc, 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(dl, c->rdesc + 16 * (nt - 1), 16, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    const DevStatus& h = c->hst[slot];
    if (h.timeout) {
        set_err(err, "device look-back watchdog expired");
        return false;
    }
    // (a copy: later attempts take other ring slots)
    const DevStatus h0 = h;
    c->last = h0;
    bool declined = h0.fast_fail != 0;
    if (declined && (h0.irregular & 3u) == 1u) {
        // record lengths that vary record to record (ids in any order: a batch updating an
        // arbitrary subset of a publisher's values): the single-pass decoder in range mode
        DevStatus* st2;
        uint32_t slot2;
        if (!begin_call(c, &st2, &slot2, err)) return false;
        bool ok2 = ensure_tstat(c, nxg_dec_f64x_groups(R), err);
        if (ok2) {
            const hipError_t e = nxg_launch_dec_f64x_range(dframe, W, begin, end, out->id,
                                                           out->fixed, out->cap_rows, c->tstat,
                                                           c->epoch, st2, c->stream);
            if (e != hipSuccess) {
                set_err(err, "range decode launch: %s", hipGetErrorString(e));
                ok2 = false;
            }
        }
        if (!end_call(c, err) || !ok2) return false;
        HIPCHK(hipMemcpyAsync(c->hst + slot2, st2, sizeof(DevStatus), hipMemcpyDeviceToHost,
                              c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        const DevStatus& h2 = c->hst[slot2];
        c->last = h2;
        if (!h2.fast_fail && h2.diag[2] && h2.diag[3]) {
            rng->entry = begin + h2.diag[2] - 1;
            rng->exit = begin + h2.diag[3] - 1;
            rng->n_rows = h2.n_rows;
            rng->ok = 1;
            rng->err_kind = h2.capacity ? NXG_CAPACITY : 0;
            out->n_rows = h2.n_rows;
            out->layout = NXG_LAYOUT_F64;
            return true;
        }
    }
    if (declined && mixed_capable(out) && R < (1ull << 32)) {
        // not an f64 frame: the fast mixed decoder in range mode (frames of short Updates and
        // Heartbeats; anything it declines is ok = 0, for the caller to decode whole)
        DevStatus* st2;
        uint32_t slot2;
        if (!begin_call(c, &st2, &slot2, err)) return false;
        const ColsDesc d = desc_of(out);
        bool ok2 = ensure_glws(c, nxg_fmx_scratch_bytes(R), err);
        if (ok2) {
            const hipError_t e = nxg_launch_dec_fmx_range(dframe, W, begin, end, d,
                                                          reinterpret_cast<uint8_t*>(c->glws),
                                                          c->wgs_fmx, st2, c->stream);
            if (e != hipSuccess) {
                set_err(err, "range decode launch: %s", hipGetErrorString(e));
                ok2 = false;
            }
        }
        if (!end_call(c, err) || !ok2) return false;
        HIPCHK(hipMemcpyAsync(c->hst + slot2, st2, sizeof(DevStatus), hipMemcpyDeviceToHost,
                              c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        const DevStatus& h2 = c->hst[slot2];
        c->last = h2;
        if (h2.fast_fail || h2.path != 4 || !h2.diag[2] || !h2.diag[3]) {  // ok = 0
            if (h2.capacity) rng->err_kind = NXG_CAPACITY;  // declined: the columns are short
            return true;
        }
        rng->entry = begin + h2.diag[2] - 1;
        rng->exit = begin + h2.diag[3] - 1;
        rng->n_rows = h2.n_rows;
        rng->ok = 1;
        out->n_rows = h2.n_rows;
        out->n_children = h2.n_children;
        out->n_ctl = h2.n_ctl;
        out->n_heartbeat = h2.n_heartbeat;
        out->layout = NXG_LAYOUT_MIXED;
        return true;
    }
    if (declined) return true;  // ok = 0: not a range these decoders take
    // Desc: base u64 | count u16 | ks u16 | x u16 | entry u8 | mode u8 (nxg_decode_f64_run.hip)
    uint16_t xl;
    memcpy(&xl, dl + 12, 2);
    rng->entry = begin + d0[14];
    rng->exit = begin + (nt - 1) * nxg_dec_f64r_tile_bytes() + xl;
    rng->n_rows = h.n_rows;
    rng->ok = 1;
    rng->err_kind = h.capacity ? NXG_CAPACITY : 0;
    out->n_rows = h.n_rows;
    out->layout = NXG_LAYOUT_F64;
    return true;
}

bool nxg_range_link(const NxgRange* r, uint32_t n, uint64_t W, uint64_t* row_off, uint32_t* bad,
                    NetidxError* err) {
    if (!r || (n && !row_off)) {
        set_err(err, "null argument");
        return false;
    }
    uint64_t at = 0, rows = 0;  // where the chain is, rows so far
    uint64_t expect_begin = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (r[i].begin != expect_begin || r[i].end < r[i].begin || !r[i].ok) {
            if (bad) *bad = i;
            set_err(err, "range %u is not the next contiguous, decoded range", i);
            return false;
        }
        expect_begin = r[i].end;
        row_off[i] = rows;
        if (r[i].begin == r[i].end) continue;  // empty: the chain passes through
        if (r[i].entry != at) {
            if (bad) *bad = i;
            set_err(err, "range %u enters the chain at %llu, its predecessor leaves at %llu", i,
                    (unsigned long long)r[i].entry, (unsigned long long)at);
            return false;
        }
        at = r[i].exit;
        rows += r[i].n_rows;
    }
    if (expect_begin != W || at != W) {
        if (bad) *bad = n ? n - 1 : 0;
        set_err(err, "the ranges cover [0, %llu) and the chain ends at %llu; the frame has %llu "
                     "bytes", (unsigned long long)expect_begin, (unsigned long long)at,
                (unsigned long long)W);
        return false;
    }
    return true;
}

// ---- one share of a frame's rows (nxg_decode_sharded's fallback) --------------------------------
// The frame decoded whole (every decoder in turn, as nxg_decode_updates), into ctx-owned device
// columns sized `shares` times the caller's (each rank's share should fit its own columns), or to
// the frame's totals when that is short; then rows [N*share/shares, N*(share+1)/shares) with their
// children and the control spans before them (the last share: also those after the last row)
// into `out`, re-based (nxg_share.hip).
bool nxg_decode_share(NxgCtx* c, const uint8_t* dframe, uint64_t W, uint32_t share,
                      uint32_t shares, NxgColumns* out, uint64_t* row_off, NxgStatus* ust,
                      NetidxError* err) {
    if (!c || !out || (!dframe && W) || shares == 0 || share >= shares) {
        set_err(err, "bad argument (share %u of %u)", share, shares);
        return false;
    }
    if (!c->pending.empty()) {
        set_err(err, "an async operation is pending on this ctx; call nxg_ctx_sync first");
        return false;
    }
    if (W >= (1ull << 40)) {
        set_err(err, "frame too large (%llu bytes)", (unsigned long long)W);
        return false;
    }
    if (out->mem != NXG_MEM_DEVICE || (W && !is_device_ptr(dframe))) {
        set_err(err, "share decode needs a device frame and device columns");
        return false;
    }
    if (!set_device(c, err)) return false;
    if (row_off) *row_off = 0;
    // the whole-frame columns: the caller's shape, `shares` times its capacities (at most the
    // frame's bounds, include/nxg_codec.h), grown to the frame's totals after a capacity miss
    auto times = [&](uint64_t x, uint64_t bound) {
        return std::max<uint64_t>(1, std::min<uint64_t>(x > bound / shares ? bound : x * shares, bound));
    };
    NxgColumns like = *out;
    like.cap_rows = times(out->cap_rows, W / 4 + 1);
    like.cap_children = times(out->cap_children, W + 1);
    like.cap_ctl = times(out->cap_ctl, W / 2 + 1);
    NxgColumns v{};
    NxgStatus s{};
    for (int attempt = 0;; attempt++) {
        if (!ensure_dcols(c, &like, err)) return false;
        v = staged_view(c, &like);
        DevStatus* st;
        uint32_t slot;
        if (!begin_call(c, &st, &slot, err)) return false;
        int fast = FAST_NONE;
        const bool ok = enqueue_dec_fast(c, dframe, W, &v, st, &fast, err);
        if (!end_call(c, err) || !ok) return false;
        if (!finish_decode(c, dframe, W, &v, fast, st, slot, &s, err)) return false;
        if (s.err_kind != NXG_CAPACITY || attempt == 2) break;
        const uint64_t r = std::min<uint64_t>(std::max(s.n_rows, 2 * like.cap_rows), W / 4 + 1);
        const uint64_t k = std::min<uint64_t>(std::max(s.n_children, 2 * like.cap_children), W + 1);
        const uint64_t q = std::min<uint64_t>(std::max(s.n_ctl, 2 * like.cap_ctl), W / 2 + 1);
        if (r == like.cap_rows && k == like.cap_children && q == like.cap_ctl) break;
        like.cap_rows = r;
        like.cap_children = k;
        like.cap_ctl = q;
    }
    NxgStatus o{};
    o.path = s.path;
    o.err_kind = s.err_kind;
    o.err_offset = s.err_offset;
    if (s.err_kind) {  // the frame fails as a whole (connection.rs:228-231): no rows in any share
        out->n_rows = out->n_children = out->n_ctl = out->n_heartbeat = 0;
        if (ust) *ust = o;
        return true;
    }
    const uint64_t N = s.n_rows;
    const uint64_t r0 = (uint64_t)((unsigned __int128)N * share / shares);
    const uint64_t r1 = (uint64_t)((unsigned __int128)N * (share + 1) / shares);
    const bool last = share + 1 == shares;
    const bool f64_rows = s.path == 1 || !mixed_capable(&v);  // tag / children not written
    ColsDesc src = desc_of(&v);
    src.n_rows = N;
    src.n_children = f64_rows ? 0 : s.n_children;
    src.n_ctl = f64_rows ? 0 : s.n_ctl;
    if (f64_rows) src.tag = nullptr;
    uint64_t c0 = 0, c1 = 0, k0 = 0, k1 = 0;
    if (!ensure_escratch(c, 8, err)) return false;
    if (!f64_rows && (src.n_children || src.n_ctl)) {
        uint64_t b[4];
        HIPCHK(nxg_launch_share_bounds(src, r0, r1, c->escratch, c->stream));
        HIPCHK(hipMemcpyAsync(b, c->escratch, sizeof b, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        c0 = std::min<uint64_t>(b[0], src.n_children);
        c1 = std::min<uint64_t>(b[1], src.n_children);
        k0 = std::min<uint64_t>(b[2], src.n_ctl);
        k1 = last ? src.n_ctl : std::min<uint64_t>(b[3], src.n_ctl);
    }
    const uint64_t nr = r1 - r0, nc = c1 - c0, nk = k1 - k0;
    if (nr > out->cap_rows || nc > out->cap_children || nk > out->cap_ctl ||
        ((nc || nk) && !mixed_capable(out))) {
        o.err_kind = (nc || nk) && !mixed_capable(out) ? NXG_NOT_F64 : NXG_CAPACITY;
        o.n_rows = nr;
        o.n_children = nc;
        o.n_ctl = nk;
        out->n_rows = out->n_children = out->n_ctl = out->n_heartbeat = 0;
        if (ust) *ust = o;
        return true;
    }
    ColsDesc dst = desc_of(out);
    if (f64_rows) dst.tag = nullptr;
    HIPCHK(nxg_launch_share_copy(src, dst, r0, nr, c0, nc, k0, nk, c->escratch + 4, c->stream));
    uint64_t hb = 0;
    HIPCHK(hipMemcpyAsync(&hb, c->escratch + 4, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    out->n_rows = nr;
    out->n_children = nc;
    out->n_ctl = nk;
    out->n_heartbeat = hb;
    out->layout = f64_rows ? NXG_LAYOUT_F64 : NXG_LAYOUT_MIXED;
    o.n_rows = nr;
    o.n_children = nc;
    o.n_ctl = nk;
    o.n_heartbeat = hb;
    if (row_off) *row_off = r0;
    if (ust) *ust = o;
    return true;
}

// ---- host framing ------------------------------------------------------------------------

// WriteChannel::queue_send (channel.rs:177-202) + try_flush (237-257). `boundries` holds chunk
// LENGTHS. A new boundary is recorded when (buf_len - last boundary length) + len > MAX_BATCH,
// i.e. the comparison uses the last chunk's length, not the sum (channel.rs:187-190).
int64_t nxg_frame_split(const uint64_t* msg_len, uint64_t n_msgs, uint64_t* chunk_len_out,
                        uint64_t cap_chunks) {
    const uint64_t MAX_BATCH = 0x3FFFFFFF;
    uint64_t buf_len = 0, sum_b = 0, last_b = 0, nb = 0;
    for (uint64_t i = 0; i < n_msgs; i++) {
        const uint64_t len = msg_len[i];
        if (len > MAX_BATCH) return -1;
        if ((buf_len - (nb ? last_b : 0)) + len > MAX_BATCH) {
            const uint64_t b = buf_len - sum_b;
            if (nb >= cap_chunks) return -1;
            chunk_len_out[nb++] = b;
            sum_b += b;
            last_b = b;
        }
        buf_len += len;
    }
    if (buf_len > sum_b) {
        if (nb >= cap_chunks) return -1;
        chunk_len_out[nb++] = buf_len - sum_b;
    }
    return (int64_t)nb;
}

// flush_buf (channel.rs:107-126)
void nxg_frame_header(uint32_t payload_len, bool encrypted, uint8_t out[4]) {
    const uint32_t v = encrypted ? (payload_len | 0x80000000u) : payload_len;
    out[0] = (uint8_t)(v >> 24);
    out[1] = (uint8_t)(v >> 16);
    out[2] = (uint8_t)(v >> 8);
    out[3] = (uint8_t)v;
}

// read_task (channel.rs:389-398): hdr > LEN_MASK => encrypted, len = hdr & LEN_MASK
uint32_t nxg_frame_parse_header(const uint8_t* buf, uint64_t avail, uint32_t* payload_len,
                                bool* encrypted) {
    if (avail < 4) return 0;
    const uint32_t hdr = ((uint32_t)buf[0] << 24) | ((uint32_t)buf[1] << 16) |
                         ((uint32_t)buf[2] << 8) | buf[3];
    *encrypted = hdr > 0x7FFFFFFFu;
    *payload_len = hdr & 0x7FFFFFFFu;
    return 4;
}

// ---- read_task's frame assembly (channel.rs:379-443) -------------------------------------------
struct NxgFrameReader {
    std::vector<uint8_t> buf;  // bytes read from the socket, not yet handed out
    size_t head = 0;           // start of the unconsumed bytes
};

NxgFrameReader* nxg_frame_reader_new(NetidxError* err) {
    try {
        return new NxgFrameReader();
    } catch (...) {
        set_err(err, "out of memory");
        return nullptr;
    }
}

void nxg_frame_reader_free(NxgFrameReader* r) { delete r; }

bool nxg_frame_reader_push(NxgFrameReader* r, const uint8_t* data, uint64_t len,
                           NetidxError* err) {
    if (!r || (len && !data)) {
        set_err(err, "null argument");
        return false;
    }
    // drop what was handed out before growing (payload pointers from _next end here)
    if (r->head) {
        r->buf.erase(r->buf.begin(), r->buf.begin() + (ptrdiff_t)r->head);
        r->head = 0;
    }
    try {
        r->buf.insert(r->buf.end(), data, data + len);
    } catch (...) {
        set_err(err, "out of memory");
        return false;
    }
    return true;
}

int nxg_frame_reader_next(NxgFrameReader* r, const uint8_t** payload, uint64_t* len,
                          NetidxError* err) {
    if (!r || !payload || !len) {
        set_err(err, "null argument");
        return -1;
    }
    const uint64_t avail = r->buf.size() - r->head;
    uint32_t plen = 0;
    bool enc = false;
    if (!nxg_frame_parse_header(r->buf.data() + r->head, avail, &plen, &enc)) return 0;
    if (avail - 4 < plen) return 0;  // "less than batch len, reading more"
    if (enc) {  // no security context here (krb5 is out of scope): channel.rs:420-422
        set_err(err, "encryption is not supported");
        return -1;
    }
    *payload = r->buf.data() + r->head + 4;
    *len = plen;
    r->head += 4 + (size_t)plen;
    return 1;
}

uint64_t nxg_frame_reader_buffered(const NxgFrameReader* r) {
    return r ? r->buf.size() - r->head : 0;
}

}  // extern "C"
