/*
 * nxg_codec.h -- C ABI of the MI355X-native netidx batch-update codec.
 *
 * The reference codec is the generic Rust `trait Pack` (netidx-core/src/pack.rs:149-165). It is
 * called once per message at two seams:
 *
 *   encode: ClientCtx::handle_updates   netidx/src/publisher/server.rs:604-629
 *           -> WriteChannel::queue_send netidx/src/channel.rs:177-202
 *           -> <From as Pack>::encode   (netidx-derive/src/lib.rs:289-381)
 *   decode: decode_task                 netidx/src/subscriber/connection.rs:209-242
 *           -> ReadChannel::receive_batch_fn   netidx/src/channel.rs:504-521
 *           -> <From as Pack>::decode   (netidx-derive/src/lib.rs:482-601)
 *
 * This ABI replaces each of those per-message loops with ONE batch call. Each call covers all
 * the messages of one frame payload, executed by hand-written gfx950 HIP kernels. The wire bytes
 * are identical to the reference.
 *
 * Conventions follow netidx-ffi (netidx-ffi/netidx.h, netidx-ffi/src/error.rs:19-29):
 * - fallible calls return `bool`;
 * - on failure they fill a caller-provided `NetidxError*` whose `msg` must be released with
 *   nxg_error_free;
 * - handles are opaque.
 *
 * Threading: an NxgCtx is not internally synchronised. Use one ctx per connection/thread. Each ctx
 * owns one HIP stream (or a caller-provided one).
 *
 * Columnar layout (the decode output and the encode input):
 *
 *   rows (one per From::Update, in wire order):
 *     id    u64  publisher::Id (netidx-netproto/src/publisher.rs:7)
 *     tag   u8   Value wire tag (netidx-value/src/lib.rs:361-468); 17 is normalised to 16, and
 *                Error(String) is always 18
 *     fixed u64  scalar payload: integers (signed values sign-extended), f32/f64 bit patterns,
 *                DateTime/Duration seconds, bool as 1/0; for String/Bytes/Error(String)/Decimal/
 *                Abstract: byte offset of the payload in the heap (decode: the frame itself);
 *                for Array/Map/Error(Value): index of the first child slot
 *     aux   u32  DateTime/Duration nanoseconds; byte length of String/Bytes/Decimal/Abstract;
 *                element count of Array, entry count of Map, 1 for Error(Value)
 *   children (elements of Array, key/value pairs of Map, inner of Error(Value)): ctag/cfixed/
 *     caux with the same meaning. Each container's elements are contiguous, allocated
 *     depth-first.
 *   ctl (every other From message, with Heartbeat included, kept as validated raw spans):
 *     ctl_row     index of the first Update row that follows it
 *     ctl_off     byte offset of the message in the frame
 *     ctl_len     byte length of the message
 *     ctl_variant From variant (0 NoSuchValue, 1 Denied, 2 Unsubscribed, 3 Subscribed,
 *                 5 Heartbeat, 6 WriteResult)
 *
 * NXG_LAYOUT_F64 is the homogeneous fast path. It is valid only when every message is
 * From::Update with an F64 value. Only id and fixed (the f64 bits) are meaningful; tag is
 * implicitly 9.
 */
#ifndef NXG_CODEC_H
#define NXG_CODEC_H
#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* netidx-ffi/netidx.h:162-164 */
typedef struct NetidxError {
    char* msg;
} NetidxError;

typedef struct NxgCtx NxgCtx;

/* PackError (netidx-core/src/pack.rs:89-95) plus codec-level kinds */
enum NxgErrKind {
    NXG_OK = 0,
    NXG_UNKNOWN_TAG = 1,
    NXG_TOO_BIG = 2,
    NXG_INVALID_FORMAT = 3,
    NXG_BUFFER_SHORT = 4,
    NXG_DEPTH = 6,    /* Value nesting deeper than NXG_MAX_DEPTH (documented deviation) */
    NXG_CAPACITY = 7, /* output columns too small */
    NXG_NOT_F64 = 8,  /* valid batch, but F64-only columns were supplied for mixed content */
    NXG_TIMEOUT = 9,  /* device-side progress watchdog fired (should never happen) */
    NXG_UNSUPPORTED = 10, /* publish: an UpdateChanged comparison of values nested deeper than
                             NXG_MAX_DEPTH levels (every Value variant's equality is implemented,
                             netidx-value/src/op.rs:133-172) */
};

#define NXG_MAX_DEPTH 32

enum NxgLayout { NXG_LAYOUT_F64 = 1, NXG_LAYOUT_MIXED = 2 };
enum NxgMem { NXG_MEM_DEVICE = 0, NXG_MEM_HOST = 1 /* pinned host */ };
enum NxgDecodeFlags {
    NXG_DECODE_DEFAULT = 0,
    NXG_DECODE_HINT_MIXED = 1, /* skip the homogeneous-f64 attempt */
};

typedef struct NxgColumns {
    uint32_t layout; /* NxgLayout: alloc-time capability; after decode, what was written */
    uint32_t mem;    /* NxgMem */
    uint64_t cap_rows, cap_children, cap_ctl;
    uint64_t n_rows, n_children, n_ctl, n_heartbeat;
    uint64_t* id;
    uint8_t* tag;
    uint64_t* fixed;
    uint32_t* aux;
    uint8_t* ctag;
    uint64_t* cfixed;
    uint32_t* caux;
    uint64_t* ctl_row;
    uint64_t* ctl_off;
    uint32_t* ctl_len;
    uint8_t* ctl_variant;
} NxgColumns;

typedef struct NxgStatus {
    uint64_t n_rows, n_children, n_ctl, n_heartbeat;
    int32_t err_kind;    /* NxgErrKind of the FIRST failing message (reference is sequential) */
    uint32_t path;       /* 1 = homogeneous-f64 kernel, 2 = general kernel, 4 = fast mixed kernel */
    uint64_t err_offset; /* byte offset of the first failing message */
} NxgStatus;

/* ---- lifetime -------------------------------------------------------------------------- */
NxgCtx* nxg_ctx_new(int device, NetidxError* err);
void nxg_ctx_destroy(NxgCtx* ctx);
/* Use `hip_stream` (a hipStream_t) instead of the ctx's own stream; NULL restores it. */
bool nxg_ctx_set_stream(NxgCtx* ctx, void* hip_stream, NetidxError* err);
void* nxg_ctx_stream(NxgCtx* ctx);
void nxg_error_free(NetidxError* err);
/* library version string, e.g. "nxg 0.1.0 gfx950" */
const char* nxg_version(void);

/* ---- columns ------------------------------------------------------------------------------
 * layout F64 allocates id+fixed only; MIXED allocates every array. mem: device or pinned host.
 * Capacity bounds for a frame of W bytes: rows <= W/4 (the smallest Update, `04 04 00 10`),
 * children <= W, ctl <= W/2 (`02 05`). */
bool nxg_columns_alloc(NxgCtx* ctx, uint32_t layout, uint64_t cap_rows, uint64_t cap_children,
                       uint64_t cap_ctl, uint32_t mem, NxgColumns* out, NetidxError* err);
void nxg_columns_free(NxgCtx* ctx, NxgColumns* cols);

/* ---- decode: replaces decode_task's receive_batch_fn loop (connection.rs:209-242) ---------
 * `frame` is one frame payload (no u32 header; channel.rs:379-443 strips it), host or device
 * memory. `out` must come from nxg_columns_alloc. Synchronous. Returns false only on API
 * misuse or a HIP failure. A malformed frame returns true with st->err_kind != 0, and the whole
 * frame is rejected, as in connection.rs:228-231. */
bool nxg_decode_updates(NxgCtx* ctx, const uint8_t* frame, uint64_t len, NxgColumns* out,
                        uint32_t flags, NxgStatus* st, NetidxError* err);
/* Asynchronous device-resident variant: enqueue on the ctx stream; no host sync. Only the
 * path selected up front runs (flags). nxg_ctx_sync completes it, runs the general fallback if
 * the homogeneous path rejected the frame, and fills the status. At most 512 async calls
 * (decode and encode together) may be in flight between syncs; the next one fails. A frame must
 * stay unchanged until nxg_ctx_sync: a fallback re-reads it there, after every later call has
 * run, and a later call of the backlog that wrote into it makes nxg_ctx_sync fail that decode
 * with an error (it never decodes the overwritten bytes). */
bool nxg_decode_updates_async(NxgCtx* ctx, const uint8_t* dframe, uint64_t len, NxgColumns* dout,
                              uint32_t flags, NetidxError* err);
bool nxg_ctx_sync(NxgCtx* ctx, NxgStatus* st, NetidxError* err);
/* A connection's backlog of frames (read_task hands decode_task frame after frame over a
 * channel, channel.rs:379-443 / connection.rs:209-242): n device frames, each decoded into its own
 * device columns (outs[j]; the same columns may be passed for several frames, the later frame then
 * overwrites them), in order, as n nxg_decode_updates_async calls would. Every frame must be
 * complete in device memory when the call is made (work still queued on the ctx stream may not
 * produce it). On the homogeneous-f64 path the frames are pipelined: the record-length probe of
 * frame j + 1 runs in the same launch as the column emit of frame j. nxg_ctx_sync completes them
 * (and reruns any frame the fast path rejected); every frame counts as one in-flight call. */
bool nxg_decode_frames_async(NxgCtx* ctx, uint32_t n, const uint8_t* const* dframes,
                             const uint64_t* lens, NxgColumns* const* douts, uint32_t flags,
                             NetidxError* err);

/* ---- encode: replaces handle_updates' queue_send loop (server.rs:610-612) ----------------
 * `heap` holds the bytes that string/bytes/decimal/abstract offsets and ctl spans refer to.
 * It may be NULL for pure fixed-width columns. in/heap/out must all be device memory, or all
 * host memory. */
bool nxg_encoded_len(NxgCtx* ctx, const NxgColumns* in, const uint8_t* heap, uint64_t* len_out,
                     NetidxError* err);
bool nxg_encode_updates(NxgCtx* ctx, const NxgColumns* in, const uint8_t* heap, uint8_t* out,
                        uint64_t cap, uint64_t* len_out, NetidxError* err);
/* Async device-resident variant (len_out is written at nxg_ctx_sync time). */
bool nxg_encode_updates_async(NxgCtx* ctx, const NxgColumns* din, const uint8_t* dheap,
                              uint8_t* dout, uint64_t cap, uint64_t* len_out, NetidxError* err);
/* nxg_encode_updates plus the frame split of WriteChannel::queue_send + try_flush
 * (netidx/src/channel.rs:177-202, 237-257): the payload is cut before the message that would take
 * a frame past MAX_BATCH = 0x3FFFFFFF bytes, so `out` holds the frames' payloads back to back and
 * chunk_len_out[0 .. *n_chunks) their lengths (each goes out behind its own u32 header,
 * nxg_frame_header). The encode kernels record the cut themselves (the message holding byte
 * MAX_BATCH). Batches that would need a second cut (more than MAX_BATCH + the first chunk's
 * length, about 2 GiB) are refused: the reference then cuts before every further message
 * (channel.rs:187 compares against the last chunk's length), which nxg_frame_split reproduces
 * from message lengths. An empty batch gives no frame, as try_flush sends nothing. */
bool nxg_encode_frames(NxgCtx* ctx, const NxgColumns* in, const uint8_t* heap, uint8_t* out,
                       uint64_t cap, uint64_t* len_out, uint64_t* chunk_len_out,
                       uint64_t cap_chunks, uint64_t* n_chunks, NetidxError* err);

/* ---- multi-GPU: one frame decoded in byte ranges, one batch encoded in shards -------------
 * One process per GPU. A frame of W bytes is cut into contiguous byte ranges; each GPU decodes
 * the messages that START in its range, reading past the range end as needed (messages never
 * straddle frames, channel.rs:187-201, but they do straddle ranges). A range's summary says
 * where its chain enters (the first message start >= begin) and leaves (the first start >= end,
 * or the frame end); nxg_range_link checks that consecutive ranges meet and numbers their rows.
 * Any f64 frame (the length-run decoder, or the single-pass decoder when ids come in any order)
 * into f64 or mixed columns, and frames of short Updates / Heartbeats (the fast mixed decoder)
 * into mixed columns; a range those decoders decline (Maps, nested containers, rare control
 * messages, content errors) reports ok = 0 (err_kind NXG_CAPACITY when it was declined because
 * the columns are too small). nxg_decode_sharded then falls back to row shares
 * (nxg_decode_share). */
typedef struct NxgRange {
    uint64_t begin, end; /* the byte range [begin, end) of the frame */
    uint64_t entry;      /* first message start >= begin (absolute byte offset) */
    uint64_t exit;       /* first message start >= end, or the frame end */
    uint64_t n_rows;     /* rows decoded from the range (at dout rows 0 .. n_rows) */
    uint32_t ok;         /* 1: decoded by bytes; 2: decoded as a row share (nxg_decode_sharded's
                            fallback: entry = exit = UINT64_MAX); 0: declined */
    uint32_t err_kind;   /* NxgErrKind: the columns overflowed (ok = 1, or ok = 0 when that is why
                            the range was declined); the frame's error (ok = 2); else 0 */
    uint64_t err_offset; /* ok = 2: the frame's error offset */
} NxgRange;
/* Device frame and device columns; synchronous. */
bool nxg_decode_range(NxgCtx* ctx, const uint8_t* dframe, uint64_t frame_len, uint64_t begin,
                      uint64_t end, NxgColumns* dout, NxgRange* rng, NetidxError* err);
/* One share of a frame's rows: the frame (device) decoded whole, as nxg_decode_updates does
 * (every decoder, every error), then rows [N*share/shares, N*(share+1)/shares) of its N rows, the
 * children of their values and the control spans before them (the last share: also those after
 * the last row) into dout (device columns) from row 0, child indices and ctl_row re-based;
 * *row_off = the share's first row. The frame's error (status->err_kind / err_offset) leaves no
 * rows in any share; a share that does not fit dout reports NXG_CAPACITY (NXG_NOT_F64 for mixed
 * content in f64 columns). The ctx grows its own whole-frame columns on demand (first `shares`
 * times dout's capacities). Synchronous. */
bool nxg_decode_share(NxgCtx* ctx, const uint8_t* dframe, uint64_t frame_len, uint32_t share,
                      uint32_t shares, NxgColumns* dout, uint64_t* row_off, NxgStatus* status,
                      NetidxError* err);
/* Ranges in frame order, contiguous from 0 to frame_len: checks ranges[0].entry == 0,
 * ranges[i].exit == ranges[i+1].entry and the last exit == frame_len; row_off[i] = rows before
 * range i. Returns false (and *bad = the first range whose entry is off the chain) otherwise. */
bool nxg_range_link(const NxgRange* ranges, uint32_t n, uint64_t frame_len, uint64_t* row_off,
                    uint32_t* bad, NetidxError* err);

/* RCCL communicator (librccl, over xGMI) for the sharded calls. nxg_comm_unique_id on one rank,
 * its 128 bytes sent to every rank by the caller (as ncclGetUniqueId's id), nxg_comm_init on
 * every rank (collective). */
typedef struct NxgComm NxgComm;
bool nxg_comm_unique_id(uint8_t id[128], NetidxError* err);
NxgComm* nxg_comm_init(NxgCtx* ctx, int nranks, int rank, const uint8_t id[128],
                       NetidxError* err);
void nxg_comm_destroy(NxgComm* comm);
/* A caller-provided transport for the sharded calls instead of RCCL (the application's own MPI
 * or TCP collectives; the tests' gloo), and optionally a caller-provided local codec instead of
 * the ctx's kernels. Collective functions are called by every rank in the same order and return
 * true on success. The protocol (nxg_encode_allgather, nxg_decode_sharded) is the same code for
 * every transport: every rank's failure is exchanged in the next collective, so all ranks return
 * false together (none is left waiting in a collective). */
typedef struct NxgCommOps {
    void* user;
    /* collective: `bytes` bytes at `mine` (host memory) from every rank, in rank order, into
     * `all` (host memory, nranks * bytes) */
    bool (*allgather)(void* user, const void* mine, void* all, uint64_t bytes);
    /* collective: `buf` (device memory; host memory with the codec hooks below) holds this
     * rank's shard at [off[rank], off[rank + 1]); afterwards every rank's buf holds every shard
     * at its offset (off has nranks + 1 entries) */
    bool (*allgatherv)(void* user, uint8_t* buf, const uint64_t* off, uint32_t nranks,
                       uint32_t rank);
    /* local codec, all three or none (NULL: the ctx's kernels): the contracts of
     * nxg_encoded_len, nxg_encode_updates and nxg_decode_range */
    bool (*encoded_len)(void* user, const NxgColumns* in, const uint8_t* heap, uint64_t* len);
    bool (*encode)(void* user, const NxgColumns* in, const uint8_t* heap, uint8_t* out,
                   uint64_t cap, uint64_t* len);
    bool (*decode_range)(void* user, const uint8_t* frame, uint64_t frame_len, uint64_t begin,
                         uint64_t end, NxgColumns* out, NxgRange* rng);
    /* optional with the codec hooks (NULL: a declined range fails nxg_decode_sharded): the
     * contract of nxg_decode_share */
    bool (*decode_share)(void* user, const uint8_t* frame, uint64_t frame_len, uint32_t share,
                         uint32_t shares, NxgColumns* out, uint64_t* row_off, NxgStatus* status);
} NxgCommOps;
/* Not collective. ctx may be NULL when ops carries the local codec. The ops struct is copied. */
NxgComm* nxg_comm_init_ops(NxgCtx* ctx, int nranks, int rank, const NxgCommOps* ops,
                           NetidxError* err);
/* BASELINE configs[4]: every rank encodes its shard of the batch (rows in rank order) straight
 * into its place in the full frame (an 8-byte all-gather of the shard sizes first), then grouped
 * send/recv deliver every shard into the same offsets on every rank: no padding, no compaction.
 * *len_out = the full frame length; shard_off[0 .. nranks) = each shard's byte offset (may be
 * NULL). Device columns and buffers (host ones with an ops comm's local codec). A failure on any
 * rank (its encode, a capacity short of the frame) makes every rank return false. */
bool nxg_encode_allgather(NxgCtx* ctx, NxgComm* comm, const NxgColumns* din, const uint8_t* dheap,
                          uint8_t* dout, uint64_t cap, uint64_t* len_out, uint64_t* shard_off,
                          NetidxError* err);
/* One frame (on every rank's device) decoded in nranks byte ranges: rank r decodes range r,
 * the summaries are all-gathered and linked; a range whose guessed entry is off the chain is
 * decoded again from its predecessor's exit. *row_off = this rank's first global row. When a
 * range is declined (rng->ok 0 on some rank: content the byte-range decoders do not take), every
 * rank sees it in the same exchange and falls back to nxg_decode_share(rank, nranks): the frame
 * decoded whole on every rank (the frame is there already; no data moves), rows in nranks row
 * shares, rng->ok = 2, the frame's error in rng->err_kind / err_offset. Every rank returns the
 * same verdict: a local failure on any rank (a launch, a range declined for capacity), or a frame
 * that does not link makes all of them return false. */
bool nxg_decode_sharded(NxgCtx* ctx, NxgComm* comm, const uint8_t* dframe, uint64_t frame_len,
                        NxgColumns* dout, uint64_t* row_off, NxgRange* rng, NetidxError* err);

/* ---- dispatch: replaces ConnectionCtx::process_updates_batch (connection.rs:546-567) ------
 * The decoded Update rows fanned out to the subscriber's channels. For each row, in batch
 * order: the subscription of its Id, found by a dense table (publisher Ids come from a counter
 * starting at 0, netidx-core/src/utils.rs:130-134); an Id with no subscription, or >= n_ids, is
 * dropped, as `self.subscriptions.get(&i)` returning None. For each stream of the
 * subscription, in stream order, the entry (SubId, row) is appended to that stream's channel
 * batch (by_chan, connection.rs:551-557), so every channel sees its updates in batch order. A
 * subscription that keeps `last` records its last row in the batch (connection.rs:559-561).
 *
 * The table is a CSR built by the host from its subscriptions map; every array is device
 * memory: */
#define NXG_NO_SLOT 0xffffffffu
typedef struct NxgSubTable {
    uint64_t n_ids;                   /* slot_of_id covers Ids [0, n_ids) */
    const uint32_t* slot_of_id;       /* [n_ids]: subscription slot, or NXG_NO_SLOT */
    uint64_t n_slots;                 /* subscriptions */
    const uint64_t* slot_sub_id;      /* [n_slots]: SubId (subscriber/mod.rs:85) */
    const uint32_t* slot_stream_off;  /* [n_slots + 1]: the slot's streams, CSR */
    const uint32_t* stream_chan;      /* [n_streams]: channel of each stream, < n_chans */
    const uint8_t* slot_has_last;     /* [n_slots]: 1 if the subscription keeps `last` */
    uint32_t n_chans;                 /* channels (ChanId) */
} NxgSubTable;
/* Output (device memory, capacities from the caller):
 *   chan_off[n_chans + 1]  channel c's batch is entries [chan_off[c], chan_off[c+1])
 *   ent_sub[cap], ent_row[cap]  (SubId, index of the update's row in the decoded columns)
 *   last_row[n_slots]      1 + the last row of the slot's subscription in this batch, 0 if none
 *                          (or if the slot keeps no `last`) */
typedef struct NxgDispatch {
    uint64_t cap_entries;
    uint64_t* chan_off;
    uint64_t* ent_sub;
    uint64_t* ent_row;
    uint64_t* last_row;
    uint64_t n_entries;   /* written by the call */
    uint64_t n_unmatched; /* rows whose Id has no subscription */
} NxgDispatch;
/* `id` = the decoded id column (device), n_rows rows. Synchronous. Returns false on API misuse,
 * a HIP failure, or entries > cap_entries (n_entries then holds the required capacity). */
bool nxg_dispatch_updates(NxgCtx* ctx, const NxgSubTable* tab, const uint64_t* id,
                          uint64_t n_rows, NxgDispatch* out, NetidxError* err);

/* ---- type-partitioned view of decoded mixed columns (optional output) --------
 * Replaces the per-value 28-way `match` on the tag (Value::decode, netidx-value/src/lib.rs:470-506)
 * for a consumer that handles values by type: the rows of `cols` grouped by their tag column, on
 * the device, from a per-tile LDS tag histogram + scan (the mechanism BASELINE configs[2] names).
 * Device memory, capacities >= cols->n_rows (rows < 2^32):
 *   rank[i]      row i's index among the rows of its tag (record -> (tag[i], rank[i]))
 *   row_of[d]    the row at dense index d; tag t's rows are d in [off[t], off[t+1]), in record
 *                order
 *   fixed[d], aux[d]   the rows' fixed / aux columns at their dense index
 * off[] and count[] are filled on the host (off[NXG_TAG_BINS] = n_rows). Children (array
 * elements) and text stay where the decode put them (fixed / aux of a row still point at them).
 * Synchronous. Returns false on API misuse (F64-only columns have no tag column) or a HIP
 * failure. */
#define NXG_TAG_BINS 256
typedef struct NxgTagView {
    uint64_t cap_rows;
    uint32_t* rank;
    uint32_t* row_of;
    uint64_t* fixed;
    uint32_t* aux;
    uint64_t n_rows;                    /* written by the call */
    uint64_t count[NXG_TAG_BINS];       /* rows per tag value */
    uint64_t off[NXG_TAG_BINS + 1];     /* exclusive prefix of count */
} NxgTagView;
bool nxg_partition_by_tag(NxgCtx* ctx, const NxgColumns* cols, NxgTagView* out, NetidxError* err);

/* ---- publisher commit: replaces UpdateBatch::commit (publisher/mod.rs:776-845) ----------
 * A queued batch (its rows in NxgColumns form: id, tag, fixed, aux, text in `heap`; kind[i] per
 * row; to_client[i] for NXG_PUB_UPDATE_CLIENT rows) becomes per-client batches of
 * From::Update(id, v), in batch order:
 *   NXG_PUB_UPDATE          Update(None, id, v)  (Val::update, mod.rs:517-519): to every client
 *                           subscribed to id (pb.by_id[id].subscribed), then current = v;
 *   NXG_PUB_UPDATE_CHANGED  UpdateChanged(id, v) (update_changed): the same, only if
 *                           current != v (Value::eq, netidx-value/src/op.rs:133-172);
 *   NXG_PUB_UPDATE_CLIENT   Update(Some(cl), id, v) (update_subscriber): to client cl only.
 * Ids that are not published are dropped (counted in n_unmatched). The table (device memory):
 * by_id as a dense slot table, each slot's subscribed clients as a CSR, and each slot's current
 * value (cur_tag NULL: all F64; text, Decimal and Abstract bytes at cur_heap + cur_fixed; the
 * elements of Array/Map/Error(Value) current values at cur_ctag/cur_cfixed/cur_caux slots
 * cur_fixed .., as NxgColumns children; the batch's children are the batch's NxgColumns
 * children). Equality is Value::eq on every variant: floats NaN == NaN, Decimal numerically
 * (rust_decimal's PartialEq: scale-independent, every zero equal), containers element by element
 * (Map entries in column order -- the reference's encoder writes them sorted and unique),
 * Abstract by its bytes. Output in NxgDispatch: per client c, entries [chan_off[c], chan_off[c+1])
 * of (ent_sub = Id, ent_row = row); last_row[slot] = 1 + the row that became current (0:
 * unchanged). Synchronous; false on misuse, HIP failure, capacity, or NXG_UNSUPPORTED (a value
 * nested deeper than 32 levels; err->msg says which). */
enum NxgPubKind { NXG_PUB_UPDATE = 0, NXG_PUB_UPDATE_CHANGED = 1, NXG_PUB_UPDATE_CLIENT = 2 };
typedef struct NxgPubTable {
    uint64_t n_ids;                   /* slot_of_id covers Ids [0, n_ids) */
    const uint32_t* slot_of_id;       /* [n_ids]: published-value slot, or NXG_NO_SLOT */
    uint64_t n_slots;
    const uint32_t* slot_client_off;  /* [n_slots + 1]: subscribed clients, CSR */
    const uint32_t* client;           /* [n_subscriptions]: client index, < n_clients */
    uint32_t n_clients;
    const uint8_t* cur_tag;           /* [n_slots] current values, columns as NxgColumns */
    const uint64_t* cur_fixed;
    const uint32_t* cur_aux;          /* NULL: 0 */
    const uint8_t* cur_heap;
    const uint8_t* cur_ctag;          /* children of the current values (NULL: none) */
    const uint64_t* cur_cfixed;
    const uint32_t* cur_caux;
} NxgPubTable;
bool nxg_publish_commit(NxgCtx* ctx, const NxgPubTable* tab, const NxgColumns* batch,
                        const uint8_t* heap, const uint8_t* kind, const uint32_t* to_client,
                        NxgDispatch* out, NetidxError* err);
/* The commit's unsubscribes (publisher/mod.rs:820-832): the queued (client, Id) pairs, in queue
 * order, onto each client's From::Unsubscribed list; clients >= n_clients are dropped
 * (pb.clients.get(&cl) is None). Output: chan_off[n_clients + 1] and ent_sub (the Ids) in `out`;
 * ent_row = the pair's index in the queue; last_row unused (may be NULL). Synchronous. */
bool nxg_publish_unsubscribes(NxgCtx* ctx, const uint64_t* id, const uint32_t* client,
                              uint64_t n, uint32_t n_clients, NxgDispatch* out, NetidxError* err);

/* ---- archive batches: replaces <GPooled<Vec<BatchItem>> as Pack>::decode ------------------
 * (netidx-archive/src/logfile/reader.rs:449/475 over logfile/mod.rs:150-205 BatchItem and
 * netidx/src/subscriber/mod.rs:154-177 Event). `buf` (device memory, `len` bytes) starts with the
 * batch: varint count, then count items of varint Id (as u32) and an Event that is not
 * length-wrapped (0x40 = Unsubscribed, else a bare Value). `len` is what remains of the buffer
 * (the uncompressed reader decodes from the record to the end of the mmap, reader.rs:449): it
 * bounds the size guard, while the fast path reads only a window of it that grows geometrically
 * until the batch fits, so the cost follows the batch. A batch the fast path declines (an error,
 * Maps, nesting, ...) is decoded by the exact decoder, which walks the whole buffer.
 * Output: MIXED-layout columns (nxg_columns_alloc), one row per item: id = the u32 Id, the
 * Event's Value in tag/fixed/aux (+ children; text offsets index `buf`), Unsubscribed as tag
 * NXG_TAG_UNSUBSCRIBED with fixed 0, aux 0. status: n_rows (= count), n_children, err_kind /
 * err_offset (the failing item's start, 0 for the count and the size guard) with the reference's
 * PackError kinds; path = NXG_PATH_ARCHIVE_FAST (the fast path) or NXG_PATH_ARCHIVE (the exact
 * decoder). *consumed = the batch's length in bytes.
 * Deviation: Event::decode on an empty buffer panics in the reference; here it is
 * NXG_BUFFER_SHORT. Synchronous; false on misuse or a HIP failure. A decode error is reported in
 * `status` (as nxg_decode_updates does), with n_rows = n_children = 0. */
#define NXG_TAG_UNSUBSCRIBED 0x40
#define NXG_PATH_ARCHIVE 3
#define NXG_PATH_ARCHIVE_FAST 5
bool nxg_decode_archive_batch(NxgCtx* ctx, const uint8_t* buf, uint64_t len, NxgColumns* out,
                              NxgStatus* status, uint64_t* consumed, NetidxError* err);
/* Replaces <GPooled<Vec<BatchItem>> as Pack>::encode (writer.rs:423-428, pack.rs:941-952):
 * device MIXED-layout columns in the same form (id = the u32 Id, tag NXG_TAG_UNSUBSCRIBED for
 * Event::Unsubscribed; text at heap + fixed, device memory; no control messages) to `out`
 * (device memory, `cap` bytes; NULL: *len_out = the length only). Synchronous. TooBig when
 * count * size_of::<BatchItem>() exceeds MAX_VEC or a value violates a size guard. */
bool nxg_encode_archive_batch(NxgCtx* ctx, const NxgColumns* in, const uint8_t* heap,
                              uint8_t* out, uint64_t cap, uint64_t* len_out, NetidxError* err);

/* ---- compressed archive batches: replaces the compressed branch of ArchiveReader::get_batch_at
 * (netidx-archive/src/logfile/reader.rs:453-477): a record after its RecordHeader is
 * u32 BE uncompressed record length | the RecordIndex (indexed files: a varint that is its own
 * length, then the ids) | one zstd frame of the batch, compressed with the archive's dictionary
 * (reader.rs:243-244, 737-801; zstd 0.13 = libzstd 1.5, RFC 8878). The frames are decompressed on
 * the device, many records per call; nxg_decode_archive_batch then decodes each batch.
 * A dictionary (the archive's, from its header): zstd format (magic EC30A437: entropy tables,
 * repeat offsets, content) or raw content. */
typedef struct NxgZstdDict NxgZstdDict;
NxgZstdDict* nxg_zstd_dict_new(NxgCtx* ctx, const uint8_t* dict, uint64_t len, NetidxError* err);
void nxg_zstd_dict_free(NxgZstdDict* d);
/* one record: in, its bytes [off, off + len) of `src` (after the RecordHeader); out, its batch at
 * [out_off, out_off + out_len) of `dout` (each record has room for its uncompressed length), and
 * err: 0, or 1 not a zstd frame / trailing bytes, 2 corrupt, 3 the batch is longer than the
 * record's uncompressed length, 4 dictionary missing or of another id, 5 checksum mismatch, 6
 * frame content size mismatch, 7 record too short. A record's failure is its own (the
 * reference fails that get_batch); the others are decompressed. */
typedef struct NxgArchiveRecord {
    uint64_t off, len;
    uint64_t out_off, out_len;
    uint32_t err, pad;
} NxgArchiveRecord;
/* src: host memory (the archive's mmap), src_len bytes; dout: device memory of `cap` bytes (NULL:
 * *need = the bytes the records need). dict may be NULL (frames without a dictionary). The host
 * reads the records' lengths and index prefixes; the frames go to the device in one copy.
 * Synchronous. Returns false on misuse, a HIP failure or cap < *need. */
bool nxg_archive_decompress(NxgCtx* ctx, const NxgZstdDict* dict, const uint8_t* src,
                            uint64_t src_len, NxgArchiveRecord* recs, uint32_t n, bool indexed,
                            uint8_t* dout, uint64_t cap, uint64_t* need, NetidxError* err);

/* ---- the publisher <-> subscriber connection (BASELINE configs[0]) ------------------------
 * Replaces hello_publisher (netidx/src/subscriber/connection.rs:120-140), ClientCtx::hello
 * (publisher/server.rs:367-381), read_task / flush_buf (channel.rs:107-126, 379-443) and the
 * To::Subscribe -> From::Subscribed exchange (publisher/server.rs:60-137, 506-516), anonymous
 * authentication only. Raw handshake messages are a u32 big-endian length + the packed value
 * (channel.rs:63-105): u64 3 both ways, then Hello::Anonymous both ways. After the handshake
 * the connection is a Channel of frames (nxg_frame_header) holding len-wrapped messages.
 * Sessions are blocking sockets; one thread per session. */
typedef struct NxgSession NxgSession;
/* subscriber side: connect and run the handshake */
NxgSession* nxg_session_connect(const char* ipv4, uint16_t port, NetidxError* err);
/* publisher side: a listening socket (port 0: any; *bound_port receives it), then one accepted,
 * handshaken connection per nxg_session_accept */
NxgSession* nxg_session_listen(const char* ipv4, uint16_t port, uint16_t* bound_port,
                               NetidxError* err);
NxgSession* nxg_session_accept(NxgSession* listener, NetidxError* err);
void nxg_session_close(NxgSession* s);
/* frames_in, bytes_in, frames_out, bytes_out */
void nxg_session_stats(const NxgSession* s, uint64_t out[4]);
/* one frame out: u32 header (channel.rs:107-126) + payload (<= MAX_BATCH) */
bool nxg_session_send(NxgSession* s, const uint8_t* payload, uint64_t len, NetidxError* err);
/* the next complete frame in (read_task, channel.rs:379-443): *payload stays valid until the
 * next receive on this session; encrypted frames are refused */
bool nxg_session_recv_frame(NxgSession* s, const uint8_t** payload, uint64_t* len,
                            NetidxError* err);
/* the data path, subscriber side: the next frame, read into page-locked memory, decoded on the
 * device into `out` as nxg_decode_updates does (status, flags likewise) */
bool nxg_session_recv_decode(NxgSession* s, NxgCtx* ctx, NxgColumns* out, uint32_t flags,
                             NxgStatus* status, uint64_t* frame_len, NetidxError* err);
/* the data path, publisher side: device columns encoded on the GPU (nxg_encode_frames: the
 * MAX_BATCH cuts), copied to page-locked memory and written as frames */
bool nxg_session_publish(NxgSession* s, NxgCtx* ctx, const NxgColumns* cols, const uint8_t* heap,
                         uint64_t* bytes_sent, NetidxError* err);
/* Control messages (len-wrapped derived enums, netidx-derive lib.rs:289-381). Builders return
 * the message length (out NULL: the length only) or -NXG_CAPACITY / -NXG_UNKNOWN_TAG. */
/* To::Subscribe { path, resolver: SocketAddr::V4, timestamp, permissions, token }
 * (netproto publisher.rs:57-63) */
int64_t nxg_msg_subscribe(const char* path, uint64_t path_len, uint32_t resolver_ipv4,
                          uint16_t resolver_port, uint64_t timestamp, uint32_t permissions,
                          const uint8_t* token, uint64_t token_len, uint8_t* out, uint64_t cap);
/* From::Subscribed(path, id, value) with a scalar value (tag/fixed/aux as NxgColumns; String and
 * Bytes bytes at `text`) */
int64_t nxg_msg_subscribed(const char* path, uint64_t path_len, uint64_t id, uint8_t tag,
                           uint64_t fixed, uint32_t aux, const uint8_t* text, uint8_t* out,
                           uint64_t cap);
/* From::Heartbeat (2 bytes) */
int64_t nxg_msg_heartbeat(uint8_t* out, uint64_t cap);
/* From::Update(id, value) with a scalar value (tag/fixed/aux as NxgColumns; String and Bytes
 * bytes at `text`): one message as Val::update + commit queue it (publisher/mod.rs:517-519,
 * 776-845) and handle_updates encodes it (server.rs:604-629) -- the host path of a publisher
 * that updates one value at a time (BASELINE configs[0]). */
int64_t nxg_msg_update(uint64_t id, uint8_t tag, uint64_t fixed, uint32_t aux,
                       const uint8_t* text, uint8_t* out, uint64_t cap);
/* One control message parsed: to = 0 a publisher::From, 1 a publisher::To. Offsets index `buf`.
 * value_fixed holds scalar payloads as read (big-endian integers, varints as decoded, zigzag
 * not undone); other values are reported by tag and span. */
typedef struct NxgCtlMsg {
    uint64_t msg_len; /* the message's bytes (len-wrapped region) */
    uint32_t variant;
    uint32_t permissions;
    uint64_t id;
    uint64_t path_off, path_len;
    uint64_t timestamp;
    uint64_t token_off, token_len;
    uint64_t value_off, value_len; /* the value's bytes, tag included */
    uint64_t value_fixed;
    uint32_t value_tag, value_aux;
} NxgCtlMsg;
bool nxg_msg_parse(const uint8_t* buf, uint64_t len, int to, NxgCtlMsg* m, NetidxError* err);

/* ---- a machine-local anonymous resolver (BASELINE configs[0]) ------------------------------
 * The control plane the examples need to find each other, host only: the resolver server's
 * anonymous read and write paths (netidx/src/resolver_server/mod.rs:458-480, 771-860), the write
 * client's hello and ToWrite::Publish (resolver_client/write_client.rs:194-221), the read client's
 * hello and ToRead::Resolve -> FromRead::Publisher + FromRead::Resolved (read_client.rs:84-99,
 * resolver_server/shard_store.rs:160-193, 600-640). Blocking sockets; the server runs a thread per
 * client. Authentication other than anonymous, referrals and clustering are out of scope. */
typedef struct NxgResolver NxgResolver;
typedef struct NxgResolverClient NxgResolverClient;
NxgResolver* nxg_resolver_start(const char* ipv4, uint16_t port, uint16_t* bound_port,
                                uint64_t writer_ttl_secs, NetidxError* err);
void nxg_resolver_stop(NxgResolver* r);
uint64_t nxg_resolver_n_published(NxgResolver* r);
/* a publisher's resolver connection: ClientHello::WriteOnly { write_addr, Anonymous, Normal } */
NxgResolverClient* nxg_resolver_connect_write(const char* ipv4, uint16_t port,
                                              uint32_t write_ipv4, uint16_t write_port,
                                              uint64_t* ttl_out, NetidxError* err);
/* a subscriber's: ClientHello::ReadOnly(Anonymous) */
NxgResolverClient* nxg_resolver_connect_read(const char* ipv4, uint16_t port, NetidxError* err);
void nxg_resolver_client_close(NxgResolverClient* c);
/* ToWrite::Publish(path), true once FromWrite::Published is back */
bool nxg_resolver_publish(NxgResolverClient* c, const char* path, uint64_t path_len,
                          NetidxError* err);
/* ToRead::Resolve(path): the Resolved reply; its first publisher's address from the
 * FromRead::Publisher that precedes it (n_publishers = 0: nobody publishes the path) */
typedef struct NxgResolved {
    uint32_t n_publishers;
    uint32_t publisher_ipv4; /* host byte order */
    uint64_t publisher_id;
    uint16_t publisher_port, resolver_port;
    uint32_t resolver_ipv4;
    uint64_t timestamp;
    uint32_t flags, permissions;
} NxgResolved;
bool nxg_resolver_resolve(NxgResolverClient* c, const char* path, uint64_t path_len,
                          NxgResolved* out, NetidxError* err);

/* ---- host framing (netidx/src/channel.rs) ------------------------------------------------
 * Frame boundaries exactly as WriteChannel::queue_send/try_flush split the buffer. The split
 * happens at MAX_BATCH = 0x3FFFFFFF (channel.rs:34, 187-191) and is recorded between messages.
 * `msg_len` holds the encoded length of each message, in order. `chunk_len_out` receives the
 * length of each frame payload. Returns the number of frames, or -1 if cap_chunks is too small
 * or a message exceeds MAX_BATCH. */
int64_t nxg_frame_split(const uint64_t* msg_len, uint64_t n_msgs, uint64_t* chunk_len_out,
                        uint64_t cap_chunks);
/* flush_buf (channel.rs:107-126): the u32 big-endian header, with bit 31 set when the frame is
 * encrypted. */
void nxg_frame_header(uint32_t payload_len, bool encrypted, uint8_t out[4]);
/* read_task (channel.rs:379-443): parse one header from `buf`. Returns the header size (4), or
 * 0 if fewer than 4 bytes are present. */
uint32_t nxg_frame_parse_header(const uint8_t* buf, uint64_t avail, uint32_t* payload_len,
                                bool* encrypted);
/* read_task's frame assembly (channel.rs:379-443), incremental: push the bytes read from the
 * socket in any pieces; _next hands out each complete frame payload, in order (the pointer stays
 * valid until the next _push or _free). _next returns 1 with a frame, 0 when the next frame is not
 * complete yet ("reading more"), -1 on an encrypted frame: this layer has no security context
 * ("encryption is not supported", channel.rs:420-422; krb5 is out of scope). */
typedef struct NxgFrameReader NxgFrameReader;
NxgFrameReader* nxg_frame_reader_new(NetidxError* err);
void nxg_frame_reader_free(NxgFrameReader* r);
bool nxg_frame_reader_push(NxgFrameReader* r, const uint8_t* data, uint64_t len, NetidxError* err);
int nxg_frame_reader_next(NxgFrameReader* r, const uint8_t** payload, uint64_t* len,
                          NetidxError* err);
uint64_t nxg_frame_reader_buffered(const NxgFrameReader* r);

#ifdef __cplusplus
}
#endif
#endif
