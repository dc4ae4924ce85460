/*
 * nx_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A scalar CPU restatement of netidx's Pack codec for the publisher->subscriber update stream
 * (reference: netidx-core/src/pack.rs, netidx-value/src/{lib,array,pbuf,abstract_type}.rs,
 * netidx-netproto/src/publisher.rs + netidx-derive/src/lib.rs, netidx/src/channel.rs).
 *
 * It is the CHECKER for the HIP codec in netidx_amd/: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product never links or calls it.
 *
 * Parity pinning: the reference is Rust-only and cannot be built or run in this image (no
 * cargo/rustc, no network). This oracle is pinned by (1) the reference's
 * own tests restated (varint sweep netidx-core/src/test.rs:16-63, encoded_len/round-trip
 * properties netidx-netproto/src/test.rs:15-21, decode-never-crashes fuzz test.rs:449-456) and
 * (2) hand-derived known-answer vectors (tests/golden/). Byte-level parity
 * against the executing reference is therefore "parity partially pinned"; see DESIGN.md.
 *
 * Columnar contract (identical to include/nxg_codec.h, restated here independently):
 *   rows     : one per From::Update            id u64, tag u8, fixed u64, aux u32
 *   children : elements of Array/Map/Error     tag u8, fixed u64, aux u32
 *   ctl      : every other From message        row u64, off u64, len u32, variant u8
 */
#ifndef NX_ORACLE_H
#define NX_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* PackError, netidx-core/src/pack.rs:89-95 (+ codec-level kinds) */
enum {
    NXO_OK = 0,
    NXO_UNKNOWN_TAG = 1,
    NXO_TOO_BIG = 2,
    NXO_INVALID_FORMAT = 3,
    NXO_BUFFER_SHORT = 4,
    NXO_DEPTH = 6,     /* nesting deeper than NXO_MAX_DEPTH (documented deviation) */
    NXO_CAPACITY = 7,  /* output columns too small */
};

#define NXO_MAX_DEPTH 32

typedef struct NxoCols {
    /* capacities (in) */
    uint64_t cap_rows, cap_children, cap_ctl;
    /* counts (out) */
    uint64_t n_rows, n_children, n_ctl, n_heartbeat;
    /* rows */
    uint64_t* id;
    uint8_t* tag;
    uint64_t* fixed;
    uint32_t* aux;
    /* children */
    uint8_t* ctag;
    uint64_t* cfixed;
    uint32_t* caux;
    /* control messages */
    uint64_t* ctl_row;
    uint64_t* ctl_off;
    uint32_t* ctl_len;
    uint8_t* ctl_variant;
    /* status (out) */
    int32_t err_kind;
    uint64_t err_offset;
} NxoCols;

/* primitives: pack.rs:472-520 */
uint32_t nxo_varint_len(uint64_t v);
uint32_t nxo_encode_varint(uint64_t v, uint8_t* out);
int nxo_decode_varint(const uint8_t* p, uint64_t avail, uint64_t* v, uint32_t* nread);
uint32_t nxo_len_wrapped_len(uint64_t inner);
/* restatement of netidx-core/src/test.rs:16-63 over d in [lo, hi); returns failures */
uint64_t nxo_varint_sweep(uint64_t lo, uint64_t hi, int short_buf);

/* frame decode: the receive_batch_fn loop (channel.rs:504-521) over From::decode. This is
 * also the timed cpu_baseline of bench.py (1 core, as one tokio decode task per connection). */
int nxo_decode_frame(const uint8_t* w, uint64_t len, NxoCols* c);

/* encode: queue_send loop (channel.rs:177-202) over From::encode; heap = bytes referenced by
 * string/bytes/decimal/abstract offsets and ctl spans. Returns bytes written or -errkind. */
int64_t nxo_encoded_len(const NxoCols* c, const uint8_t* heap);
int64_t nxo_encode(const NxoCols* c, const uint8_t* heap, uint8_t* out, uint64_t cap);

/* f64 batch encode from id/val columns (config 4) */
int64_t nxo_encode_f64(const uint64_t* id, const uint64_t* val, uint64_t n, uint8_t* out,
                       uint64_t cap);

/* chrono DateTime::from_timestamp validity (pack.rs:1567-1575; chrono 0.4.35+ rules) */
int nxo_datetime_valid(int64_t secs, uint32_t nsecs);
/* std str::from_utf8 validity (pack.rs:462) */
int nxo_utf8_valid(const uint8_t* p, uint64_t n);

/*
 * Subscriber update dispatch: ConnectionCtx::process_updates_batch
 * (netidx/src/subscriber/connection.rs:546-567). For each Update row i, in batch order: the
 * subscription of id[i] (the Id -> Sub map, here a dense table: slot_of_id[id], NXO_NO_SLOT or
 * an id >= n_ids = not subscribed, the update is dropped); for each of the subscription's
 * streams (chan_id, channel), in stream order, (sub_id, Event::Update) is pushed onto that
 * channel's batch; and the subscription's `last` (if kept) becomes this update.
 *
 * Output, grouped by channel: chan_off[n_chans + 1] (CSR), ent_sub / ent_row (SubId and the
 * row of the update) in push order; last_row[slot] = 1 + the last row of the slot's
 * subscription in the batch, 0 if none (or if the slot keeps no `last`). Returns the number of
 * entries, or -NXO_CAPACITY if they exceed cap. *n_unmatched: rows without a subscription.
 */
#define NXO_NO_SLOT 0xffffffffu
int64_t nxo_dispatch(const uint64_t* id, uint64_t n_rows, uint64_t n_ids,
                     const uint32_t* slot_of_id, uint64_t n_slots, const uint64_t* slot_sub_id,
                     const uint32_t* slot_stream_off, const uint32_t* stream_chan,
                     const uint8_t* slot_has_last, uint32_t n_chans, uint64_t* chan_off,
                     uint64_t* ent_sub, uint64_t* ent_row, uint64_t cap, uint64_t* last_row,
                     uint64_t* n_unmatched);

/*
 * Publisher commit: UpdateBatch::commit (netidx/src/publisher/mod.rs:776-845). For each queued
 * message, in batch order (kind[i]):
 *   NXO_PUB_UPDATE          Update(None, id, v): if id is published (by_id), push Update(id, v)
 *                           onto every subscribed client's batch, then current = v;
 *   NXO_PUB_UPDATE_CHANGED  UpdateChanged(id, v): the same, only if current != v (Value::eq,
 *                           netidx-value/src/op.rs:133-172);
 *   NXO_PUB_UPDATE_CLIENT   Update(Some(cl), id, v): push Update(id, v) onto client cl's batch.
 * Values are rows of (tag, fixed, aux) columns with text bytes at heap + fixed (cur_heap for the
 * current values). Output as nxo_dispatch: per-client CSR (client_off, ent_id, ent_row) in push
 * order, cur_row[slot] = 1 + the row that became current (0: unchanged). Returns the number of
 * entries, -NXO_CAPACITY, or -NXO_UNSUPPORTED when an UpdateChanged compares a value whose
 * equality the columns do not carry (Decimal, Array, Map, Error(Value), Abstract).
 */
enum { NXO_PUB_UPDATE = 0, NXO_PUB_UPDATE_CHANGED = 1, NXO_PUB_UPDATE_CLIENT = 2 };
#define NXO_UNSUPPORTED 10
int64_t nxo_publish_commit(const uint64_t* id, const uint8_t* tag, const uint64_t* fixed,
                           const uint32_t* aux, const uint8_t* heap, const uint8_t* kind,
                           const uint32_t* to_client, uint64_t n_rows, uint64_t n_ids,
                           const uint32_t* slot_of_id, uint64_t n_slots,
                           const uint32_t* slot_client_off, const uint32_t* client,
                           uint32_t n_clients, const uint8_t* cur_tag, const uint64_t* cur_fixed,
                           const uint32_t* cur_aux, const uint8_t* cur_heap, uint64_t* client_off,
                           uint64_t* ent_id, uint64_t* ent_row, uint64_t cap, uint64_t* cur_row,
                           uint64_t* n_unmatched);

/* commit with child columns (Array/Map/Error(Value) equality) for the batch and the current
 * values; children may be NULL when no value has any */
int64_t nxo_publish_commit2(const uint64_t* id, const uint8_t* tag, const uint64_t* fixed,
                            const uint32_t* aux, const uint8_t* ctag, const uint64_t* cfixed,
                            const uint32_t* caux, const uint8_t* heap, const uint8_t* kind,
                            const uint32_t* to_client, uint64_t n_rows, uint64_t n_ids,
                            const uint32_t* slot_of_id, uint64_t n_slots,
                            const uint32_t* slot_client_off, const uint32_t* client,
                            uint32_t n_clients, const uint8_t* cur_tag, const uint64_t* cur_fixed,
                            const uint32_t* cur_aux, const uint8_t* cur_ctag,
                            const uint64_t* cur_cfixed, const uint32_t* cur_caux,
                            const uint8_t* cur_heap, uint64_t* client_off, uint64_t* ent_id,
                            uint64_t* ent_row, uint64_t cap, uint64_t* cur_row,
                            uint64_t* n_unmatched);
int nxo_decimal_eq(const uint8_t* a, const uint8_t* b);

/* archive batches (netidx-archive logfile/mod.rs:188-205): see nx_oracle.c */
#define NXO_TAG_UNSUBSCRIBED 0x40
int64_t nxo_decode_archive(const uint8_t* w, uint64_t len, NxoCols* c);
int64_t nxo_encode_archive(const NxoCols* c, const uint8_t* heap, uint8_t* out, uint64_t cap);
int64_t nxo_publish_unsubscribes(const uint64_t* id, const uint32_t* cl, uint64_t n,
                                 uint32_t n_clients, uint64_t* client_off, uint64_t* ent_id);

#ifdef __cplusplus
}
#endif
#endif
