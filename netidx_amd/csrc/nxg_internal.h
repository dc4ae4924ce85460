// nxg_internal.h -- structures shared by the kernels and the host dispatch layer (not ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nxg_codec.h"

// Per-call device status block (a ring slot, zeroed kStatusRing/2 = 512 calls ahead: zero_status).
struct DevStatus {
    uint64_t n_rows, n_children, n_ctl, n_heartbeat;  // totals written by the last tile
    uint32_t err_kind;                                 // first error in wire order
    uint32_t path;
    uint64_t err_offset;
    uint32_t fast_fail;  // homogeneous-f64 kernel rejected the frame (=> general path)
    uint32_t timeout;    // a bounded spin expired (protocol bug); reported as NXG_TIMEOUT
    uint32_t capacity;   // a column overflowed its capacity
    uint32_t runs_valid;   // general decode: runs on the true chain, 0 = all (resolve -> emit)
    uint64_t total_bytes;  // encode: bytes written
    uint32_t nonf64;       // general path ran into content that F64-only columns cannot hold
    // f64 run decode: bit 0 record lengths vary too often (=> the single-pass decoder), bit 1
    // not an f64 frame (=> the mixed decoders); sequential-id decode: bit 2 the ids do not count
    // up by one (=> the length-run decoder)
    uint32_t irregular;
    // general decode: first error as ~(offset << 8 | kind), combined with atomicMax (0 = none)
    uint64_t err_key;
    // encode: 1 + the start offset of the message that holds byte MAX_BATCH, i.e. where
    // WriteChannel::queue_send records its first frame boundary (channel.rs:187-191); 0 = none
    uint64_t split_start;
    // diagnostics (general decode): 0 redo tiles, 1 look-back fallbacks, 2 repair rounds,
    // 3 lane walks, 4 speculation attempts, 5 tiles without a speculated entry,
    // 6 exhausted (budgeted) walks, 7 work-list entries of the emit pass. The fast mixed decode
    // (path 4) uses diag[7] as its resolve pass's arrival counter (zeroed with the slot).
    unsigned long long diag[8];
};
static_assert(sizeof(DevStatus) == 160, "DevStatus layout");

// Look-back status granule (one 8-byte word, written with one sc1 store):
//   bits 63:62 flag (1 aggregate, 2 inclusive), 61:44 call epoch, 43:0 value.
// A word whose epoch differs from the current call's reads as "not ready", so the status
// arrays need no per-call memset (they are zeroed only when the 18-bit epoch wraps).
constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagInc = 2ull << 62;
constexpr uint64_t kFlagMask = 3ull << 62;
constexpr int kEpochShift = 44;
constexpr uint64_t kEpochMax = (1ull << 18) - 1;
constexpr uint64_t kValMask = (1ull << kEpochShift) - 1;
constexpr uint64_t kMaxBatch = 0x3FFFFFFF;  // MAX_BATCH, netidx/src/channel.rs:34
constexpr uint64_t kMaxVecBytes = 2ull * 1024 * 1024 * 1024;  // MAX_VEC, pack.rs:917
constexpr uint64_t kBatchItemSize = 24;  // size_of::<BatchItem>() (logfile/mod.rs:188; unpinned)
// encode: note the message [pos, pos + len) if it holds byte MAX_BATCH (exactly one does, in a
// frame longer than MAX_BATCH)
__device__ inline void note_split(DevStatus* st, uint64_t pos, uint64_t len) {
    if (pos <= kMaxBatch && kMaxBatch < pos + len) st->split_start = pos + 1;
}
__host__ __device__ inline uint64_t lb_word(uint64_t flag, uint32_t epoch, uint64_t v) {
    return flag | ((uint64_t)epoch << kEpochShift) | (v & kValMask);
}
__host__ __device__ inline uint64_t lb_flag(uint64_t w, uint32_t epoch) {
    return ((w >> kEpochShift) & kEpochMax) == epoch ? (w & kFlagMask) : 0ull;
}

// ---- general decode geometry (nxg_decode_gen.hip) ----
namespace gdec2 {
constexpr int TPB = 256;            // 4 independent waves per workgroup, one run each
constexpr int CH = 64;              // bytes per lane
constexpr uint32_t TILE = 64 * CH;  // 4 KiB per tile
constexpr uint32_t IMG = TILE + 1024;  // LDS image: tile + 1 KiB look-ahead
constexpr int MAX_RUNS = 8192;      // runs (waves) per pass
constexpr int RUN_WORDS = 8;        // per-run summary words
}  // namespace gdec2

// ---- f64 encode geometry ----
namespace f64enc {
constexpr int LB_U = 1;                 // look-back window rows (64 tiles each); wider measured slower
constexpr int TPB = 256;
constexpr int RPT = 4;                 // records per thread
constexpr int TILE = TPB * RPT;        // records per tile
constexpr int MAXB = TILE * 15 + 32;   // staging bytes (f64 records <= 15 B for ids < 2^28)
}  // namespace f64enc

// Polls of an unpublished look-back predecessor before its aggregate is computed by the waiting
// workgroup itself (self-help look-backs); NXG_LOOKBACK_PATIENCE at context creation (tests: 0,
// every unpublished predecessor computed).
extern thread_local uint32_t nxg_patience;

// launchers (each defined next to its kernel)
struct ColsDesc;
// Every launcher takes the call's status slot `st` and `zst`, the slot that the call 512 calls
// later will use (nxg_take_zero_slot()). Block 0 of the kernel that receives it zeroes `zst` on
// entry, so the ring needs no per-call memset; a call that launches no such kernel (an empty
// frame or batch) has the host zero it instead (nxg_zero_used, nxg_api.cpp).
__device__ inline void zero_status(DevStatus* zst) {
    if (zst && blockIdx.x == 0 && threadIdx.x == 0) *zst = DevStatus{};
}
extern thread_local DevStatus* nxg_zero_slot;  // host side: passed through to the kernels
extern thread_local bool nxg_zero_used;         // a kernel of this call zeroes nxg_zero_slot
inline DevStatus* nxg_take_zero_slot() {
    nxg_zero_used = true;
    return nxg_zero_slot;
}
// f64 decode of any f64 frame in one pass (nxg_decode_f64_x.hip): `tstat` holds
// nxg_dec_f64x_groups(W) epoch-tagged words (no initialisation needed).
uint64_t nxg_dec_f64x_groups(uint64_t W);
// the records that start in [begin, end) of a W-byte frame; entry / exit (+1, relative to begin)
// in DevStatus.diag[2] / diag[3]
hipError_t nxg_launch_dec_f64x_range(const uint8_t* wire, uint64_t W, uint64_t begin,
                                     uint64_t end, uint64_t* oid, uint64_t* oval, uint64_t cap,
                                     uint64_t* tstat, uint32_t epoch, DevStatus* st,
                                     hipStream_t s);
hipError_t nxg_launch_dec_f64x(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                               uint64_t cap, uint64_t* tstat, uint32_t epoch, DevStatus* st,
                               hipStream_t s);
// f64 decode of a frame whose ids count up by one (nxg_decode_f64_seq.hip): one launch, no scratch.
// Declines with fast_fail + DevStatus.irregular bit 1 (not f64) or bit 2 (another f64 frame).
uint64_t nxg_dec_f64s_groups(uint64_t W);
hipError_t nxg_launch_dec_f64s(const uint8_t* wire, uint64_t W, uint64_t* oid, uint64_t* oval,
                               uint64_t cap, DevStatus* st, DevStatus* zst, hipStream_t s);
// f64 decode by length runs (nxg_decode_f64_run.hip): probe + emit launches. `desc` holds 16 bytes
// per tile (nxg_dec_f64r_tiles(W)), `tstat` nxg_dec_f64r_groups(W) epoch-tagged words. Sets
// DevStatus.irregular (and fast_fail) for frames whose record lengths vary record to record.
uint64_t nxg_dec_f64r_tiles(uint64_t W);
uint64_t nxg_dec_f64r_tile_bytes();
uint64_t nxg_dec_f64r_groups(uint64_t W);
// Records starting in [begin, end) of a W-byte frame (the whole frame: begin 0, end W).
hipError_t nxg_launch_dec_f64r(const uint8_t* wire, uint64_t W, uint64_t begin, uint64_t end,
                               uint64_t* oid, uint64_t* oval, uint64_t cap, void* desc,
                               uint64_t* tstat, uint32_t epoch, uint32_t flags, DevStatus* st,
                               hipStream_t s);
// A stream of whole frames (nxg_decode_frames_async): probe(0), then per frame one fused launch
// of emit(j) and probe(j + 1). Consecutive frames need different `desc` arrays; each frame has its
// own status slot and zero slot (`zst`, zeroed by its probe).
struct NxgF64rFrame {
    const uint8_t* wire;
    uint64_t W;
    uint64_t* oid;
    uint64_t* oval;
    uint64_t cap;
    void* desc;
    uint32_t epoch;
    DevStatus* st;
    DevStatus* zst;
};
hipError_t nxg_launch_dec_f64r_stream(const NxgF64rFrame* fr, uint32_t n, uint64_t* tstat,
                                      uint32_t flags, hipStream_t s);
uint64_t nxg_enc_f64_tiles(uint64_t n);  // tiles (and tstat words) of an f64 encode
hipError_t nxg_launch_enc_f64(const uint64_t* id, const uint64_t* val, uint64_t n, uint8_t* out,
                              uint64_t cap, uint64_t* tstat, uint32_t epoch, DevStatus* st,
                              int grid, hipStream_t s);
// f64 encode of a batch whose ids count up by one (nxg_encode_f64_seq.hip): one launch, no
// look-back; declines with fast_fail + DevStatus.irregular bit 2 (out NULL: sizing only)
uint64_t nxg_enc_f64s_groups(uint64_t n);
hipError_t nxg_launch_enc_f64s(const uint64_t* id, const uint64_t* val, uint64_t n, uint8_t* out,
                               uint64_t cap, DevStatus* st, hipStream_t s);
// the type-partitioned view (nxg_partition.hip): count + scan + offsets + place launches;
// `scratch` holds nxg_part_scratch_bytes(n) bytes; *off_out = the per-tag offsets (device, 257)
uint64_t nxg_part_scratch_bytes(uint64_t n);
hipError_t nxg_launch_partition(const uint8_t* tag, const uint64_t* fixed, const uint32_t* aux,
                                uint64_t n, uint8_t* scratch, uint32_t* rank, uint32_t* row_of,
                                uint64_t* dfixed, uint32_t* daux, uint64_t** off_out,
                                hipStream_t s);
uint64_t nxg_enc_general_tiles(uint64_t n);  // tiles (and tstat words) of a general encode
// arch_base > 0: archive-batch rows after an arch_base-byte count header (nxg_encode_general.hip)
hipError_t nxg_launch_enc_general(const ColsDesc& cols, const uint8_t* heap, uint8_t* out,
                                  uint64_t cap, uint64_t* scratch, uint64_t* tstat,
                                  uint32_t epoch, DevStatus* st, int grid, hipStream_t s,
                                  uint64_t arch_base = 0);
// general decode: count + resolve + emit + fix. `lws` holds nxg_dec_gen_scratch_bytes(W) bytes
// (64 u32 lane words per tile, then the emit pass's work list), `runs` gdec2::MAX_RUNS *
// RUN_WORDS u64, `base` gdec2::MAX_RUNS * 4 u64; none needs zeroing.
uint64_t nxg_dec_gen_tiles(uint64_t W);
uint64_t nxg_dec_gen_scratch_bytes(uint64_t W);
hipError_t nxg_launch_dec_gen(const uint8_t* wire, uint64_t W, const ColsDesc& cols, uint32_t* lws,
                              uint64_t* runs, uint64_t* base, int wgs, DevStatus* st,
                              hipStream_t s);
int nxg_dec_gen_wgs(int ncu);
// fast mixed decode (nxg_decode_mixed.hip): frames of Update messages shorter than 128 bytes with
// flat values; sets fast_fail for anything else. `scratch`: nxg_fmx_scratch_bytes(W), no zeroing.
uint64_t nxg_fmx_scratch_bytes(uint64_t W);
void nxg_fmx_wgs(int ncu, int* wgs);  // persistent grid sizes (count, emit)
// lean_count: the count pass from one-byte-prefix Update candidates only, then a recount of the
// tiles where that found no chain from every candidate kind (DevStatus.diag[5] counts them, with
// the resolve pass's recounts)
hipError_t nxg_launch_dec_fmx(const uint8_t* wire, uint64_t W, const ColsDesc& cols,
                              uint8_t* scratch, const int* wgs, DevStatus* st, hipStream_t s,
                              bool lean_count = false);
// the messages that start in [begin, end) of a W-byte frame (rows etc. from 0, text / control
// offsets in frame bytes); entry / exit (+1, relative to begin) in DevStatus.diag[2] / diag[3]
hipError_t nxg_launch_dec_fmx_range(const uint8_t* wire, uint64_t W, uint64_t begin, uint64_t end,
                                    const ColsDesc& cols, uint8_t* scratch, const int* wgs,
                                    DevStatus* st, hipStream_t s, bool lean_count = false);
// subscriber dispatch (nxg_dispatch.hip): `scratch` holds nxg_disp_scratch_bytes(n, n_chans)
// bytes (no initialisation needed); `unmatched` one u64.
uint64_t nxg_disp_scratch_bytes(uint64_t n, uint32_t n_chans);
hipError_t nxg_launch_dispatch(const NxgSubTable& tb, const uint64_t* id, uint64_t n,
                               uint8_t* scratch, uint64_t* chan_off, uint64_t* ent_sub,
                               uint64_t* ent_row, uint64_t cap, uint64_t* last_row,
                               uint64_t* unmatched, int ncu, hipStream_t s,
                               const uint8_t* row_mode = nullptr,
                               const uint32_t* to_client = nullptr);
// publisher commit (nxg_publish.hip): stage 1 counts slots and sets flags (dup, changed,
// unsupported: three u32 at nxg_pub_flags(scratch)); stage 2 routes the UpdateChanged rows
// (mode array for nxg_launch_dispatch, or null when the kinds route as they are).
struct NxgPubBatch {
    const uint64_t* id;
    const uint8_t* tag;
    const uint64_t* fixed;
    const uint32_t* aux;
    const uint8_t* ctag;  // the batch's children (Array/Map/Error(Value) elements)
    const uint64_t* cfixed;
    const uint32_t* caux;
    const uint8_t* heap;
    const uint8_t* kind;
    uint64_t n_rows;
};
uint64_t nxg_pub_scratch_bytes(uint64_t n, uint64_t n_slots);
hipError_t nxg_launch_pub_stage1(const NxgPubTable& tb, const NxgPubBatch& b, uint8_t* scratch,
                                 int ncu, hipStream_t s);
const uint32_t* nxg_pub_flags(uint8_t* scratch);
hipError_t nxg_launch_pub_stage2(const NxgPubTable& tb, const NxgPubBatch& b, uint8_t* scratch,
                                 bool dup, bool changed, int ncu, hipStream_t s,
                                 const uint8_t** mode_out);
// stage 3, when flags[3] is set: the UpdateChanged comparisons that need the stack walk
// (prev_used: nxg_pub_prev(scratch) if stage 2 sorted, else null)
hipError_t nxg_launch_pub_deep(const NxgPubTable& tb, const NxgPubBatch& b, uint8_t* scratch,
                               const uint32_t* prev_used, int ncu, hipStream_t s);
const uint32_t* nxg_pub_prev(uint8_t* scratch, uint64_t n, uint64_t n_slots);
// exclusive sums of M u32 counts into u64 offsets (nxg_publish.hip); bsum: M / 4096 + 2 words
hipError_t nxg_scan_u32(const uint32_t* hist, uint64_t M, uint64_t* off, uint64_t* bsum,
                        hipStream_t s);
// archive batches (nxg_archive.hip): Vec<BatchItem> decode. Synchronous on `s`.
struct NxgArchResult {
    uint64_t count, n_rows, n_children, consumed, err_offset;
    uint32_t err_kind;
    int rounds;  // chain rounds run (-1: the serial fallback)
};
uint64_t nxg_arch_scratch_bytes(uint64_t W);
// the fast path of archive batch decode (nxg_archive_fast.hip)
uint64_t nxg_fa_scratch_bytes(uint64_t W);
hipError_t nxg_launch_dec_fa(const uint8_t* buf, uint64_t W, uint32_t p0, uint64_t count,
                             const ColsDesc& cols, uint8_t* scratch, void* hhead, DevStatus* st,
                             hipStream_t s);
hipError_t nxg_arch_decode(const uint8_t* buf, uint64_t W, const ColsDesc& cols, uint8_t* scratch,
                           uint32_t* cap_flag, int max_rounds, NxgArchResult* res, hipStream_t s);
// zstd decompression of compressed archive records (nxg_zstd.hip): host-side table builders and
// the launch; the device structures are opaque here (their sizes from the *_bytes functions)
struct NxzDictDev;
struct NxzDefaults;
bool nxg_zstd_build_dict(const uint8_t* d, uint64_t n, NxzDictDev* out, uint64_t* content_off);
bool nxg_zstd_build_defaults(NxzDefaults* o);
void nxg_zstd_set_content(NxzDictDev* d, const uint8_t* dcontent);
uint64_t nxg_zstd_dict_dev_bytes();
uint64_t nxg_zstd_defaults_bytes();
uint64_t nxg_zstd_rec_bytes();
uint64_t nxg_zstd_res_bytes();
uint64_t nxg_zstd_litbuf_bytes();
int nxg_zstd_grid(int ncu);
hipError_t nxg_launch_zstd(const uint8_t* dsrc, const void* drecs, uint32_t n, const void* ddict,
                           const void* ddefs, uint8_t* dout, uint8_t* dlit, void* dres, int grid,
                           hipStream_t s);
// one share of a decoded frame's rows (nxg_share.hip): bounds (4 u64 in device memory: the first
// child slot of a container row >= r0 / >= r1, the first control span with ctl_row >= r0 / >= r1;
// ~0 for none), then the copy of rows [r0, r0 + nr), children [c0, c0 + nc) and control spans
// [k0, k0 + nk), re-based, with the Heartbeats among those spans counted into *hb (device u64)
hipError_t nxg_launch_share_bounds(const ColsDesc& src, uint64_t r0, uint64_t r1, uint64_t* b,
                                   hipStream_t s);
hipError_t nxg_launch_share_copy(const ColsDesc& src, const ColsDesc& dst, uint64_t r0,
                                 uint64_t nr, uint64_t c0, uint64_t nc, uint64_t k0, uint64_t nk,
                                 uint64_t* hb, hipStream_t s);
int nxg_occupancy_enc_f64();
int nxg_occupancy_enc_general();

// Device-side copy of the column pointers (passed by value to kernels).
struct ColsDesc {
    uint64_t cap_rows, cap_children, cap_ctl;
    uint64_t n_rows, n_children, n_ctl;  // encode input counts
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
};
