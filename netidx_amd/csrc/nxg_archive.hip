// nxg_archive.hip -- archive batches for gfx950: <GPooled<Vec<BatchItem>> as Pack>::decode
// (netidx-core/src/pack.rs:167-185, 934-973) with BatchItem(Id, Event)
// (netidx-archive/src/logfile/mod.rs:150-205) and Event::decode (netidx/src/subscriber/mod.rs:
// 154-177). A batch is
//     varint count | count x ( varint Id (as u32) | 0x40 = Unsubscribed, or a bare Value )
// and, unlike the publisher stream, no item carries a length: where an item ends follows from its
// value's tags alone (a String's length varint, an Array's count, ...).
//
// Boundary discovery without a sequential scan. The batch after the count is cut into 1 KiB
// chunks, one lane each.
//   spec    each lane walks item by item from its chunk's first byte, as if an item started
//           there (on a decode error it restarts one byte later), and records where its walk
//           leaves the chunk: a guessed exit.
//   chain   each lane walks its chunk again, exactly, from its predecessor's guessed exit:
//           the exit, items and child slots it meets. Lane 0 starts at the true first item, so
//           by induction every chunk is right up to the first chunk k whose guess differs from
//           what the chain computed for it (y[k] != guess[k]): lane k+1 walked from a wrong
//           entry. About 1.5 % of 1 KiB chunks of the config-3 mix are such breaks.
//   repair  one walker per break, in parallel: from the chain's exit of chunk k it walks chunk
//           k+1, k+2, ... until its exit equals the guess the next chunk's chain walk started
//           from (the chain rejoins; almost always after one chunk). Chunks that a long item
//           covers entirely pass through at no cost.
//   stitch  one workgroup takes the walkers in chunk order: a walker is real when it starts past
//           the previous real walker's path (+1, where the rejoin made the next chain walk true);
//           the others started from a wrong exit and are dropped. Real walkers' paths replace
//           the chain's values. A walker that does not rejoin within its budget hands the rest of
//           the batch to one lane that walks it in order (exact, slow, rare).
//   scan    exclusive sums of the items and child slots per chunk: each chunk's first row and
//           first child slot.
//   emit    each lane decodes its chunk's items from the true entry with full validation
//           (nxg_msg.h dvalue, the same restatement as the publisher-stream decoder) into rows
//           rbase.. and children cbase.., depth-first as the reference allocates them.
//   final   status: the first error in stream order among the first `count` items, rows,
//           children and the bytes consumed (the end of item count - 1).
// Items past `count` (the rest of an mmap'd file follows a record's batch, reader.rs:449) are
// walked but never written or reported.
#include <utility>

#include "nxg_internal.h"
#include "nxg_msg.h"

namespace {

using namespace nxgmsg;

#ifndef NXG_ARCH_CH
#define NXG_ARCH_CH 1024  // timing experiments: 512 and 256 measured slower (more breaks)
#endif
constexpr uint32_t CH = NXG_ARCH_CH;  // bytes per chunk (one lane)
constexpr uint32_t TPB = 256;
constexpr uint64_t ERR = ~0ull;       // a chunk exit after a structural decode error
constexpr uint32_t BATCH_ITEM = 24;   // size_of::<BatchItem>() for check_sz! (parity unpinned)
constexpr uint32_t UNSUB = 0x40;      // Event::Unsubscribed (subscriber/mod.rs:168)
constexpr DMode kStruct{0xffffffffu, 1, 0};  // boundaries only: no UTF-8 scan, no writes
constexpr DMode kEmit{0xffffffffu, 0, 1};    // full validation, written to the columns

}  // namespace

// The batch header and the call's device-side results (scratch memory).
struct ArchHead {
    uint64_t count, p0;  // items, first item
    uint32_t err_kind;   // header error (count varint, size guard)
    uint32_t pad;
    uint64_t err_key;    // first item error: err_key(offset, kind), atomicMax
    uint64_t end;        // 1 + the end of item count - 1 (0: not seen)
    uint64_t end_children;
    uint32_t again;      // chain round: some exit changed
    uint32_t pad2;
};

namespace {

// One item at p: varint Id, then the Event. Structure mode (EMIT false, md kStruct or a bounded
// spec mode) or a full decode into row `row`.
template <bool EMIT>
NXG_DEV uint32_t arch_item(const GlbSrc& g, uint64_t& p, uint64_t W, const Sink* k, uint64_t row,
                           uint64_t& child_next, uint32_t& work, const DMode& md, uint64_t& id) {
    uint32_t e = dvar(g, p, W, id);
    if (e) return e;
    if (p >= W) return E_SHORT;  // Event::decode reads chunk()[0]: a panic in the reference
    if (g.byte(p) == UNSUB) {
        p++;
        put<EMIT>(k, md.write, true, row, UNSUB, 0, 0);
        return E_OK;
    }
    return dvalue<EMIT>(g, p, W, k, true, row, child_next, work, md);
}

NXG_DEV uint64_t chunk_start(const ArchHead& h, uint64_t k) { return h.p0 + k * CH; }

// the chain walk of chunk k from `entry`: exit (ERR on a structural error), items, child slots
NXG_DEV void chain_chunk(const GlbSrc& g, uint64_t W, uint64_t s, uint64_t entry, uint64_t& exit,
                         uint32_t& items, uint32_t& kids) {
    items = 0;
    kids = 0;
    if (entry == ERR) {
        exit = ERR;
        return;
    }
    const uint64_t lim = s + CH < W ? s + CH : W;
    uint64_t q = entry;
#pragma unroll 1
    while (q < lim) {
        uint64_t r = q, cn = 0, id;
        uint32_t work = 0;
        if (arch_item<false>(g, r, W, nullptr, 0, cn, work, kStruct, id)) {
            exit = ERR;
            return;
        }
        items++;
        kids += (uint32_t)cn;
        q = r;
    }
    exit = q;
}

}  // namespace

// header: varint count and check_sz!(count, remaining, BatchItem) (pack.rs:919-925, 955-956)
__global__ void nxg_arch_head_kernel(const uint8_t* __restrict__ buf, uint64_t W,
                                     ArchHead* __restrict__ h) {
    const GlbSrc g{(gbl_bytes)buf};
    ArchHead r{};
    uint64_t p = 0, count = 0;
    uint32_t e = dvar(g, p, W, count);
    if (!e) {
        const uint64_t sz = count > ~0ull / BATCH_ITEM ? ~0ull : count * BATCH_ITEM;
        if (sz > kMaxVec || sz > ((W - p) << 8)) e = E_TOO_BIG;
    }
    r.count = e ? 0 : count;
    r.p0 = e ? W : p;
    r.err_kind = e;
    *h = r;
}

// guessed exits: the walk from the chunk's first byte, restarting one byte later on an error
__global__ __launch_bounds__(TPB) void nxg_arch_spec_kernel(const uint8_t* __restrict__ buf,
                                                            uint64_t W, uint64_t nch,
                                                            const ArchHead* __restrict__ hp,
                                                            uint64_t* __restrict__ xg) {
    const uint64_t k = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (k >= nch) return;
    const ArchHead h = *hp;
    const uint64_t s = chunk_start(h, k);
    if (h.err_kind || s >= W) {
        xg[k] = W;
        return;
    }
    const GlbSrc g{(gbl_bytes)buf};
    const uint64_t lim = s + CH < W ? s + CH : W;
    const DMode md{kWalkBudget, 1, 0};
    uint64_t q = s;
#pragma unroll 1
    while (q < lim) {
        uint64_t r = q, cn = 0, id;
        uint32_t work = 0;
        if (arch_item<false>(g, r, W, nullptr, 0, cn, work, md, id)) q++;
        else q = r;
    }
    xg[k] = q;
}

// the chain walk of every chunk from its predecessor's guessed exit
__global__ __launch_bounds__(TPB) void nxg_arch_chain_kernel(
    const uint8_t* __restrict__ buf, uint64_t W, uint64_t nch, const ArchHead* __restrict__ hp,
    const uint64_t* __restrict__ xg, uint64_t* __restrict__ y, uint32_t* __restrict__ n,
    uint32_t* __restrict__ c, uint32_t* __restrict__ brk) {
    const uint64_t k = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (k >= nch) return;
    const ArchHead h = *hp;
    uint64_t x = W;
    uint32_t items = 0, kids = 0;
    if (!h.err_kind) {
        const GlbSrc g{(gbl_bytes)buf};
        chain_chunk(g, W, chunk_start(h, k), k == 0 ? h.p0 : xg[k - 1], x, items, kids);
    }
    y[k] = x;
    n[k] = items;
    c[k] = kids;
    // a break: the next chunk's chain walk started from a guess the chain does not produce
    brk[k] = k + 1 < nch && x != xg[k] && x != ERR;
}

// walker records: chunks [from, from + count) exit at `exit` with n items, c child slots (count
// > 1 only for chunks a long item passes through: n = c = 0)
struct ArchRec {
    uint64_t exit;
    uint32_t from, count, n, c;
};
constexpr uint32_t WREC = 16;   // records per walker
constexpr uint32_t WWALK = 8;   // chunk walks per walker
struct ArchWalker {
    uint32_t start;  // first chunk of the path (the break's chunk + 1)
    uint32_t nrec;
    uint32_t last;   // last chunk of the path
    uint32_t state;  // 0 rejoined (or reached the end), 1 out of budget, 2 decode error
};

// break list in chunk order: brk (scanned to pos) -> start chunks
__global__ __launch_bounds__(TPB) void nxg_arch_brk_kernel(const uint32_t* __restrict__ brk,
                                                           const uint64_t* __restrict__ pos,
                                                           uint64_t nch, uint64_t maxw,
                                                           ArchWalker* __restrict__ w) {
    const uint64_t k = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (k < nch && brk[k] && pos[k] < maxw) w[pos[k]].start = (uint32_t)(k + 1);
}

__global__ __launch_bounds__(TPB) void nxg_arch_walk_kernel(
    const uint8_t* __restrict__ buf, uint64_t W, uint64_t nch, const ArchHead* __restrict__ hp,
    const uint64_t* __restrict__ xg, const uint64_t* __restrict__ y, uint64_t nw,
    ArchWalker* __restrict__ w, ArchRec* __restrict__ rec) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= nw) return;
    const ArchHead h = *hp;
    const GlbSrc g{(gbl_bytes)buf};
    ArchWalker wk = w[i];
    ArchRec* r = rec + i * WREC;
    uint64_t j = wk.start, e = y[j - 1];
    uint32_t nrec = 0, walks = 0, state = 1;
#pragma unroll 1
    while (nrec < WREC && walks < WWALK) {
        const uint64_t s = chunk_start(h, j);
        const uint64_t lim = s + CH < W ? s + CH : W;
        if (e >= lim && j + 1 < nch) {  // chunks j.. that the item before e covers entirely
            uint64_t home = (e - h.p0) / CH;
            if (home > nch - 1) home = nch - 1;
            r[nrec++] = ArchRec{e, (uint32_t)j, (uint32_t)(home - j), 0, 0};
            j = home;
            if (e == xg[j - 1]) {  // chunk `home` walked from e in the chain pass: rejoined
                state = 0;
                break;
            }
            continue;
        }
        uint64_t x;
        uint32_t items, kids;
        chain_chunk(g, W, s, e, x, items, kids);
        walks++;
        r[nrec++] = ArchRec{x, (uint32_t)j, 1, items, kids};
        if (x == ERR) {
            state = 2;
            break;
        }
        if (j + 1 >= nch || x == xg[j]) {  // the end, or the next chain walk started from x
            state = 0;
            break;
        }
        e = x;
        j++;
    }
    wk.nrec = nrec;  // >= 1: the loop makes at least one record
    wk.last = r[nrec - 1].from + r[nrec - 1].count - 1;  // the path's last chunk
    wk.state = state;
    w[i] = wk;
}

// the walkers in chunk order: real ones start past the previous real walker's path + 1. Marks
// them (state |= 8) and writes the chunk from which one lane must walk on (or nch) to *resume.
// One wave: 64 walkers per step in lane registers, taken in order with uniform readlanes.
__global__ __launch_bounds__(64) void nxg_arch_stitch_kernel(uint64_t nw, uint64_t nch,
                                                             ArchWalker* __restrict__ w,
                                                             uint64_t* __restrict__ resume) {
    const uint32_t lane = threadIdx.x;
    int64_t last = -2;  // the previous real walker's last chunk (uniform)
    uint64_t res = nch;
    bool stop = false;
#pragma unroll 1
    for (uint64_t b = 0; b < nw && !stop; b += 64) {
        const uint64_t i = b + lane;
        ArchWalker x{};
        if (i < nw) x = w[i];
        const uint32_t m = (uint32_t)(nw - b < 64 ? nw - b : 64);
        uint64_t real = 0;  // lane mask of the real walkers in this step
#pragma unroll 1
        for (uint32_t q = 0; q < m; q++) {
            const int64_t st = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)x.start, (int)q);
            if (st <= last + 1) continue;  // started from a wrong exit
            real |= 1ull << q;
            const uint32_t state = (uint32_t)__builtin_amdgcn_readlane((int)x.state, (int)q);
            const int64_t ls = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)x.last, (int)q);
            if (state == 1u) {  // out of budget: one lane walks on from here
                res = (uint64_t)ls + 1;
                stop = true;
                break;
            }
            if (state == 2u) {  // the batch's first error: nothing after matters
                stop = true;
                break;
            }
            last = ls;
        }
        if (i < nw && ((real >> lane) & 1ull)) w[i].state = x.state | 8u;
    }
    if (lane == 0) *resume = res;
}

// real walkers' paths replace the chain's values
__global__ __launch_bounds__(TPB) void nxg_arch_apply_kernel(uint64_t nw,
                                                             const ArchWalker* __restrict__ w,
                                                             const ArchRec* __restrict__ rec,
                                                             uint64_t* __restrict__ y,
                                                             uint32_t* __restrict__ n,
                                                             uint32_t* __restrict__ c) {
    const uint64_t i = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (i >= nw || !(w[i].state & 8u)) return;
    const ArchWalker wk = w[i];
    for (uint32_t q = 0; q < wk.nrec; q++) {
        const ArchRec r = rec[i * WREC + q];
        for (uint32_t j = r.from; j < r.from + r.count; j++) {
            y[j] = r.exit;
            n[j] = r.n;
            c[j] = r.c;
        }
    }
}

// the fallback: one lane walks the chain in order from chunk `from` (every exit before it true)
__global__ void nxg_arch_serial_kernel(const uint8_t* __restrict__ buf, uint64_t W, uint64_t nch,
                                       const ArchHead* __restrict__ hp,
                                       const uint64_t* __restrict__ from_p,
                                       uint64_t* __restrict__ x, uint32_t* __restrict__ n,
                                       uint32_t* __restrict__ c) {
    const ArchHead h = *hp;
    const uint64_t from = *from_p;
    if (h.err_kind || from >= nch) return;
    const GlbSrc g{(gbl_bytes)buf};
    uint64_t entry = from == 0 ? h.p0 : x[from - 1];
#pragma unroll 1
    for (uint64_t k = from; k < nch; k++) {
        uint32_t items, kids;
        chain_chunk(g, W, chunk_start(h, k), entry, x[k], items, kids);
        n[k] = items;
        c[k] = kids;
        entry = x[k];
    }
}

// decode every item of the chunk from its true entry
__global__ __launch_bounds__(TPB) void nxg_arch_emit_kernel(
    const uint8_t* __restrict__ buf, uint64_t W, uint64_t nch, ArchHead* __restrict__ hp,
    const uint64_t* __restrict__ x, const uint64_t* __restrict__ rbase,
    const uint64_t* __restrict__ cbase, ColsDesc cols, uint32_t* __restrict__ cap_flag) {
    const uint64_t k = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    if (k >= nch) return;
    const ArchHead h = *hp;
    if (h.err_kind) return;
    const uint64_t entry = k == 0 ? h.p0 : x[k - 1];
    if (entry == ERR) return;
    const GlbSrc g{(gbl_bytes)buf};
    const Sink sink{cols, cap_flag, cap_flag};
    const uint64_t s = chunk_start(h, k);
    const uint64_t lim = s + CH < W ? s + CH : W;
    uint64_t q = entry, row = rbase[k], cn = cbase[k];
    if (h.count == 0 && k == 0) {  // an empty batch ends after its count
        hp->end = h.p0 + 1;
        hp->end_children = 0;
        return;
    }
#pragma unroll 1
    for (;;) {
        // (the batch's end is written only by the lane that decodes item count - 1: a chunk after
        // it may be walked from a wrong entry in trailing bytes and reach row == count too)
        if (q >= lim || row >= h.count) return;
        if (row >= cols.cap_rows) {
            atomicMax((unsigned long long*)&hp->err_key, err_key(q, NXG_CAPACITY));
            return;
        }
        uint64_t r = q, id;
        uint32_t work = 0;
        const uint32_t e = arch_item<true>(g, r, W, &sink, row, cn, work, kEmit, id);
        if (!e && cn > cols.cap_children) {
            atomicMax((unsigned long long*)&hp->err_key, err_key(q, NXG_CAPACITY));
            return;
        }
        if (e) {
            atomicMax((unsigned long long*)&hp->err_key, err_key(q, e));
            return;
        }
        cols.id[row] = (uint32_t)id;
        row++;
        q = r;
        if (row == h.count) {  // the batch ends here
            hp->end = q + 1;
            hp->end_children = cn;
            return;
        }
    }
}

// ---- launch (host) ------------------------------------------------------------------------------
uint64_t nxg_arch_chunks(uint64_t W) { return W / CH + 2; }

static uint64_t arch_max_walkers(uint64_t nch) { return nch / 4 + 64; }

uint64_t nxg_arch_scratch_bytes(uint64_t W) {
    const uint64_t nch = nxg_arch_chunks(W);
    const uint64_t mw = arch_max_walkers(nch);
    // head, guesses, exits, rbase, cbase, wpos, bsum x3, n, c, brk, walkers, records, resume
    return 256 + 8 * nch * 5 + 3 * 8 * (nch / 1024 + 2) + 4 * nch * 3 + 16 * mw +
           sizeof(ArchRec) * WREC * mw + 64 + 64;
}

struct ArchScratch {
    ArchHead* head;
    uint64_t *xg, *y, *rbase, *cbase, *wpos, *bs0, *bs1, *bs2, *resume;
    uint32_t *n, *c, *brk;
    ArchWalker* w;
    ArchRec* rec;
};

static ArchScratch arch_layout(uint8_t* p, uint64_t nch) {
    ArchScratch a;
    const uint64_t mw = arch_max_walkers(nch);
    a.head = reinterpret_cast<ArchHead*>(p);
    p += 256;
    auto u64 = [&](uint64_t cnt) {
        uint64_t* r = reinterpret_cast<uint64_t*>(p);
        p += 8 * cnt;
        return r;
    };
    a.xg = u64(nch);
    a.y = u64(nch);
    a.rbase = u64(nch);
    a.cbase = u64(nch);
    a.wpos = u64(nch);
    a.bs0 = u64(nch / 1024 + 2);
    a.bs1 = u64(nch / 1024 + 2);
    a.bs2 = u64(nch / 1024 + 2);
    a.resume = u64(8);
    a.rec = reinterpret_cast<ArchRec*>(p);
    p += sizeof(ArchRec) * WREC * mw;
    a.w = reinterpret_cast<ArchWalker*>(p);
    p += 16 * mw;
    a.n = reinterpret_cast<uint32_t*>(p);
    p += 4 * nch;
    a.c = reinterpret_cast<uint32_t*>(p);
    p += 4 * nch;
    a.brk = reinterpret_cast<uint32_t*>(p);
    return a;
}

// Decode the batch in buf[0, W). `scratch`: nxg_arch_scratch_bytes(W) bytes, no initialisation.
// Writes the result to host memory `res` (count, rows, children, consumed, error).
hipError_t nxg_arch_decode(const uint8_t* buf, uint64_t W, const ColsDesc& cols, uint8_t* scratch,
                           uint32_t* cap_flag, int max_rounds, NxgArchResult* res,
                           hipStream_t s) {
    (void)max_rounds;
    const uint64_t nch = nxg_arch_chunks(W);
    const uint64_t mw = arch_max_walkers(nch);
    const ArchScratch a = arch_layout(scratch, nch);
    const uint32_t grid = (uint32_t)((nch + TPB - 1) / TPB);
    hipError_t e;
    if ((e = hipMemsetAsync(a.head, 0, sizeof(ArchHead), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(nxg_arch_head_kernel, dim3(1), dim3(1), 0, s, buf, W, a.head);
    hipLaunchKernelGGL(nxg_arch_spec_kernel, dim3(grid), dim3(TPB), 0, s, buf, W, nch, a.head, a.xg);
    hipLaunchKernelGGL(nxg_arch_chain_kernel, dim3(grid), dim3(TPB), 0, s, buf, W, nch, a.head,
                       a.xg, a.y, a.n, a.c, a.brk);
    if ((e = nxg_scan_u32(a.brk, nch, a.wpos, a.bs2, s)) != hipSuccess) return e;
    uint64_t nw = 0;
    uint32_t lastb = 0;
    if ((e = hipMemcpyAsync(&nw, a.wpos + nch - 1, 8, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return e;
    if ((e = hipMemcpyAsync(&lastb, a.brk + nch - 1, 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    nw += lastb;
    res->rounds = (int)(nw < 0x7fffffff ? nw : 0x7fffffff);  // breaks repaired
    if (nw > mw) {  // too many breaks for the walkers: one lane walks the whole chain
        if ((e = hipMemsetAsync(a.resume, 0, 8, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(nxg_arch_serial_kernel, dim3(1), dim3(1), 0, s, buf, W, nch, a.head,
                           a.resume, a.y, a.n, a.c);
        res->rounds = -1;
    } else if (nw) {
        const uint32_t gw = (uint32_t)((nw + TPB - 1) / TPB);
        hipLaunchKernelGGL(nxg_arch_brk_kernel, dim3(grid), dim3(TPB), 0, s, a.brk, a.wpos, nch, mw,
                           a.w);
        hipLaunchKernelGGL(nxg_arch_walk_kernel, dim3(gw), dim3(TPB), 0, s, buf, W, nch, a.head,
                           a.xg, a.y, nw, a.w, a.rec);
        hipLaunchKernelGGL(nxg_arch_stitch_kernel, dim3(1), dim3(64), 0, s, nw, nch, a.w,
                           a.resume);
        hipLaunchKernelGGL(nxg_arch_apply_kernel, dim3(gw), dim3(TPB), 0, s, nw, a.w, a.rec, a.y,
                           a.n, a.c);
        hipLaunchKernelGGL(nxg_arch_serial_kernel, dim3(1), dim3(1), 0, s, buf, W, nch, a.head,
                           a.resume, a.y, a.n, a.c);
    }
    const uint64_t* xin = a.y;
    if ((e = nxg_scan_u32(a.n, nch, a.rbase, a.bs0, s)) != hipSuccess) return e;
    if ((e = nxg_scan_u32(a.c, nch, a.cbase, a.bs1, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(nxg_arch_emit_kernel, dim3(grid), dim3(TPB), 0, s, buf, W, nch, a.head, xin,
                       a.rbase, a.cbase, cols, cap_flag);
    ArchHead h;
    uint64_t last[3];
    if ((e = hipMemcpyAsync(&h, a.head, sizeof h, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(&last[0], xin + nch - 1, 8, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return e;
    if ((e = hipMemcpyAsync(&last[1], a.rbase + nch - 1, 8, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return e;
    uint32_t nl = 0;
    if ((e = hipMemcpyAsync(&nl, a.n + nch - 1, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    last[2] = last[1] + nl;  // items on the chain
    res->count = h.count;
    res->n_rows = 0;
    res->n_children = 0;
    res->consumed = 0;
    res->err_kind = 0;
    res->err_offset = 0;
    if (h.err_kind) {
        res->err_kind = h.err_kind;
        return hipSuccess;
    }
    if (h.err_key) {
        const uint64_t key = ~h.err_key;
        res->err_kind = (uint32_t)(key & 0xff);
        res->err_offset = key >> 8;
        return hipSuccess;
    }
    if (!h.end) {  // the chain ended (at W) before `count` items: the next Id varint is short
        res->err_kind = E_SHORT;
        res->err_offset = last[0] == ERR ? W : last[0];
        (void)last[2];
        return hipSuccess;
    }
    res->n_rows = h.count;
    res->n_children = h.end_children;
    res->consumed = h.end - 1;
    return hipSuccess;
}
