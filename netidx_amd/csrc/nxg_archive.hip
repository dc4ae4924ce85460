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
//   chain   each lane walks its chunk again from its predecessor's guessed exit -- the true
//           entry if the predecessor's guess was right -- and records the exit, the items and the
//           child slots it met. Lane 0 starts at the true first item. A chunk whose exit differs
//           from the guess re-runs its successor in the next round; rounds repeat until no exit
//           changes (a wrong walk re-synchronises with the true one within a few items, so this
//           ends after one or two rounds). After the last round every exit is on the true chain
//           by induction from chunk 0. A bounded number of rounds, then one lane walks the
//           remaining chain in order (still exact, only slower).
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

constexpr uint32_t CH = 1024;  // bytes per chunk (one lane)
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

// one chain round: chunks whose entry changed (all of them in round 0) walk from it
__global__ __launch_bounds__(TPB) void nxg_arch_chain_kernel(
    const uint8_t* __restrict__ buf, uint64_t W, uint64_t nch, ArchHead* __restrict__ hp,
    const uint64_t* __restrict__ xin, uint64_t* __restrict__ xout, const uint8_t* __restrict__ cin,
    uint8_t* __restrict__ cout, uint32_t* __restrict__ n, uint32_t* __restrict__ c, int first) {
    const uint64_t k = (uint64_t)blockIdx.x * TPB + threadIdx.x;
    bool chg = false;
    if (k < nch) {
        const ArchHead h = *hp;
        const bool run = !h.err_kind && (first || (k > 0 && cin[k - 1]));
        if (run) {
            const GlbSrc g{(gbl_bytes)buf};
            const uint64_t entry = k == 0 ? h.p0 : xin[k - 1];
            uint64_t x;
            uint32_t items, kids;
            chain_chunk(g, W, chunk_start(h, k), entry, x, items, kids);
            n[k] = items;
            c[k] = kids;
            xout[k] = x;
            chg = x != xin[k];
        } else {
            xout[k] = xin[k];
            if (h.err_kind) n[k] = c[k] = 0;
        }
        cout[k] = chg;
    }
    if (__any(chg) && (threadIdx.x & 63) == 0) atomicOr(&hp->again, 1u);
}

// the fallback: one lane walks the chain in order from chunk `from` (every entry before it true)
__global__ void nxg_arch_serial_kernel(const uint8_t* __restrict__ buf, uint64_t W, uint64_t nch,
                                       const ArchHead* __restrict__ hp, uint64_t* __restrict__ x,
                                       uint32_t* __restrict__ n, uint32_t* __restrict__ c) {
    const ArchHead h = *hp;
    if (h.err_kind) return;
    const GlbSrc g{(gbl_bytes)buf};
    uint64_t entry = h.p0;
#pragma unroll 1
    for (uint64_t k = 0; k < nch; k++) {
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
#pragma unroll 1
    for (;;) {
        if (row == h.count) {  // the batch ends here
            hp->end = q + 1;
            hp->end_children = cn;
            return;
        }
        if (q >= lim || row > h.count) return;
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
    }
}

// ---- launch (host) ------------------------------------------------------------------------------
uint64_t nxg_arch_chunks(uint64_t W) { return W / CH + 2; }

uint64_t nxg_arch_scratch_bytes(uint64_t W) {
    const uint64_t nch = nxg_arch_chunks(W);
    // head, x0, x1, rbase, cbase, bsum x2, n, c, chg0, chg1
    return 256 + 8 * nch * 4 + 2 * 8 * (nch / 1024 + 2) + 4 * nch * 2 + 2 * nch + 64;
}

struct ArchScratch {
    ArchHead* head;
    uint64_t *x0, *x1, *rbase, *cbase, *bs0, *bs1;
    uint32_t *n, *c;
    uint8_t *chg0, *chg1;
};

static ArchScratch arch_layout(uint8_t* p, uint64_t nch) {
    ArchScratch a;
    a.head = reinterpret_cast<ArchHead*>(p);
    p += 256;
    auto u64 = [&](uint64_t cnt) {
        uint64_t* r = reinterpret_cast<uint64_t*>(p);
        p += 8 * cnt;
        return r;
    };
    a.x0 = u64(nch);
    a.x1 = u64(nch);
    a.rbase = u64(nch);
    a.cbase = u64(nch);
    a.bs0 = u64(nch / 1024 + 2);
    a.bs1 = u64(nch / 1024 + 2);
    a.n = reinterpret_cast<uint32_t*>(p);
    p += 4 * nch;
    a.c = reinterpret_cast<uint32_t*>(p);
    p += 4 * nch;
    a.chg0 = p;
    p += nch;
    a.chg1 = p;
    return a;
}

// Decode the batch in buf[0, W). `scratch`: nxg_arch_scratch_bytes(W) bytes, no initialisation.
// Writes the result to host memory `res` (count, rows, children, consumed, error).
hipError_t nxg_arch_decode(const uint8_t* buf, uint64_t W, const ColsDesc& cols, uint8_t* scratch,
                           uint32_t* cap_flag, int max_rounds, NxgArchResult* res,
                           hipStream_t s) {
    const uint64_t nch = nxg_arch_chunks(W);
    const ArchScratch a = arch_layout(scratch, nch);
    const uint32_t grid = (uint32_t)((nch + TPB - 1) / TPB);
    hipError_t e;
    if ((e = hipMemsetAsync(a.head, 0, sizeof(ArchHead), s)) != hipSuccess) return e;
    hipLaunchKernelGGL(nxg_arch_head_kernel, dim3(1), dim3(1), 0, s, buf, W, a.head);
    hipLaunchKernelGGL(nxg_arch_spec_kernel, dim3(grid), dim3(TPB), 0, s, buf, W, nch, a.head, a.x0);
    uint64_t *xin = a.x0, *xout = a.x1;
    uint8_t *cin = a.chg0, *cout = a.chg1;
    bool done = false;
    for (int round = 0; round < max_rounds && !done; round++) {
        hipLaunchKernelGGL(nxg_arch_chain_kernel, dim3(grid), dim3(TPB), 0, s, buf, W, nch, a.head,
                           xin, xout, cin, cout, a.n, a.c, round == 0 ? 1 : 0);
        std::swap(xin, xout);
        std::swap(cin, cout);
        uint32_t again = 0;
        if ((e = hipMemcpyAsync(&again, &a.head->again, 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
            return e;
        if ((e = hipMemsetAsync(&a.head->again, 0, 4, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        done = again == 0;
        res->rounds = round + 1;
    }
    if (!done) {  // exact, one lane: the chain in order
        hipLaunchKernelGGL(nxg_arch_serial_kernel, dim3(1), dim3(1), 0, s, buf, W, nch, a.head, xin,
                           a.n, a.c);
        res->rounds = -1;
    }
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
