/*
 * nx_oracle.c -- TEST INFRASTRUCTURE ONLY (see nx_oracle.h). Never linked into the product.
 *
 * Scalar, sequential restatement of the reference Pack codec, one message at a time, exactly as
 * ReadChannel::receive_batch_fn (netidx/src/channel.rs:504-521) drives From::decode and
 * WriteChannel::queue_send (channel.rs:177-202) drives From::encode.
 *
 * Buffer model: the reference decodes from a contiguous PBuf through nested bytes::Take
 * wrappers. chunk() of a Take is [pos, min(limit, end)), so every reader below sees the window
 * [pos, lim) of a Buf and nothing past lim.
 */
#include "nx_oracle.h"
#include <string.h>
#include <stdlib.h>

#define MAX_VEC ((uint64_t)2 * 1024 * 1024 * 1024) /* pack.rs:917 */

typedef struct Buf {
    const uint8_t* w;
    uint64_t pos;
    uint64_t lim;
} Buf;

static inline uint64_t rem(const Buf* b) { return b->lim - b->pos; }

/* pack.rs:472-474 */
uint32_t nxo_varint_len(uint64_t v) {
    uint32_t hb = (uint32_t)__builtin_clzll(v | 1) ^ 63u;
    return (hb * 9u + 73u) >> 6;
}

/* pack.rs:476-486 */
uint32_t nxo_encode_varint(uint64_t v, uint8_t* out) {
    uint32_t n = 0;
    for (int i = 0; i < 10; i++) {
        if (v < 0x80) {
            out[n++] = (uint8_t)v;
            break;
        }
        out[n++] = (uint8_t)((v & 0x7F) | 0x80);
        v >>= 7;
    }
    return n;
}

/* pack.rs:504-520: reads at most 10 bytes from chunk(); BufferShort if the chunk ends first;
 * InvalidFormat if the 10th byte still has its continuation bit; bits past 64 are dropped. */
int nxo_decode_varint(const uint8_t* p, uint64_t avail, uint64_t* v, uint32_t* nread) {
    uint64_t value = 0;
    for (uint32_t i = 0; i < 10; i++) {
        if (i >= avail) return NXO_BUFFER_SHORT;
        uint8_t byte = p[i];
        value |= ((uint64_t)(byte & 0x7F)) << (i * 7);
        if (byte <= 0x7F) {
            *v = value;
            *nread = i + 1;
            return NXO_OK;
        }
    }
    *nread = 10;
    return NXO_INVALID_FORMAT;
}

/* pack.rs:522-525 */
uint32_t nxo_len_wrapped_len(uint64_t len) {
    return (uint32_t)(len + nxo_varint_len(len + nxo_varint_len(len)));
}
static inline uint64_t lwlen(uint64_t len) { return len + nxo_varint_len(len + nxo_varint_len(len)); }

/* netidx-core/src/test.rs:16-63 (check_encode_decode / check_encode_decode_short) */
uint64_t nxo_varint_sweep(uint64_t lo, uint64_t hi, int short_buf) {
    uint64_t fails = 0;
    uint8_t buf[16];
    uint64_t cap = short_buf ? 7 : 16;
    for (uint64_t d = lo; d < hi; d++) {
        memset(buf, 0, sizeof buf);
        uint32_t n = nxo_encode_varint(d, buf);
        uint64_t u = 0;
        uint32_t nr = 0;
        int e = nxo_decode_varint(buf, cap, &u, &nr);
        if (e || u != d || nr != nxo_varint_len(d) || n != nr || cap - nr != cap - nxo_varint_len(d))
            fails++;
    }
    return fails;
}

static int dvar(Buf* b, uint64_t* v) {
    uint32_t n = 0;
    int e = nxo_decode_varint(b->w + b->pos, rem(b), v, &n);
    if (e == NXO_INVALID_FORMAT) b->pos += 10;
    if (e) return e;
    b->pos += n;
    return NXO_OK;
}

static inline uint64_t be(const uint8_t* p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | p[i];
    return v;
}

/* fixed-width BE primitive (pack.rs:557-874): remaining() < size -> BufferShort */
static int dfix(Buf* b, int n, uint64_t* v) {
    if (rem(b) < (uint64_t)n) return NXO_BUFFER_SHORT;
    *v = be(b->w + b->pos, n);
    b->pos += n;
    return NXO_OK;
}

/* std::str::from_utf8 (pack.rs:462) */
int nxo_utf8_valid(const uint8_t* p, uint64_t n) {
    uint64_t i = 0;
    while (i < n) {
        uint8_t c = p[i];
        if (c < 0x80) {
            i++;
            continue;
        }
        uint8_t lo = 0x80, hi = 0xBF;
        int need;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c == 0xE0) { need = 2; lo = 0xA0; }
        else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) need = 2;
        else if (c == 0xED) { need = 2; hi = 0x9F; }
        else if (c == 0xF0) { need = 3; lo = 0x90; }
        else if (c >= 0xF1 && c <= 0xF3) need = 3;
        else if (c == 0xF4) { need = 3; hi = 0x8F; }
        else return 0;
        if (i + (uint64_t)need >= n) return 0; /* truncated sequence */
        uint8_t c1 = p[i + 1];
        if (c1 < lo || c1 > hi) return 0;
        for (int k = 2; k <= need; k++)
            if ((p[i + k] & 0xC0) != 0x80) return 0;
        i += need + 1;
    }
    return 1;
}

/* proleptic Gregorian days since 1970-01-01 (H. Hinnant's days_from_civil) */
static int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
    y -= m <= 2;
    int64_t era = (y >= 0 ? y : y - 399) / 400;
    int64_t yoe = y - era * 400;
    int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + doe - 719468;
}

/* chrono DateTime::from_timestamp(secs, nsecs) (called at pack.rs:1572).
 * chrono is not vendored; Cargo.toml pins "^0.4.24" with no lock file. Restated from chrono
 * >= 0.4.35: NaiveDate range [-262143-01-01, 262142-12-31], nsecs < 2e9, and nsecs >= 1e9
 * (leap second) only when secs % 60 == 59. Edge validity is "parity unpinned" (SURVEY 8c). */
int nxo_datetime_valid(int64_t secs, uint32_t nsecs) {
    int64_t days = secs / 86400;
    int64_t sod = secs % 86400;
    if (sod < 0) {
        sod += 86400;
        days -= 1;
    }
    int64_t days_ce = days + 719163; /* UNIX_EPOCH_DAY: days from CE of 1970-01-01 */
    static int64_t min_ce = 0, max_ce = 0;
    if (!min_ce) {
        min_ce = days_from_civil(-262143, 1, 1) + 719163;
        max_ce = days_from_civil(262142, 12, 31) + 719163;
    }
    if (days_ce < min_ce || days_ce > max_ce) return 0;
    if (nsecs >= 2000000000u) return 0;
    if (nsecs >= 1000000000u && sod % 60 != 59) return 0;
    return 1;
}

/* ---------------------------------------------------------------------------------------------
 * Value decode (netidx-value/src/lib.rs:470-506) into the columnar contract.
 * ------------------------------------------------------------------------------------------- */
typedef struct Ctx {
    NxoCols* c;
    int emit; /* 0: validate only (values inside control messages) */
} Ctx;

static void put_slot(Ctx* x, int is_row, uint64_t slot, uint8_t tag, uint64_t fixed, uint32_t aux) {
    if (!x->emit) return;
    if (is_row) {
        x->c->tag[slot] = tag;
        x->c->fixed[slot] = fixed;
        x->c->aux[slot] = aux;
    } else {
        x->c->ctag[slot] = tag;
        x->c->cfixed[slot] = fixed;
        x->c->caux[slot] = aux;
    }
}

static int alloc_children(Ctx* x, uint64_t k, uint64_t* base) {
    *base = x->c->n_children;
    if (!x->emit) return NXO_OK;
    if (x->c->n_children + k > x->c->cap_children) return NXO_CAPACITY;
    x->c->n_children += k;
    return NXO_OK;
}

/* ArcStr (pack.rs:457-469) / PBytes (pbuf.rs:139-147) payload: varint len, TooBig if len >
 * remaining, UTF-8 checked for strings. */
static int dstr(Buf* b, int utf8, uint64_t* off, uint64_t* len) {
    uint64_t n;
    int e = dvar(b, &n);
    if (e) return e;
    if (n > rem(b)) return NXO_TOO_BIG;
    if (utf8 && !nxo_utf8_valid(b->w + b->pos, n)) return NXO_INVALID_FORMAT;
    *off = b->pos;
    *len = n;
    b->pos += n;
    return NXO_OK;
}

static int dvalue(Ctx* x, Buf* b, int is_row, uint64_t slot, int depth) {
    if (depth > NXO_MAX_DEPTH) return NXO_DEPTH;
    uint64_t t, v, v2, off, len, base;
    int e;
    if ((e = dfix(b, 1, &t))) return e; /* <u8 as Pack>::decode */
    switch (t) {
    case 0: /* U32 */
        if ((e = dfix(b, 4, &v))) return e;
        put_slot(x, is_row, slot, 0, v, 0);
        return NXO_OK;
    case 1: /* V32: decode_varint as u32 (truncating) */
        if ((e = dvar(b, &v))) return e;
        put_slot(x, is_row, slot, 1, (uint32_t)v, 0);
        return NXO_OK;
    case 2: /* I32 */
        if ((e = dfix(b, 4, &v))) return e;
        put_slot(x, is_row, slot, 2, (uint64_t)(int64_t)(int32_t)(uint32_t)v, 0);
        return NXO_OK;
    case 3: { /* Z32: i32_uzz(decode_varint as u32) pack.rs:492-494 */
        if ((e = dvar(b, &v))) return e;
        uint32_t n = (uint32_t)v;
        int32_t r = (int32_t)(n >> 1) ^ (int32_t)(0u - (n & 1u));
        put_slot(x, is_row, slot, 3, (uint64_t)(int64_t)r, 0);
        return NXO_OK;
    }
    case 4: /* U64 */
    case 6: /* I64 */
    case 9: /* F64 */
        if ((e = dfix(b, 8, &v))) return e;
        put_slot(x, is_row, slot, (uint8_t)t, v, 0);
        return NXO_OK;
    case 5: /* V64 */
        if ((e = dvar(b, &v))) return e;
        put_slot(x, is_row, slot, 5, v, 0);
        return NXO_OK;
    case 7: { /* Z64: i64_uzz pack.rs:500-502 */
        if ((e = dvar(b, &v))) return e;
        uint64_t r = (v >> 1) ^ (0ull - (v & 1ull));
        put_slot(x, is_row, slot, 7, r, 0);
        return NXO_OK;
    }
    case 8: /* F32 */
        if ((e = dfix(b, 4, &v))) return e;
        put_slot(x, is_row, slot, 8, v, 0);
        return NXO_OK;
    case 10: /* DateTime pack.rs:1567-1575 */
        if ((e = dfix(b, 8, &v))) return e;
        if ((e = dfix(b, 4, &v2))) return e;
        if (!nxo_datetime_valid((int64_t)v, (uint32_t)v2)) return NXO_INVALID_FORMAT;
        put_slot(x, is_row, slot, 10, v, (uint32_t)v2);
        return NXO_OK;
    case 11: { /* Duration pack.rs:1591-1595: Duration::new normalises ns >= 1e9 */
        if ((e = dfix(b, 8, &v))) return e;
        if ((e = dfix(b, 4, &v2))) return e;
        uint64_t secs = v;
        uint32_t ns = (uint32_t)v2;
        if (ns >= 1000000000u) {
            uint64_t add = ns / 1000000000u;
            if (secs + add < secs) return NXO_INVALID_FORMAT; /* reference panics: deviation */
            secs += add;
            ns %= 1000000000u;
        }
        put_slot(x, is_row, slot, 11, secs, ns);
        return NXO_OK;
    }
    case 12: /* String */
    case 18: /* Error(String) lib.rs:485-489 */
        if ((e = dstr(b, 1, &off, &len))) return e;
        put_slot(x, is_row, slot, (uint8_t)t, off, (uint32_t)len);
        return NXO_OK;
    case 13: /* Bytes */
        if ((e = dstr(b, 0, &off, &len))) return e;
        put_slot(x, is_row, slot, 13, off, (uint32_t)len);
        return NXO_OK;
    case 14:
        put_slot(x, is_row, slot, 14, 1, 0);
        return NXO_OK;
    case 15:
        put_slot(x, is_row, slot, 15, 0, 0);
        return NXO_OK;
    case 16:
    case 17: /* 17 (old Ok) decodes to Null, lib.rs:489 */
        put_slot(x, is_row, slot, 16, 0, 0);
        return NXO_OK;
    case 19: { /* Array: array.rs:595-612 */
        if ((e = dvar(b, &v))) return e;
        uint64_t sz = (v > UINT64_MAX / 16) ? UINT64_MAX : v * 16; /* saturating_mul */
        if (sz > MAX_VEC || sz > (rem(b) << 8)) return NXO_TOO_BIG;
        if ((e = alloc_children(x, v, &base))) return e;
        put_slot(x, is_row, slot, 19, base, (uint32_t)v);
        for (uint64_t i = 0; i < v; i++)
            if ((e = dvalue(x, b, 0, base + i, depth + 1))) return e;
        return NXO_OK;
    }
    case 20: /* Decimal pack.rs:614-622: 16 raw bytes */
        if (rem(b) < 16) return NXO_BUFFER_SHORT;
        put_slot(x, is_row, slot, 20, b->pos, 16);
        b->pos += 16;
        return NXO_OK;
    case 21: { /* Map pack.rs:1225-1239 (check_sz with K=V=Value, 32 B per entry) */
        if ((e = dvar(b, &v))) return e;
        uint64_t sz = (v > UINT64_MAX / 32) ? UINT64_MAX : v * 32;
        if (sz > MAX_VEC || sz > (rem(b) << 8)) return NXO_TOO_BIG;
        if ((e = alloc_children(x, 2 * v, &base))) return e;
        put_slot(x, is_row, slot, 21, base, (uint32_t)v);
        for (uint64_t i = 0; i < 2 * v; i++)
            if ((e = dvalue(x, b, 0, base + i, depth + 1))) return e;
        return NXO_OK;
    }
    case 22: /* Error(Value) lib.rs:497. Error(String) is the same Value as tag 18 (lib.rs:437-446
              * re-encodes it as 18), so an inner String is normalised into an 18 slot. */
        if (rem(b) >= 1 && b->w[b->pos] == 12) {
            b->pos += 1;
            if ((e = dstr(b, 1, &off, &len))) return e;
            put_slot(x, is_row, slot, 18, off, (uint32_t)len);
            return NXO_OK;
        }
        if ((e = alloc_children(x, 1, &base))) return e;
        put_slot(x, is_row, slot, 22, base, 1);
        return dvalue(x, b, 0, base, depth + 1);
    case 23: /* U8 */
        if ((e = dfix(b, 1, &v))) return e;
        put_slot(x, is_row, slot, 23, v, 0);
        return NXO_OK;
    case 24: /* I8 */
        if ((e = dfix(b, 1, &v))) return e;
        put_slot(x, is_row, slot, 24, (uint64_t)(int64_t)(int8_t)(uint8_t)v, 0);
        return NXO_OK;
    case 25: /* U16 */
        if ((e = dfix(b, 2, &v))) return e;
        put_slot(x, is_row, slot, 25, v, 0);
        return NXO_OK;
    case 26: /* I16 */
        if ((e = dfix(b, 2, &v))) return e;
        put_slot(x, is_row, slot, 26, (uint64_t)(int64_t)(int16_t)(uint16_t)v, 0);
        return NXO_OK;
    case 27: { /* Abstract abstract_type.rs:280-298: len-wrapped {uuid u128, payload}; with no
                * registered decoder the payload is kept whole (UnknownAbstractType, :116-121) */
        if ((e = dvar(b, &v))) return e;
        if (v < 1) return NXO_BUFFER_SHORT;
        uint64_t take = v - nxo_varint_len(v);
        uint64_t lim = take < rem(b) ? b->pos + take : b->lim;
        if (lim - b->pos < 16) return NXO_BUFFER_SHORT; /* Uuid = u128 */
        put_slot(x, is_row, slot, 27, b->pos, (uint32_t)(lim - b->pos));
        b->pos = lim;
        return NXO_OK;
    }
    default:
        return NXO_UNKNOWN_TAG;
    }
}

/* From::decode: len_wrapped_decode (pack.rs:537-555) around the derived enum decode
 * (netidx-derive/src/lib.rs:482-601) of netidx-netproto/src/publisher.rs:73-96. */
static int dfrom(Ctx* x, Buf* b, uint64_t msg_start) {
    uint64_t L, variant, v, off, len;
    int e;
    if ((e = dvar(b, &L))) return e;
    if (L < 1) return NXO_BUFFER_SHORT;
    uint64_t take = L - nxo_varint_len(L);
    Buf in = {b->w, b->pos, take < rem(b) ? b->pos + take : b->lim};
    NxoCols* c = x->c;
    e = dfix(&in, 1, &variant);
    if (!e) {
        switch (variant) {
        case 0: /* NoSuchValue(Path) */
        case 1: /* Denied(Path) */
            e = dstr(&in, 1, &off, &len);
            break;
        case 2: /* Unsubscribed(Id) */
            e = dvar(&in, &v);
            break;
        case 3: { /* Subscribed(Path, Id, Value) */
            Ctx vx = {c, 0};
            if (!(e = dstr(&in, 1, &off, &len)))
                if (!(e = dvar(&in, &v))) e = dvalue(&vx, &in, 0, 0, 0);
            break;
        }
        case 4: { /* Update(Id, Value) */
            if ((e = dvar(&in, &v))) break;
            if (c->n_rows >= c->cap_rows) {
                e = NXO_CAPACITY;
                break;
            }
            uint64_t r = c->n_rows;
            e = dvalue(x, &in, 1, r, 0);
            if (!e) {
                c->id[r] = v;
                c->n_rows++;
            }
            break;
        }
        case 5: /* Heartbeat */
            break;
        case 6: { /* WriteResult(Id, Value, #[pack(default)] WriteId): derive lib.rs:392-401 */
            Ctx vx = {c, 0};
            if ((e = dvar(&in, &v))) break;
            if ((e = dvalue(&vx, &in, 0, 0, 0))) break;
            e = dvar(&in, &v);
            if (e == NXO_BUFFER_SHORT) e = NXO_OK;
            break;
        }
        default:
            e = NXO_UNKNOWN_TAG;
        }
    }
    b->pos = in.lim; /* limited.advance(limited.remaining()) */
    if (e) return e;
    if (variant != 4) {
        if (c->n_ctl >= c->cap_ctl) return NXO_CAPACITY;
        uint64_t k = c->n_ctl++;
        c->ctl_row[k] = c->n_rows;
        c->ctl_off[k] = msg_start;
        c->ctl_len[k] = (uint32_t)(b->pos - msg_start);
        c->ctl_variant[k] = (uint8_t)variant;
        if (variant == 5) c->n_heartbeat++;
    }
    return NXO_OK;
}

int nxo_decode_frame(const uint8_t* w, uint64_t len, NxoCols* c) {
    c->n_rows = c->n_children = c->n_ctl = c->n_heartbeat = 0;
    c->err_kind = 0;
    c->err_offset = 0;
    Ctx x = {c, 1};
    Buf b = {w, 0, len};
    while (b.pos < b.lim) { /* while self.buf.has_remaining() */
        uint64_t start = b.pos;
        int e = dfrom(&x, &b, start);
        if (e) {
            c->err_kind = e;
            c->err_offset = start;
            return e;
        }
    }
    return NXO_OK;
}

/* ---------------------------------------------------------------------------------------------
 * Archive batches: <GPooled<Vec<BatchItem>> as Pack> (pack.rs:167-185 -> Vec<T>, pack.rs:934-973)
 * with BatchItem(Id, Event) (netidx-archive/src/logfile/mod.rs:150-205) and Event::decode
 * (netidx/src/subscriber/mod.rs:154-177): varint count, check_sz!(count, remaining, BatchItem),
 * then per item varint(id) as u32 and an Event that is NOT length-wrapped -- byte 0x40 is
 * Unsubscribed, anything else a bare Value. Boundaries follow from the values' tags alone.
 * size_of::<BatchItem>() is taken as 24 (Id u32 + Event 16 with its niche in Value's repr(u32)
 * tag, align 8): parity unpinned, it only sets the TooBig guard. Deviation: Event::decode on an
 * empty buffer indexes chunk()[0] and panics in the reference; here it is BufferShort.
 * Rows: id = the u32 Id, the value (Unsubscribed: tag NXO_TAG_UNSUBSCRIBED, 0, 0). Returns the
 * bytes consumed (trailing bytes after the count items are not read), or -kind with err_offset =
 * the failing item's start (0 for the count and the size guard).
 * ------------------------------------------------------------------------------------------- */
#define BATCH_ITEM_SIZE 24

int64_t nxo_decode_archive(const uint8_t* w, uint64_t len, NxoCols* c) {
    c->n_rows = c->n_children = c->n_ctl = c->n_heartbeat = 0;
    c->err_kind = 0;
    c->err_offset = 0;
    Ctx x = {c, 1};
    Buf b = {w, 0, len};
    uint64_t count, start = 0, id;
    int e;
    if ((e = dvar(&b, &count))) goto fail;
    {
        const uint64_t sz = count > UINT64_MAX / BATCH_ITEM_SIZE ? UINT64_MAX : count * BATCH_ITEM_SIZE;
        if (sz > MAX_VEC || sz > (rem(&b) << 8)) {
            e = NXO_TOO_BIG;
            goto fail;
        }
    }
    for (uint64_t i = 0; i < count; i++) {
        start = b.pos;
        if (c->n_rows >= c->cap_rows) {
            e = NXO_CAPACITY;
            goto fail;
        }
        const uint64_t r = c->n_rows;
        if ((e = dvar(&b, &id))) goto fail;
        if (rem(&b) == 0) {
            e = NXO_BUFFER_SHORT;
            goto fail;
        }
        if (w[b.pos] == NXO_TAG_UNSUBSCRIBED) {
            b.pos++;
            put_slot(&x, 1, r, NXO_TAG_UNSUBSCRIBED, 0, 0);
        } else if ((e = dvalue(&x, &b, 1, r, 0))) {
            goto fail;
        }
        c->id[r] = (uint32_t)id;
        c->n_rows++;
    }
    return (int64_t)b.pos;
fail:
    c->err_kind = e;
    c->err_offset = start;
    return -(int64_t)e;
}

/* ---------------------------------------------------------------------------------------------
 * Encode (lib.rs:361-468, array.rs:583-593, pack.rs:1212-1223, abstract_type.rs:272-278)
 * ------------------------------------------------------------------------------------------- */
static uint32_t zz32(int32_t n) { return ((uint32_t)n << 1) ^ (uint32_t)(n >> 31); }
static uint64_t zz64(int64_t n) { return ((uint64_t)n << 1) ^ (uint64_t)(n >> 63); }

static int64_t vlen(const NxoCols* c, int is_row, uint64_t slot, int depth) {
    if (depth > NXO_MAX_DEPTH) return -NXO_DEPTH;
    uint8_t t = is_row ? c->tag[slot] : c->ctag[slot];
    uint64_t f = is_row ? c->fixed[slot] : c->cfixed[slot];
    uint32_t a = is_row ? c->aux[slot] : c->caux[slot];
    switch (t) {
    case 0: case 2: case 8: return 5;
    case 1: return 1 + nxo_varint_len((uint32_t)f);
    case 3: return 1 + nxo_varint_len(zz32((int32_t)(uint32_t)f));
    case 4: case 6: case 9: return 9;
    case 5: return 1 + nxo_varint_len(f);
    case 7: return 1 + nxo_varint_len(zz64((int64_t)f));
    case 10: case 11: return 13;
    case 12: case 13: case 18: return 1 + nxo_varint_len(a) + (int64_t)a;
    case 14: case 15: case 16: return 1;
    case 19: case 21: {
        uint64_t k = (t == 19) ? a : 2ull * a;
        if ((uint64_t)a * (t == 19 ? 16 : 32) > MAX_VEC) return -NXO_TOO_BIG;
        int64_t s = 1 + nxo_varint_len(a);
        for (uint64_t i = 0; i < k; i++) {
            int64_t l = vlen(c, 0, f + i, depth + 1);
            if (l < 0) return l;
            s += l;
        }
        return s;
    }
    case 20: return 17;
    case 22: {
        int64_t l = vlen(c, 0, f, depth + 1);
        return l < 0 ? l : 1 + l;
    }
    case 23: case 24: return 2;
    case 25: case 26: return 3;
    case 27: return 1 + (int64_t)lwlen(a);
    default: return -NXO_UNKNOWN_TAG;
    }
}

static inline void putbe(uint8_t** o, uint64_t v, int n) {
    for (int i = n - 1; i >= 0; i--) *(*o)++ = (uint8_t)(v >> (8 * i));
}
static inline void putvar(uint8_t** o, uint64_t v) { *o += nxo_encode_varint(v, *o); }

static void venc(const NxoCols* c, const uint8_t* heap, int is_row, uint64_t slot, uint8_t** o) {
    uint8_t t = is_row ? c->tag[slot] : c->ctag[slot];
    uint64_t f = is_row ? c->fixed[slot] : c->cfixed[slot];
    uint32_t a = is_row ? c->aux[slot] : c->caux[slot];
    *(*o)++ = t;
    switch (t) {
    case 0: case 2: case 8: putbe(o, f, 4); break;
    case 1: putvar(o, (uint32_t)f); break;
    case 3: putvar(o, zz32((int32_t)(uint32_t)f)); break;
    case 4: case 6: case 9: putbe(o, f, 8); break;
    case 5: putvar(o, f); break;
    case 7: putvar(o, zz64((int64_t)f)); break;
    case 10: case 11: putbe(o, f, 8); putbe(o, a, 4); break;
    case 12: case 13: case 18:
        putvar(o, a);
        memcpy(*o, heap + f, a);
        *o += a;
        break;
    case 19: case 21: {
        uint64_t k = (t == 19) ? a : 2ull * a;
        putvar(o, a);
        for (uint64_t i = 0; i < k; i++) venc(c, heap, 0, f + i, o);
        break;
    }
    case 20: memcpy(*o, heap + f, 16); *o += 16; break;
    case 22: venc(c, heap, 0, f, o); break;
    case 23: case 24: putbe(o, f, 1); break;
    case 25: case 26: putbe(o, f, 2); break;
    case 27:
        putvar(o, lwlen(a));
        memcpy(*o, heap + f, a);
        *o += a;
        break;
    default: break;
    }
}

static int64_t row_len(const NxoCols* c, uint64_t r) {
    int64_t l = vlen(c, 1, r, 0);
    if (l < 0) return l;
    return (int64_t)lwlen(1 + nxo_varint_len(c->id[r]) + (uint64_t)l);
}

static int64_t enc_all(const NxoCols* c, const uint8_t* heap, uint8_t* out, uint64_t cap) {
    uint64_t total = 0, k = 0;
    uint8_t* o = out;
    for (uint64_t r = 0; r <= c->n_rows; r++) {
        while (k < c->n_ctl && c->ctl_row[k] <= r) {
            uint64_t l = c->ctl_len[k];
            if (out) {
                if (total + l > cap) return -NXO_CAPACITY;
                memcpy(o, heap + c->ctl_off[k], l);
                o += l;
            }
            total += l;
            k++;
        }
        if (r == c->n_rows) break;
        int64_t l = row_len(c, r);
        if (l < 0) return l;
        if (out) {
            if (total + (uint64_t)l > cap) return -NXO_CAPACITY;
            uint64_t inner = (uint64_t)l - nxo_varint_len((uint64_t)l);
            putvar(&o, (uint64_t)l); /* len_wrapped_encode writes encoded_len (pack.rs:533) */
            *o++ = 4;                /* From::Update is variant 4 */
            putvar(&o, c->id[r]);
            venc(c, heap, 1, r, &o);
            (void)inner;
        }
        total += (uint64_t)l;
    }
    return (int64_t)total;
}

int64_t nxo_encoded_len(const NxoCols* c, const uint8_t* heap) { return enc_all(c, heap, 0, 0); }

int64_t nxo_encode(const NxoCols* c, const uint8_t* heap, uint8_t* out, uint64_t cap) {
    return enc_all(c, heap, out, cap);
}

int64_t nxo_encode_f64(const uint64_t* id, const uint64_t* val, uint64_t n, uint8_t* out,
                       uint64_t cap) {
    uint8_t* o = out;
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t L = lwlen(1 + nxo_varint_len(id[i]) + 9);
        if (total + L > cap) return -NXO_CAPACITY;
        putvar(&o, L);
        *o++ = 4;
        putvar(&o, id[i]);
        *o++ = 9;
        putbe(&o, val[i], 8);
        total += L;
    }
    return (int64_t)total;
}

/* ---- subscriber update dispatch (connection.rs:546-567) ------------------------------------ */
int64_t nxo_dispatch(const uint64_t* id, uint64_t n_rows, uint64_t n_ids,
                     const uint32_t* slot_of_id, uint64_t n_slots, const uint64_t* slot_sub_id,
                     const uint32_t* slot_stream_off, const uint32_t* stream_chan,
                     const uint8_t* slot_has_last, uint32_t n_chans, uint64_t* chan_off,
                     uint64_t* ent_sub, uint64_t* ent_row, uint64_t cap, uint64_t* last_row,
                     uint64_t* n_unmatched) {
    /* pass 1: per-channel batch lengths (the by_chan vectors' final sizes) */
    for (uint32_t c = 0; c <= n_chans; c++) chan_off[c] = 0;
    for (uint64_t s = 0; s < n_slots; s++) last_row[s] = 0;
    uint64_t unmatched = 0;
    for (uint64_t i = 0; i < n_rows; i++) {
        const uint32_t s = id[i] < n_ids ? slot_of_id[id[i]] : NXO_NO_SLOT;
        if (s == NXO_NO_SLOT) { /* self.subscriptions.get(&i) == None */
            unmatched++;
            continue;
        }
        for (uint32_t k = slot_stream_off[s]; k < slot_stream_off[s + 1]; k++)
            chan_off[stream_chan[k] + 1]++;
    }
    for (uint32_t c = 0; c < n_chans; c++) chan_off[c + 1] += chan_off[c];
    const uint64_t total = chan_off[n_chans];
    if (n_unmatched) *n_unmatched = unmatched;
    if (total > cap) return -NXO_CAPACITY;
    /* pass 2: the pushes, in batch order, each channel's batch in push order */
    uint64_t* cur = (uint64_t*)malloc((n_chans ? n_chans : 1) * sizeof(uint64_t));
    if (!cur) return -NXO_CAPACITY;
    for (uint32_t c = 0; c < n_chans; c++) cur[c] = chan_off[c];
    for (uint64_t i = 0; i < n_rows; i++) {
        const uint32_t s = id[i] < n_ids ? slot_of_id[id[i]] : NXO_NO_SLOT;
        if (s == NXO_NO_SLOT) continue;
        for (uint32_t k = slot_stream_off[s]; k < slot_stream_off[s + 1]; k++) {
            const uint64_t e = cur[stream_chan[k]]++;
            ent_sub[e] = slot_sub_id[s]; /* (sub.sub_id, Event::Update(m.clone())) */
            ent_row[e] = i;
        }
        if (slot_has_last[s]) last_row[s] = i + 1; /* *last.lock() = Event::Update(m) */
    }
    free(cur);
    return (int64_t)total;
}

/* ---- publisher commit (publisher/mod.rs:776-845) ------------------------------------------- */
/* Value::eq (netidx-value/src/op.rs:133-172) over the columnar contract: a value is a slot
 * (tag, fixed, aux) of a column set, its text/Decimal/Abstract bytes at heap + fixed, its
 * children (Array elements, Map key/value pairs, Error(Value)'s inner value) at child slots
 * fixed .. fixed + count. */
typedef struct {
    const uint8_t* tag; /* NULL: every top-level slot is F64 (tag 9) */
    const uint64_t* fixed;
    const uint32_t* aux; /* NULL: 0 */
    const uint8_t* ctag;
    const uint64_t* cfixed;
    const uint32_t* caux;
    const uint8_t* heap;
} NxoVSrc;

static uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* rust_decimal (Decimal::serialize: flags, lo, mid, hi as little-endian u32; scale = flags bits
 * 16..23, sign = bit 31) compared numerically, as Decimal's PartialEq (via cmp) does: equal
 * values at different scales are equal, and every zero is equal. Exact for any scale byte: a
 * mantissa below 2^96 < 10^29 cannot equal a non-zero one scaled by 10^29 or more. */
int nxo_decimal_eq(const uint8_t* a, const uint8_t* b) {
    const uint32_t fa = le32(a), fb = le32(b);
    uint32_t ma[3] = {le32(a + 4), le32(a + 8), le32(a + 12)};
    uint32_t mb[3] = {le32(b + 4), le32(b + 8), le32(b + 12)};
    const int za = !(ma[0] | ma[1] | ma[2]), zb = !(mb[0] | mb[1] | mb[2]);
    if (za || zb) return za && zb;
    if ((fa >> 31) != (fb >> 31)) return 0;
    uint32_t sa = (fa >> 16) & 0xff, sb = (fb >> 16) & 0xff;
    if (sa > sb) { /* scale the smaller-scale side up: m_small * 10^d == m_large */
        uint32_t t[3] = {ma[0], ma[1], ma[2]};
        memcpy(ma, mb, sizeof t);
        memcpy(mb, t, sizeof t);
        const uint32_t u = sa;
        sa = sb;
        sb = u;
    }
    const uint32_t d = sb - sa;
    if (d > 28) return 0;
    uint64_t w[6] = {ma[0], ma[1], ma[2], 0, 0, 0}; /* 192 bits in 32-bit limbs */
    for (uint32_t k = 0; k < d; k++) {
        uint64_t carry = 0;
        for (int i = 0; i < 6; i++) {
            const uint64_t x = w[i] * 10 + carry;
            w[i] = x & 0xffffffffu;
            carry = x >> 32;
        }
    }
    return w[0] == mb[0] && w[1] == mb[1] && w[2] == mb[2] && !(w[3] | w[4] | w[5]);
}

static int nxo_f_eq(uint8_t t, uint64_t fa, uint64_t fb) {
    if (t == 8) { /* F32: NaN == NaN, otherwise IEEE == (+0 == -0) */
        float l, r;
        uint32_t lb = (uint32_t)fa, rb = (uint32_t)fb;
        memcpy(&l, &lb, 4);
        memcpy(&r, &rb, 4);
        return (l != l && r != r) || l == r;
    }
    double l, r;
    memcpy(&l, &fa, 8);
    memcpy(&r, &fb, 8);
    return (l != l && r != r) || l == r;
}

/* one slot of a source: top level (child = 0) or a child slot */
static void nxo_slot(const NxoVSrc* s, int child, uint64_t i, uint8_t* t, uint64_t* f,
                     uint32_t* a) {
    if (child) {
        *t = s->ctag[i];
        *f = s->cfixed[i];
        *a = s->caux[i];
    } else {
        *t = s->tag ? s->tag[i] : 9;
        *f = s->fixed[i];
        *a = s->aux ? s->aux[i] : 0;
    }
}

/* Error(String) has two spellings in the columns: tag 18, or tag 22 over a String child */
static void nxo_norm_error(const NxoVSrc* s, uint8_t* t, uint64_t* f, uint32_t* a) {
    if (*t == 22 && s->ctag && s->ctag[*f] == 12) {
        const uint64_t c = *f;
        *t = 18;
        *f = s->cfixed[c];
        *a = s->caux[c];
    }
}

/* 1 equal, 0 different, -1 nested deeper than NXG_MAX_DEPTH (32) or a container without child
 * columns */
static int nxo_val_eq_at(const NxoVSrc* A, int ca, uint64_t ia, const NxoVSrc* B, int cb,
                         uint64_t ib, int depth) {
    uint8_t ta, tb;
    uint64_t fa, fb;
    uint32_t aa, ab;
    nxo_slot(A, ca, ia, &ta, &fa, &aa);
    nxo_slot(B, cb, ib, &tb, &fb, &ab);
    if (depth > 32) return -1;
    if (ta == 22) nxo_norm_error(A, &ta, &fa, &aa);
    if (tb == 22) nxo_norm_error(B, &tb, &fb, &ab);
    if (ta == 17) ta = 16; /* Null */
    if (tb == 17) tb = 16;
    if (ta != tb) return 0; /* different Typ, or Bool(true) vs Bool(false) */
    switch (ta) {
    case 8: case 9: return nxo_f_eq(ta, fa, fb);
    case 10: case 11: return fa == fb && aa == ab; /* DateTime / Duration */
    case 12: case 13: case 18: case 27: /* String / Bytes / Error(String) / Abstract bytes */
        return aa == ab && memcmp(A->heap + fa, B->heap + fb, aa) == 0;
    case 20: return nxo_decimal_eq(A->heap + fa, B->heap + fb);
    case 14: case 15: case 16: return 1;
    case 19: case 21: case 22: { /* Array, Map (entries in order), Error(Value) */
        const uint64_t n = ta == 19 ? aa : ta == 21 ? 2ull * aa : 1;
        if (ta != 22 && aa != ab) return 0;
        if (n && (!A->ctag || !B->ctag)) return -1; /* no child columns */
        for (uint64_t k = 0; k < n; k++) {
            const int e = nxo_val_eq_at(A, 1, fa + k, B, 1, fb + k, depth + 1);
            if (e <= 0) return e;
        }
        return 1;
    }
    default: return fa == fb; /* integers (sign-extended), V32/Z32 as u32 */
    }
}

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
                            uint64_t* n_unmatched) {
    const NxoVSrc BS = {tag, fixed, aux, ctag, cfixed, caux, heap};
    const NxoVSrc CS = {cur_tag, cur_fixed, cur_aux, cur_ctag, cur_cfixed, cur_caux, cur_heap};
    /* current value of each slot: the table's, or the batch row that replaced it */
    uint64_t* cur = (uint64_t*)malloc((n_slots ? n_slots : 1) * sizeof(uint64_t));
    uint8_t* emit = (uint8_t*)malloc(n_rows ? n_rows : 1);
    if (!cur || !emit) return -NXO_CAPACITY;
    for (uint64_t s = 0; s < n_slots; s++) cur[s] = 0; /* 0: the table's value */
    for (uint32_t c = 0; c <= n_clients; c++) client_off[c] = 0;
    uint64_t unmatched = 0;
    int64_t rc = 0;
    /* pass 1: which messages are pushed, and the per-client batch lengths */
    for (uint64_t i = 0; i < n_rows && rc == 0; i++) {
        emit[i] = 0;
        if (kind[i] == NXO_PUB_UPDATE_CLIENT) { /* batch.entry(cl).push(Update(id, v)) */
            if (to_client[i] < n_clients) {
                emit[i] = 1;
                client_off[to_client[i] + 1]++;
            }
            continue;
        }
        const uint32_t s = id[i] < n_ids ? slot_of_id[id[i]] : NXO_NO_SLOT;
        if (s == NXO_NO_SLOT) { /* pb.by_id.get_mut(&id) == None */
            unmatched++;
            continue;
        }
        if (kind[i] == NXO_PUB_UPDATE_CHANGED) { /* if pbl.current != v */
            int eq;
            if (cur[s]) eq = nxo_val_eq_at(&BS, 0, cur[s] - 1, &BS, 0, i, 0);
            else eq = nxo_val_eq_at(&CS, 0, s, &BS, 0, i, 0);
            if (eq < 0) {
                rc = -NXO_UNSUPPORTED;
                break;
            }
            if (eq) continue;
        }
        emit[i] = 2;
        for (uint32_t k = slot_client_off[s]; k < slot_client_off[s + 1]; k++)
            if (client[k] < n_clients) client_off[client[k] + 1]++;
        cur[s] = i + 1; /* pbl.current = v */
    }
    if (rc == 0) {
        for (uint32_t c = 0; c < n_clients; c++) client_off[c + 1] += client_off[c];
        if (client_off[n_clients] > cap) rc = -NXO_CAPACITY;
    }
    if (rc == 0) {
        uint64_t* pos = (uint64_t*)malloc((n_clients ? n_clients : 1) * sizeof(uint64_t));
        for (uint32_t c = 0; c < n_clients; c++) pos[c] = client_off[c];
        for (uint64_t i = 0; i < n_rows; i++) {
            if (emit[i] == 1) {
                const uint64_t e = pos[to_client[i]]++;
                ent_id[e] = id[i];
                ent_row[e] = i;
            } else if (emit[i] == 2) {
                const uint32_t s = slot_of_id[id[i]];
                for (uint32_t k = slot_client_off[s]; k < slot_client_off[s + 1]; k++) {
                    if (client[k] >= n_clients) continue;
                    const uint64_t e = pos[client[k]]++;
                    ent_id[e] = id[i];
                    ent_row[e] = i;
                }
            }
        }
        free(pos);
        for (uint64_t s = 0; s < n_slots; s++) cur_row[s] = cur[s];
        rc = (int64_t)client_off[n_clients];
    }
    if (n_unmatched) *n_unmatched = unmatched;
    free(cur);
    free(emit);
    return rc;
}

int64_t nxo_publish_commit(const uint64_t* id, const uint8_t* tag, const uint64_t* fixed,
                           const uint32_t* aux, const uint8_t* heap, const uint8_t* kind,
                           const uint32_t* to_client, uint64_t n_rows, uint64_t n_ids,
                           const uint32_t* slot_of_id, uint64_t n_slots,
                           const uint32_t* slot_client_off, const uint32_t* client,
                           uint32_t n_clients, const uint8_t* cur_tag, const uint64_t* cur_fixed,
                           const uint32_t* cur_aux, const uint8_t* cur_heap, uint64_t* client_off,
                           uint64_t* ent_id, uint64_t* ent_row, uint64_t cap, uint64_t* cur_row,
                           uint64_t* n_unmatched) {
    return nxo_publish_commit2(id, tag, fixed, aux, NULL, NULL, NULL, heap, kind, to_client,
                               n_rows, n_ids, slot_of_id, n_slots, slot_client_off, client,
                               n_clients, cur_tag, cur_fixed, cur_aux, NULL, NULL, NULL, cur_heap,
                               client_off, ent_id, ent_row, cap, cur_row, n_unmatched);
}

/* UpdateBatch::commit's unsubscribes (publisher/mod.rs:820-832): each (client, id), in queue
 * order, onto that client's Update.unsubscribes. client_off[n_clients + 1] (CSR), ent_id[n].
 * Clients >= n_clients are dropped (pb.clients.get(&cl) is None). Returns the entries kept. */
int64_t nxo_publish_unsubscribes(const uint64_t* id, const uint32_t* cl, uint64_t n,
                                 uint32_t n_clients, uint64_t* client_off, uint64_t* ent_id) {
    for (uint32_t c = 0; c <= n_clients; c++) client_off[c] = 0;
    for (uint64_t i = 0; i < n; i++)
        if (cl[i] < n_clients) client_off[cl[i] + 1]++;
    for (uint32_t c = 0; c < n_clients; c++) client_off[c + 1] += client_off[c];
    uint64_t* pos = (uint64_t*)malloc((n_clients ? n_clients : 1) * sizeof(uint64_t));
    if (!pos) return -NXO_CAPACITY;
    for (uint32_t c = 0; c < n_clients; c++) pos[c] = client_off[c];
    for (uint64_t i = 0; i < n; i++)
        if (cl[i] < n_clients) ent_id[pos[cl[i]]++] = id[i];
    free(pos);
    return (int64_t)client_off[n_clients];
}

/* <Vec<BatchItem> as Pack>::encode (pack.rs:941-952): varint(count), then per row varint(id)
 * and the Event (tag NXO_TAG_UNSUBSCRIBED: the byte 0x40; else the bare Value). out == NULL:
 * the length only. TooBig if count * size_of::<BatchItem>() > MAX_VEC. */
int64_t nxo_encode_archive(const NxoCols* c, const uint8_t* heap, uint8_t* out, uint64_t cap) {
    if (c->n_rows > MAX_VEC / BATCH_ITEM_SIZE) return -NXO_TOO_BIG;
    uint64_t total = nxo_varint_len(c->n_rows);
    for (uint64_t r = 0; r < c->n_rows; r++) {
        int64_t l = 1;
        if (c->tag[r] != NXO_TAG_UNSUBSCRIBED) {
            l = vlen(c, 1, r, 0);
            if (l < 0) return l;
        }
        total += nxo_varint_len((uint32_t)c->id[r]) + (uint64_t)l;
    }
    if (!out) return (int64_t)total;
    if (total > cap) return -NXO_CAPACITY;
    uint8_t* o = out;
    putvar(&o, c->n_rows);
    for (uint64_t r = 0; r < c->n_rows; r++) {
        putvar(&o, (uint32_t)c->id[r]);
        if (c->tag[r] == NXO_TAG_UNSUBSCRIBED) *o++ = NXO_TAG_UNSUBSCRIBED;
        else venc(c, heap, 1, r, &o);
    }
    return (int64_t)total;
}
