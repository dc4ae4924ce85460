// nxg_session.cpp -- the publisher <-> subscriber TCP connection (BASELINE configs[0]) in C++:
// the handshake, the subscription, and the data path's receive / send loops around the codec.
//
// Handshake (raw messages: u32 big-endian length + the packed value, channel.rs:63-105):
//   subscriber: write u64 3, read u64 3, write Hello::Anonymous, read Hello::Anonymous
//               (subscriber/connection.rs:120-140)
//   publisher:  write u64 3, read u64 3, read Hello, answer Hello::Anonymous
//               (publisher/server.rs:367-381)
// Then the connection is a Channel: frames of u32 length (bit 31: encrypted, refused here) whose
// payloads are len-wrapped messages (channel.rs:107-126, 379-443). The subscriber sends
// To::Subscribe { path, resolver, timestamp, permissions, token } (netproto publisher.rs:51-70);
// the publisher answers From::Subscribed(path, id, current) (publisher/server.rs:60-137) and then
// streams From::Update(id, v) batches and Heartbeats.
//
// The data path: nxg_session_recv_decode reads the socket straight into a pinned reassembly
// buffer (one recv per up to 4 MiB), and hands each complete frame payload to nxg_decode_updates,
// which copies it to the device and decodes it there; nxg_session_publish encodes device columns
// with nxg_encode_frames (MAX_BATCH cuts), copies the payload into pinned memory and writes each
// frame behind its header. Control messages (the handshake, Subscribe, Subscribed, Heartbeat)
// are built and parsed here on the host: they are a few bytes each.
#include <algorithm>
#include <arpa/inet.h>
#include <hip/hip_runtime.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/nxg_codec.h"
#include "nxg_wire.h"

namespace {
using namespace nxgwire;

void serr(NetidxError* err, const char* fmt, ...) {
    if (!err) return;
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    free(err->msg);
    err->msg = strdup(buf);
}

constexpr uint32_t kLenMask = 0x7FFFFFFFu;   // channel.rs:35 (bit 31: encrypted)
constexpr uint64_t kMaxBatch = 0x3FFFFFFF;   // channel.rs:34
constexpr uint64_t kProtocolVersion = 3;     // subscriber/connection.rs:128
constexpr size_t kRecvChunk = 4u << 20;      // bytes per recv

// a scalar Value (netidx-value lib.rs:361-468): fixed-width and varint tags, text from `text`
bool put_value(Out& o, uint8_t tag, uint64_t fixed, uint32_t aux, const uint8_t* text,
               NetidxError* err) {
    o.u8(tag);
    switch (tag) {
    case 0: case 2: case 8: o.be(fixed, 4); return true;
    case 1: o.var((uint32_t)fixed); return true;
    case 3: {
        const int32_t n = (int32_t)(uint32_t)fixed;
        o.var(((uint32_t)n << 1) ^ (uint32_t)(n >> 31));
        return true;
    }
    case 4: case 6: case 9: o.be(fixed, 8); return true;
    case 5: o.var(fixed); return true;
    case 7: {
        const int64_t n = (int64_t)fixed;
        o.var(((uint64_t)n << 1) ^ (uint64_t)(n >> 63));
        return true;
    }
    case 10: case 11: o.be(fixed, 8); o.be(aux, 4); return true;
    case 12: case 13:
        if (aux && !text) break;
        o.var(aux);
        o.bytes(text, aux);
        return true;
    case 14: case 15: case 16: return true;
    case 23: case 24: o.be(fixed, 1); return true;
    case 25: case 26: o.be(fixed, 2); return true;
    default: break;
    }
    serr(err, "value tag %u is not a scalar this builder writes", tag);
    return false;
}

bool send_all(int fd, const void* p, size_t n, NetidxError* err) {
    const uint8_t* q = static_cast<const uint8_t*>(p);
    while (n) {
        const ssize_t k = ::send(fd, q, n, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            serr(err, "send: %s", strerror(errno));
            return false;
        }
        q += k;
        n -= (size_t)k;
    }
    return true;
}

}  // namespace

struct NxgSession {
    int fd = -1;
    bool listener = false;
    // reassembly: bytes [head, tail) of buf are read and not yet handed out
    uint8_t* buf = nullptr;
    size_t cap = 0, head = 0, tail = 0;
    bool pinned = false;
    // publish staging (pinned) and device output
    uint8_t* sbuf = nullptr;
    size_t scap = 0;
    uint8_t* dout = nullptr;
    size_t dcap = 0;
    uint64_t frames_in = 0, bytes_in = 0, frames_out = 0, bytes_out = 0;
};

namespace {

void free_buf(NxgSession* s) {
    if (!s->buf) return;
    if (s->pinned) (void)hipHostFree(s->buf);
    else free(s->buf);
    s->buf = nullptr;
    s->cap = 0;
}

// room for `need` contiguous bytes from head (moving or growing the buffer)
bool reserve(NxgSession* s, size_t need, NetidxError* err) {
    if (s->head + need <= s->cap) return true;
    const size_t have = s->tail - s->head;
    if (need <= s->cap && s->head) {
        memmove(s->buf, s->buf + s->head, have);
        s->head = 0;
        s->tail = have;
        return true;
    }
    size_t n = s->cap ? s->cap : kRecvChunk;
    while (n < need) n *= 2;
    uint8_t* nb = nullptr;
    if (s->pinned) {
        if (hipHostMalloc((void**)&nb, n, hipHostMallocDefault) != hipSuccess) nb = nullptr;
    } else {
        nb = static_cast<uint8_t*>(malloc(n));
    }
    if (!nb) {
        serr(err, "receive buffer of %zu bytes: out of memory", n);
        return false;
    }
    if (have) memcpy(nb, s->buf + s->head, have);
    free_buf(s);
    s->buf = nb;
    s->cap = n;
    s->head = 0;
    s->tail = have;
    return true;
}

// read until `n` bytes are buffered from head; false on EOF or error. The buffer grows only as
// bytes arrive (room for at most twice what is buffered, or one receive chunk more), so a peer's
// length field alone never allocates (pins) a large buffer -- as read_task's buffer grows with
// what it has read (channel.rs:426-437).
bool fill(NxgSession* s, size_t n, NetidxError* err) {
    while (s->tail - s->head < n) {
        const size_t have = s->tail - s->head;
        const size_t want = std::min(n, std::max(2 * have, have + kRecvChunk));
        if (!reserve(s, want, err)) return false;
        size_t room = s->cap - s->tail;
        if (room > kRecvChunk && have + kRecvChunk >= n) room = kRecvChunk;
        const ssize_t k = ::recv(s->fd, s->buf + s->tail, room, 0);
        if (k < 0) {
            if (errno == EINTR) continue;
            serr(err, "recv: %s", strerror(errno));
            return false;
        }
        if (k == 0) {
            serr(err, "connection closed");
            return false;
        }
        s->tail += (size_t)k;
        s->bytes_in += (uint64_t)k;
    }
    return true;
}

// read_raw (channel.rs:85-105): one small unencrypted message, decoded exactly
bool read_raw(NxgSession* s, size_t max, const uint8_t** body, uint32_t* len, NetidxError* err) {
    if (!fill(s, 4, err)) return false;
    const uint8_t* h = s->buf + s->head;
    const uint32_t n = ((uint32_t)h[0] << 24) | ((uint32_t)h[1] << 16) | ((uint32_t)h[2] << 8) | h[3];
    if (n > kLenMask) {
        serr(err, "message is encrypted");
        return false;
    }
    if (n > max) {
        serr(err, "message is too large");
        return false;
    }
    if (!fill(s, 4 + (size_t)n, err)) return false;
    *body = s->buf + s->head + 4;
    *len = n;
    s->head += 4 + (size_t)n;
    return true;
}

bool write_raw(NxgSession* s, const std::vector<uint8_t>& msg, NetidxError* err) {
    uint8_t h[4];
    nxg_frame_header((uint32_t)msg.size(), false, h);
    std::vector<uint8_t> all(h, h + 4);
    all.insert(all.end(), msg.begin(), msg.end());
    return send_all(s->fd, all.data(), all.size(), err);
}

std::vector<uint8_t> version_msg() {
    Out o;
    o.be(kProtocolVersion, 8);  // <u64 as Pack>: big-endian (pack.rs:669-690)
    return o.b;
}

bool check_version(const uint8_t* b, uint32_t n, NetidxError* err) {
    if (n != 8) {
        serr(err, n < 8 ? "version: buffer short" : "batch contained more than one message");
        return false;
    }
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | b[i];
    if (v != kProtocolVersion) {
        serr(err, "incompatible protocol version");
        return false;
    }
    return true;
}

// Hello (netproto publisher.rs:17-48) as a derived enum: 0 Anonymous, 1 Krb5, 2 Local, 3 Tls..
// returns the variant, or -1 (err set) when the raw message is not one well-formed Hello
int parse_hello(const uint8_t* b, uint32_t n, NetidxError* err) {
    uint64_t L = 0;
    uint32_t k = 0, shift = 0;
    for (; k < n && k < 10; k++) {
        L |= (uint64_t)(b[k] & 0x7f) << shift;
        shift += 7;
        if (b[k] < 0x80) break;
    }
    if (k >= n || L < 1) {
        serr(err, "hello: buffer short");
        return -1;
    }
    k++;
    const uint64_t take = L - vlen(L);
    if (take < 1 || k + take > n) {
        serr(err, "hello: buffer short");
        return -1;
    }
    if (k + take != n) {
        serr(err, "batch contained more than one message");
        return -1;
    }
    return b[k];
}

NxgSession* new_session(int fd, NetidxError* err) {
    NxgSession* s = new (std::nothrow) NxgSession();
    if (!s) {
        close(fd);
        serr(err, "out of memory");
        return nullptr;
    }
    s->fd = fd;
    const int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    int big = 16 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof big);
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof big);
    return s;
}

}  // namespace

extern "C" {

NxgSession* nxg_session_connect(const char* ipv4, uint16_t port, NetidxError* err) {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(port);
    if (!ipv4 || inet_pton(AF_INET, ipv4, &a.sin_addr) != 1) {
        serr(err, "bad IPv4 address");
        return nullptr;
    }
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) {
        serr(err, "socket: %s", strerror(errno));
        return nullptr;
    }
    if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
        serr(err, "connect: %s", strerror(errno));
        close(fd);
        return nullptr;
    }
    NxgSession* s = new_session(fd, err);
    if (!s) return nullptr;
    // hello_publisher (subscriber/connection.rs:120-140), anonymous
    const uint8_t* b;
    uint32_t n;
    int v;
    if (!write_raw(s, version_msg(), err) || !read_raw(s, 1024, &b, &n, err) ||
        !check_version(b, n, err) || !write_raw(s, wrap(0, {}), err) ||
        !read_raw(s, 8124, &b, &n, err) || (v = parse_hello(b, n, err)) < 0) {
        nxg_session_close(s);
        return nullptr;
    }
    if (v != 0) {
        serr(err, "unexpected response from publisher");
        nxg_session_close(s);
        return nullptr;
    }
    return s;
}

NxgSession* nxg_session_listen(const char* ipv4, uint16_t port, uint16_t* bound_port,
                               NetidxError* err) {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(port);
    if (!ipv4 || inet_pton(AF_INET, ipv4, &a.sin_addr) != 1) {
        serr(err, "bad IPv4 address");
        return nullptr;
    }
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) {
        serr(err, "socket: %s", strerror(errno));
        return nullptr;
    }
    const int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    socklen_t al = sizeof a;
    if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 || listen(fd, 16) != 0 ||
        getsockname(fd, reinterpret_cast<sockaddr*>(&a), &al) != 0) {
        serr(err, "bind/listen: %s", strerror(errno));
        close(fd);
        return nullptr;
    }
    NxgSession* s = new (std::nothrow) NxgSession();
    if (!s) {
        close(fd);
        serr(err, "out of memory");
        return nullptr;
    }
    s->fd = fd;
    s->listener = true;
    if (bound_port) *bound_port = ntohs(a.sin_port);
    return s;
}

NxgSession* nxg_session_accept(NxgSession* l, NetidxError* err) {
    if (!l || !l->listener) {
        serr(err, "not a listening session");
        return nullptr;
    }
    int fd;
    do {
        fd = accept(l->fd, nullptr, nullptr);
    } while (fd < 0 && errno == EINTR);
    if (fd < 0) {
        serr(err, "accept: %s", strerror(errno));
        return nullptr;
    }
    NxgSession* s = new_session(fd, err);
    if (!s) return nullptr;
    // ClientCtx::hello (publisher/server.rs:367-381): anonymous only
    const uint8_t* b;
    uint32_t n;
    int v;
    if (!write_raw(s, version_msg(), err) || !read_raw(s, 1024, &b, &n, err) ||
        !check_version(b, n, err) || !read_raw(s, 8124, &b, &n, err) ||
        (v = parse_hello(b, n, err)) < 0) {
        nxg_session_close(s);
        return nullptr;
    }
    if (v != 0) {
        serr(err, "authentication mechanism not supported");
        nxg_session_close(s);
        return nullptr;
    }
    if (!write_raw(s, wrap(0, {}), err)) {
        nxg_session_close(s);
        return nullptr;
    }
    return s;
}

void nxg_session_close(NxgSession* s) {
    if (!s) return;
    if (s->fd >= 0) close(s->fd);
    free_buf(s);
    if (s->sbuf) (void)hipHostFree(s->sbuf);
    if (s->dout) (void)hipFree(s->dout);
    delete s;
}

void nxg_session_stats(const NxgSession* s, uint64_t out[4]) {
    out[0] = s ? s->frames_in : 0;
    out[1] = s ? s->bytes_in : 0;
    out[2] = s ? s->frames_out : 0;
    out[3] = s ? s->bytes_out : 0;
}

// ---- control messages ---------------------------------------------------------------------------
int64_t nxg_msg_subscribe(const char* path, uint64_t path_len, uint32_t resolver_ipv4,
                          uint16_t resolver_port, uint64_t timestamp, uint32_t permissions,
                          const uint8_t* token, uint64_t token_len, uint8_t* out, uint64_t cap) {
    Out f;
    f.var(path_len);  // Path = ArcStr (pack.rs:449-469)
    f.bytes(path, path_len);
    f.u8(0);  // SocketAddr::V4 (pack.rs:187-205)
    f.be(resolver_ipv4, 4);
    f.be(resolver_port, 2);
    f.be(timestamp, 8);
    f.be(permissions, 4);
    f.var(token_len);  // Bytes (pack.rs:238-247)
    if (token_len) f.bytes(token, token_len);
    const std::vector<uint8_t> m = wrap(0, f.b);  // To::Subscribe is variant 0
    if (out) {
        if (m.size() > cap) return -(int64_t)NXG_CAPACITY;
        memcpy(out, m.data(), m.size());
    }
    return (int64_t)m.size();
}

int64_t nxg_msg_subscribed(const char* path, uint64_t path_len, uint64_t id, uint8_t tag,
                           uint64_t fixed, uint32_t aux, const uint8_t* text, uint8_t* out,
                           uint64_t cap) {
    Out f;
    f.var(path_len);
    f.bytes(path, path_len);
    f.var(id);
    if (!put_value(f, tag, fixed, aux, text, nullptr)) return -(int64_t)NXG_UNKNOWN_TAG;
    const std::vector<uint8_t> m = wrap(3, f.b);  // From::Subscribed is variant 3
    if (out) {
        if (m.size() > cap) return -(int64_t)NXG_CAPACITY;
        memcpy(out, m.data(), m.size());
    }
    return (int64_t)m.size();
}

int64_t nxg_msg_update(uint64_t id, uint8_t tag, uint64_t fixed, uint32_t aux,
                       const uint8_t* text, uint8_t* out, uint64_t cap) {
    Out f;
    f.var(id);  // publisher::Id (netidx-core utils.rs:147-164)
    if (!put_value(f, tag, fixed, aux, text, nullptr)) return -NXG_UNKNOWN_TAG;
    const std::vector<uint8_t> m = wrap(4, f.b);  // From::Update (netproto publisher.rs:90)
    if (!out) return (int64_t)m.size();
    if (cap < m.size()) return -NXG_CAPACITY;
    memcpy(out, m.data(), m.size());
    return (int64_t)m.size();
}

int64_t nxg_msg_heartbeat(uint8_t* out, uint64_t cap) {
    if (out) {
        if (cap < 2) return -(int64_t)NXG_CAPACITY;
        out[0] = 2;  // lw(1)
        out[1] = 5;  // From::Heartbeat
    }
    return 2;
}

// One publisher::From or To message at buf (a len-wrapped derived enum). Fields of the variants
// the connection's control plane needs; anything else is reported by variant and span only.
bool nxg_msg_parse(const uint8_t* buf, uint64_t len, int to, NxgCtlMsg* m, NetidxError* err) {
    memset(m, 0, sizeof *m);
    uint64_t p = 0, L = 0;
    uint32_t shift = 0;
    for (;; p++) {
        if (p >= len || p >= 10) {
            serr(err, "message length: buffer short");
            return false;
        }
        L |= (uint64_t)(buf[p] & 0x7f) << shift;
        shift += 7;
        if (buf[p] < 0x80) break;
    }
    p++;
    if (L < 1) {
        serr(err, "message length: buffer short");
        return false;
    }
    const uint64_t take = L - vlen(L);
    const uint64_t lim = take < len - p ? p + take : len;
    m->msg_len = lim;
    if (p >= lim) {
        serr(err, "message: buffer short");
        return false;
    }
    m->variant = buf[p++];
    auto var = [&](uint64_t& v) {
        v = 0;
        uint32_t sh = 0;
        for (int i = 0; i < 10; i++) {
            if (p >= lim) return false;
            const uint8_t b = buf[p++];
            v |= (uint64_t)(b & 0x7f) << sh;
            sh += 7;
            if (b < 0x80) return true;
        }
        return false;
    };
    auto be = [&](int n, uint64_t& v) {
        if (lim - p < (uint64_t)n) return false;
        v = 0;
        for (int i = 0; i < n; i++) v = (v << 8) | buf[p++];
        return true;
    };
    auto text = [&](uint64_t& off, uint64_t& n) {
        if (!var(n) || n > lim - p) return false;
        off = p;
        p += n;
        return true;
    };
    auto value = [&]() {  // the value's span; scalars decoded
        m->value_off = p;
        if (p >= lim) return false;
        const uint8_t t = buf[p++];
        m->value_tag = t;
        uint64_t v, v2, off, n;
        switch (t) {
        case 0: case 2: case 8: if (!be(4, v)) return false; m->value_fixed = v; break;
        case 4: case 6: case 9: if (!be(8, v)) return false; m->value_fixed = v; break;
        case 1: case 3: case 5: case 7: if (!var(v)) return false; m->value_fixed = v; break;
        case 10: case 11:
            if (!be(8, v) || !be(4, v2)) return false;
            m->value_fixed = v;
            m->value_aux = (uint32_t)v2;
            break;
        case 12: case 13: case 18:
            if (!text(off, n)) return false;
            m->value_fixed = off;
            m->value_aux = (uint32_t)n;
            break;
        case 14: case 15: case 16: case 17: break;
        case 23: case 24: if (!be(1, v)) return false; m->value_fixed = v; break;
        case 25: case 26: if (!be(2, v)) return false; m->value_fixed = v; break;
        default: p = lim; break;  // containers, Decimal, Abstract: the span only
        }
        m->value_len = p - m->value_off;
        return true;
    };
    bool ok = true;
    if (!to) {  // publisher::From (netproto publisher.rs:73-96)
        switch (m->variant) {
        case 0: case 1: ok = text(m->path_off, m->path_len); break;  // NoSuchValue / Denied
        case 2: ok = var(m->id); break;                               // Unsubscribed(Id)
        case 3: ok = text(m->path_off, m->path_len) && var(m->id) && value(); break;
        case 4: ok = var(m->id) && value(); break;                    // Update
        case 5: break;                                                // Heartbeat
        case 6: ok = var(m->id) && value(); break;                    // WriteResult
        default: serr(err, "unknown From variant %u", m->variant); return false;
        }
    } else {  // publisher::To (publisher.rs:51-70)
        uint64_t v;
        switch (m->variant) {
        case 0:  // Subscribe { path, resolver, timestamp, permissions, token }
            ok = text(m->path_off, m->path_len) && be(1, v);
            if (ok && v == 0) ok = be(4, v) && be(2, v);
            else if (ok && v == 1) ok = lim - p >= 26 && (p += 26, true);
            else if (ok) ok = false;
            ok = ok && be(8, m->timestamp) && be(4, v) && text(m->token_off, m->token_len);
            m->permissions = (uint32_t)v;
            break;
        case 1: ok = var(m->id); break;  // Unsubscribe(Id)
        case 2: ok = var(m->id) && be(1, v) && value(); break;  // Write(Id, bool, Value, ..)
        default: serr(err, "unknown To variant %u", m->variant); return false;
        }
    }
    if (!ok) {
        serr(err, "malformed message (variant %u)", m->variant);
        return false;
    }
    return true;
}

// ---- the channel: frames ------------------------------------------------------------------------
bool nxg_session_send(NxgSession* s, const uint8_t* payload, uint64_t len, NetidxError* err) {
    if (!s || s->listener || (len && !payload)) {
        serr(err, "bad session or payload");
        return false;
    }
    if (len > kMaxBatch) {
        serr(err, "frame of %llu bytes exceeds MAX_BATCH", (unsigned long long)len);
        return false;
    }
    uint8_t h[4];
    nxg_frame_header((uint32_t)len, false, h);
    if (!send_all(s->fd, h, 4, err) || !send_all(s->fd, payload, len, err)) return false;
    s->frames_out++;
    s->bytes_out += 4 + len;
    return true;
}

bool nxg_session_recv_frame(NxgSession* s, const uint8_t** payload, uint64_t* len,
                            NetidxError* err) {
    if (!s || s->listener || !payload || !len) {
        serr(err, "bad session or output");
        return false;
    }
    if (!fill(s, 4, err)) return false;
    uint32_t n;
    bool enc;
    nxg_frame_parse_header(s->buf + s->head, 4, &n, &enc);
    if (enc) {  // read_task without a security context (channel.rs:420-422)
        serr(err, "encryption is not supported");
        return false;
    }
    if (!fill(s, 4 + (size_t)n, err)) return false;
    *payload = s->buf + s->head + 4;
    *len = n;
    s->head += 4 + (size_t)n;
    if (s->head == s->tail) s->head = s->tail = 0;
    s->frames_in++;
    return true;
}

bool nxg_session_recv_decode(NxgSession* s, NxgCtx* ctx, NxgColumns* out, uint32_t flags,
                             NxgStatus* status, uint64_t* frame_len, NetidxError* err) {
    if (!s || !ctx || !out) {
        serr(err, "null argument");
        return false;
    }
    if (!s->pinned) {  // receive straight into page-locked memory from now on
        const size_t have = s->tail - s->head;
        uint8_t* nb = nullptr;
        const size_t n = s->cap > kRecvChunk ? s->cap : kRecvChunk;
        if (hipHostMalloc((void**)&nb, n, hipHostMallocDefault) != hipSuccess) {
            serr(err, "pinned receive buffer of %zu bytes failed", n);
            return false;
        }
        if (have) memcpy(nb, s->buf + s->head, have);
        free_buf(s);
        s->buf = nb;
        s->cap = n;
        s->head = 0;
        s->tail = have;
        s->pinned = true;
    }
    const uint8_t* p;
    uint64_t n;
    if (!nxg_session_recv_frame(s, &p, &n, err)) return false;
    if (frame_len) *frame_len = n;
    return nxg_decode_updates(ctx, p, n, out, flags, status, err);
}

bool nxg_session_publish(NxgSession* s, NxgCtx* ctx, const NxgColumns* cols, const uint8_t* heap,
                         uint64_t* bytes_sent, NetidxError* err) {
    if (!s || !ctx || !cols || s->listener) {
        serr(err, "null argument");
        return false;
    }
    uint64_t need = 0;
    if (!nxg_encoded_len(ctx, cols, heap, &need, err)) return false;
    if (need + 64 > s->dcap) {
        if (s->dout) (void)hipFree(s->dout);
        s->dout = nullptr;
        s->dcap = 0;
        if (hipMalloc((void**)&s->dout, need + 64) != hipSuccess) {
            serr(err, "device frame buffer of %llu bytes failed", (unsigned long long)need);
            return false;
        }
        s->dcap = need + 64;
    }
    if (need > s->scap) {
        if (s->sbuf) (void)hipHostFree(s->sbuf);
        s->sbuf = nullptr;
        s->scap = 0;
        if (hipHostMalloc((void**)&s->sbuf, need, hipHostMallocDefault) != hipSuccess) {
            serr(err, "pinned send buffer of %llu bytes failed", (unsigned long long)need);
            return false;
        }
        s->scap = need;
    }
    uint64_t total = 0, chunks[8], nc = 0;
    if (!nxg_encode_frames(ctx, cols, heap, s->dout, s->dcap, &total, chunks, 8, &nc, err))
        return false;
    if (total && hipMemcpy(s->sbuf, s->dout, total, hipMemcpyDeviceToHost) != hipSuccess) {
        serr(err, "device-to-host copy of the frames failed");
        return false;
    }
    uint64_t off = 0;
    for (uint64_t k = 0; k < nc; k++) {
        if (!nxg_session_send(s, s->sbuf + off, chunks[k], err)) return false;
        off += chunks[k];
    }
    if (bytes_sent) *bytes_sent = total + 4 * nc;
    return true;
}

}  // extern "C"
