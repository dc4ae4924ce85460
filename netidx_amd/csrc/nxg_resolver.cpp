// nxg_resolver.cpp -- a minimal, anonymous, machine-local resolver for BASELINE configs[0]
// (simple_publisher + simple_subscriber over loopback), in C++ on the host: the server, and the
// write (publisher) and read (subscriber) clients, speaking the reference's resolver protocol
// byte for byte. Control plane only: no kernels, no GPU.
//
//   handshake (netidx/src/resolver_server/mod.rs:823-860 hello_client): both sides write the
//     version u64 3 and read the other's as raw messages (u32 big-endian length + packed value,
//     channel.rs:63-105), then the client sends its ClientHello (netproto resolver.rs:60-72):
//   ReadOnly(AuthRead::Anonymous) (resolver_client/read_client.rs:84-99): the server answers
//     AuthRead::Anonymous (mod.rs:779-781); then frames of ToRead, answered per batch by
//     FromRead::Publisher for each publisher named, then one reply per request in order
//     (shard_store.rs:575-640): Resolve(path) -> Resolved { resolver, publishers: [PublisherRef
//     { id, token: empty }], timestamp: now, flags, permissions: Permissions::all() }
//     (shard_store.rs:176-193, store.rs:581-609); other requests -> FromRead::Error.
//   WriteOnly(ClientHelloWrite { write_addr, auth: Anonymous, priority }) (write_client.rs:
//     194-221): the server answers ServerHelloWrite { ttl, ttl_expired, auth: Anonymous,
//     resolver_id } (mod.rs:458-480); then frames of ToWrite: Publish / PublishDefault /
//     PublishWithFlags (flags kept) -> FromWrite::Published, Unpublish / UnpublishDefault / Clear
//     -> FromWrite::Unpublished, a batch of one Heartbeat -> nothing (mod.rs:300-345).
//
// Message layouts are the derive rules (netidx-derive lib.rs): structs and enums length-wrapped,
// enum variants by declaration order; SocketAddr V4 = 00 u32 u16 (pack.rs:187-237); Option =
// 0 / 1 + value (pack.rs:1389-1414); Vec = varint count + elements; Bytes / Path / ArcStr =
// varint length + bytes.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <map>
#include <mutex>
#include <string>
#include <list>
#include <thread>
#include <vector>

#include "../../include/nxg_codec.h"
#include "nxg_wire.h"

namespace {
using namespace nxgwire;

void rerr(NetidxError* err, const char* fmt, ...) {
    if (!err) return;
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    free(err->msg);
    err->msg = strdup(buf);
}

constexpr uint64_t kVersion = 3;          // resolver_server/mod.rs:829-834
constexpr uint32_t kMaxFrame = 64u << 20; // control frames only
constexpr uint32_t kPermAll = 0x3f;       // Permissions::all() (resolver_server/auth.rs:23-30)

struct Addr4 {
    uint32_t ip = 0;  // host order
    uint16_t port = 0;
};
void put_addr(Out& o, Addr4 a) {  // SocketAddr::V4 (pack.rs:195-201)
    o.u8(0);
    o.be(a.ip, 4);
    o.be(a.port, 2);
}
bool get_addr(In& in, Addr4& a) {
    uint32_t t;
    uint64_t ip, port;
    if (!in.u8(t) || t != 0) return false;  // V6 is not spoken on the loopback path
    if (!in.be(ip, 4) || !in.be(port, 2)) return false;
    a.ip = (uint32_t)ip;
    a.port = (uint16_t)port;
    return true;
}
void put_str(Out& o, const std::string& s) {
    o.var(s.size());
    o.bytes(s.data(), s.size());
}
std::vector<uint8_t> unit(uint32_t variant) { return wrap(variant, {}); }

bool send_all(int fd, const uint8_t* p, size_t n) {
    while (n) {
        const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
        if (k < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        p += k;
        n -= (size_t)k;
    }
    return true;
}
bool recv_all(int fd, uint8_t* p, size_t n) {
    while (n) {
        const ssize_t k = ::recv(fd, p, n, 0);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        p += k;
        n -= (size_t)k;
    }
    return true;
}
// one frame / raw message: u32 big-endian length (bit 31: encrypted, refused) + payload
bool send_frame(int fd, const std::vector<uint8_t>& payload) {
    uint8_t h[4];
    nxg_frame_header((uint32_t)payload.size(), false, h);
    std::vector<uint8_t> all(h, h + 4);
    all.insert(all.end(), payload.begin(), payload.end());
    return send_all(fd, all.data(), all.size());
}
bool recv_frame(int fd, std::vector<uint8_t>& payload) {
    uint8_t h[4];
    if (!recv_all(fd, h, 4)) return false;
    uint32_t n;
    bool enc;
    nxg_frame_parse_header(h, 4, &n, &enc);
    if (enc || n > kMaxFrame) return false;
    payload.resize(n);
    return n == 0 || recv_all(fd, payload.data(), n);
}
std::vector<uint8_t> version_msg() {
    Out o;
    o.be(kVersion, 8);
    return o.b;
}
bool check_version(const std::vector<uint8_t>& b) {
    In in(b.data(), b.size());
    uint64_t v;
    return in.be(v, 8) && in.left() == 0 && v == kVersion;
}

int dial(const char* ipv4, uint16_t port, NetidxError* err) {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(port);
    if (!ipv4 || inet_pton(AF_INET, ipv4, &a.sin_addr) != 1) {
        rerr(err, "bad IPv4 address");
        return -1;
    }
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) {
        rerr(err, "socket: %s", strerror(errno));
        return -1;
    }
    if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
        rerr(err, "connect %s:%u: %s", ipv4, port, strerror(errno));
        close(fd);
        return -1;
    }
    const int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    return fd;
}

// ---- messages --------------------------------------------------------------------------------
// Publisher (resolver.rs:181-192): resolver, id, addr, hash_method, target_auth, user_info,
// priority; an anonymous publisher: Sha3_512, TargetAuth::Anonymous, no UserInfo
std::vector<uint8_t> publisher_msg(Addr4 resolver, uint64_t id, Addr4 addr, uint32_t priority) {
    Out f;
    put_addr(f, resolver);
    f.var(id);
    put_addr(f, addr);
    f.bytes(unit(0).data(), 2);          // HashMethod::Sha3_512
    f.bytes(unit(0).data(), 2);          // TargetAuth::Anonymous
    f.u8(0);                             // user_info: None
    const auto pr = unit(priority);      // PublisherPriority
    f.bytes(pr.data(), pr.size());
    return wrap(0, wrap_struct(f.b));    // FromRead::Publisher
}
// Resolved (resolver.rs:201-208)
std::vector<uint8_t> resolved_msg(Addr4 resolver, const std::vector<uint64_t>& ids, uint64_t now,
                                  uint32_t flags) {
    Out f;
    put_addr(f, resolver);
    f.var(ids.size());
    for (uint64_t id : ids) {  // PublisherRef { id, token: Bytes::new() }
        Out r;
        r.var(id);
        r.var(0);
        const auto w = wrap_struct(r.b);
        f.bytes(w.data(), w.size());
    }
    f.be(now, 8);
    f.be(flags, 4);
    f.be(kPermAll, 4);
    return wrap(1, wrap_struct(f.b));  // FromRead::Resolved
}
std::vector<uint8_t> error_msg(uint32_t variant, const char* what) {
    Out f;
    put_str(f, what);
    return wrap(variant, f.b);
}

}  // namespace

// ---- server ------------------------------------------------------------------------------------
struct NxgResolver {
    int lfd = -1;
    Addr4 self;
    uint64_t ttl = 0;
    std::atomic<bool> stop{false};
    std::thread acceptor;
    std::mutex mu;
    // one thread per connection; a finished connection closes its socket at once (the peer sees
    // EOF) and its thread is joined by the acceptor at the next accept, or by nxg_resolver_stop
    struct Conn {
        std::thread t;
        int fd;
        bool done = false;
    };
    std::list<Conn> conns;
    struct Pub {
        uint64_t id;
        Addr4 addr;
        uint32_t priority;
        uint64_t last_seen;  // seconds: the last message on its write connection (writer TTL)
        int fd;              // its write connection
    };
    std::vector<Pub> pubs;                                  // by connection, PublisherId order
    std::map<std::string, std::pair<uint64_t, uint32_t>> published;  // path -> (id, flags)
    uint64_t next_id = 0;

    void serve(int fd);
    void serve_read(int fd);
    void serve_write(int fd, const Addr4& write_addr, uint32_t priority);
    // (under mu) forget a publisher: its paths and its entry
    void drop_publisher(uint64_t id) {
        for (auto it = published.begin(); it != published.end();)
            it = it->second.first == id ? published.erase(it) : std::next(it);
        for (auto it = pubs.begin(); it != pubs.end();)
            it = it->id == id ? pubs.erase(it) : std::next(it);
    }
    // (under mu) publishers silent for longer than the writer TTL are expired: their data is
    // dropped and their write connection shut down, as the reference's resolver times out a
    // silent writer's connection (resolver_server/mod.rs:289-299) -- the publisher reconnects
    // and is told ttl_expired; its serving thread sees the socket end and leaves
    void expire(uint64_t now) {
        if (!ttl) return;
        std::vector<std::pair<uint64_t, int>> dead;
        for (const Pub& p : pubs)
            if (now > p.last_seen + ttl) dead.push_back({p.id, p.fd});
        for (const auto& d : dead) {
            drop_publisher(d.first);
            shutdown(d.second, SHUT_RDWR);
        }
    }
    bool live(uint64_t id) const {
        for (const Pub& p : pubs)
            if (p.id == id) return true;
        return false;
    }
    void touch(uint64_t id, uint64_t now) {
        for (Pub& p : pubs)
            if (p.id == id) p.last_seen = now;
    }
    // (under mu) join the threads of finished connections
    void reap() {
        for (auto it = conns.begin(); it != conns.end();) {
            if (it->done) {
                if (it->t.joinable()) it->t.join();
                it = conns.erase(it);
            } else {
                ++it;
            }
        }
    }
};

void NxgResolver::serve(int fd) {
    std::vector<uint8_t> m;
    if (!send_frame(fd, version_msg()) || !recv_frame(fd, m) || !check_version(m)) return;
    if (!recv_frame(fd, m)) return;
    In in(m.data(), m.size());
    size_t end;
    uint32_t variant;
    if (!in.wrapped(end) || !in.u8(variant)) return;
    if (variant == 0) {  // ReadOnly(AuthRead)
        size_t e2;
        uint32_t auth;
        if (!in.wrapped(e2) || !in.u8(auth) || auth != 0) return;  // Anonymous only
        if (!send_frame(fd, unit(0))) return;                       // AuthRead::Anonymous
        serve_read(fd);
    } else if (variant == 1) {  // WriteOnly(ClientHelloWrite)
        size_t e2, e3;
        Addr4 wa;
        uint32_t auth, prio = 1;  // #[pack(default)] priority: Normal
        if (!in.wrapped(e2) || !get_addr(in, wa) || !in.wrapped(e3) || !in.u8(auth) || auth != 0)
            return;
        in.i = e3;
        size_t e4;
        if (in.i < e2 && in.wrapped(e4)) {
            uint32_t p;
            if (in.u8(p) && p <= 2) prio = p;
        }
        serve_write(fd, wa, prio);
    }
}

void NxgResolver::serve_read(int fd) {
    std::vector<uint8_t> m;
    while (!stop && recv_frame(fd, m)) {
        Out reply;
        std::vector<std::vector<uint8_t>> answers;
        std::vector<uint64_t> named;  // publishers to describe first (once per batch)
        In in(m.data(), m.size());
        const uint64_t now = (uint64_t)time(nullptr);
        while (in.left()) {
            size_t end;
            uint32_t variant;
            if (!in.wrapped(end) || !in.u8(variant)) return;  // PackError: drop the client
            if (variant == 0) {  // Resolve(Path)
                std::string path;
                if (!in.str(path)) return;
                std::vector<uint64_t> ids;
                uint32_t flags = 0;
                {
                    std::lock_guard<std::mutex> g(mu);
                    expire(now);
                    auto it = published.find(path);
                    if (it != published.end()) {
                        ids.push_back(it->second.first);
                        flags = it->second.second;
                    }
                }
                for (uint64_t id : ids) {
                    bool seen = false;
                    for (uint64_t x : named) seen |= x == id;
                    if (!seen) named.push_back(id);
                }
                answers.push_back(resolved_msg(self, ids, now, flags));
            } else {
                answers.push_back(error_msg(6, "not supported by the machine-local resolver"));
            }
            in.i = end;
        }
        {
            std::lock_guard<std::mutex> g(mu);
            for (uint64_t id : named)
                for (const Pub& p : pubs)
                    if (p.id == id) {
                        const auto b = publisher_msg(self, p.id, p.addr, p.priority);
                        reply.bytes(b.data(), b.size());
                    }
        }
        for (const auto& a : answers) reply.bytes(a.data(), a.size());
        if (!send_frame(fd, reply.b)) return;
    }
}

void NxgResolver::serve_write(int fd, const Addr4& write_addr, uint32_t priority) {
    uint64_t id;
    {
        std::lock_guard<std::mutex> g(mu);
        id = next_id++;
        pubs.push_back(Pub{id, write_addr, priority, (uint64_t)time(nullptr), fd});
    }
    // a write connection that ends (peer gone, or dropped on a PackError) takes its paths with it
    struct Drop {
        NxgResolver* r;
        uint64_t id;
        ~Drop() {
            std::lock_guard<std::mutex> g(r->mu);
            r->drop_publisher(id);
        }
    } drop{this, id};
    {  // ServerHelloWrite { ttl, ttl_expired, auth: Anonymous, resolver_id }
        Out f;
        f.be(ttl, 8);
        f.u8(1);  // ttl_expired: a new publisher has nothing to keep
        f.bytes(unit(0).data(), 2);
        put_addr(f, self);
        if (!send_frame(fd, wrap_struct(f.b))) return;
    }
    std::vector<uint8_t> m;
    while (!stop && recv_frame(fd, m)) {
        Out reply;
        In in(m.data(), m.size());
        size_t n_msgs = 0, n_heartbeat = 0;
        {
            std::lock_guard<std::mutex> g(mu);
            if (!live(id)) return;  // expired while this batch was on its way
            touch(id, (uint64_t)time(nullptr));
        }
        while (in.left()) {
            size_t end;
            uint32_t variant;
            if (!in.wrapped(end) || !in.u8(variant)) return;
            n_msgs++;
            std::string path;
            uint64_t flags = 0;
            switch (variant) {
            case 0: case 1: case 5: case 6:  // Publish, PublishDefault, ..WithFlags(path, u32)
                if (!in.str(path)) return;
                if ((variant == 5 || variant == 6) && !in.be(flags, 4)) return;
                {
                    std::lock_guard<std::mutex> g(mu);
                    if (!live(id)) return;  // expired: no path under an id resolve cannot map
                    published[path] = {id, (uint32_t)flags};
                }
                reply.bytes(unit(0).data(), 2);  // FromWrite::Published
                break;
            case 2: case 7:  // Unpublish, UnpublishDefault
                if (!in.str(path)) return;
                {
                    std::lock_guard<std::mutex> g(mu);
                    auto it = published.find(path);
                    if (it != published.end() && it->second.first == id) published.erase(it);
                }
                reply.bytes(unit(1).data(), 2);  // FromWrite::Unpublished
                break;
            case 3: {  // Clear
                std::lock_guard<std::mutex> g(mu);
                for (auto it = published.begin(); it != published.end();)
                    it = it->second.first == id ? published.erase(it) : std::next(it);
                reply.bytes(unit(1).data(), 2);
                break;
            }
            case 4:  // Heartbeat
                n_heartbeat++;
                break;
            default:
                return;  // UnknownTag: drop the client
            }
            in.i = end;
        }
        if (n_msgs == n_heartbeat) continue;  // a batch of heartbeats is not answered
        if (!send_frame(fd, reply.b)) return;
    }
}

// ---- write / read clients ---------------------------------------------------------------------
struct NxgResolverClient {
    int fd = -1;
    bool write = false;
    uint64_t ttl = 0;
};

namespace {
NxgResolverClient* client_hello(const char* ipv4, uint16_t port, const std::vector<uint8_t>& hello,
                                bool write, NetidxError* err) {
    const int fd = dial(ipv4, port, err);
    if (fd < 0) return nullptr;
    std::vector<uint8_t> m;
    auto fail = [&](const char* what) -> NxgResolverClient* {
        rerr(err, "resolver handshake: %s", what);
        close(fd);
        return nullptr;
    };
    if (!send_frame(fd, version_msg()) || !recv_frame(fd, m)) return fail("version");
    if (!check_version(m)) return fail("incompatible protocol version");
    if (!send_frame(fd, hello) || !recv_frame(fd, m)) return fail("hello");
    NxgResolverClient* c = new NxgResolverClient();
    c->fd = fd;
    c->write = write;
    In in(m.data(), m.size());
    size_t end;
    if (!write) {  // AuthRead::Anonymous
        uint32_t v;
        if (!in.wrapped(end) || !in.u8(v) || v != 0) {
            delete c;
            return fail("the resolver did not accept anonymous reads");
        }
    } else {  // ServerHelloWrite
        size_t e2;
        uint32_t ex, auth;
        uint64_t ttl;
        if (!in.wrapped(end) || !in.be(ttl, 8) || !in.u8(ex) || !in.wrapped(e2) || !in.u8(auth) ||
            auth != 0) {
            delete c;
            return fail("the resolver did not accept an anonymous publisher");
        }
        c->ttl = ttl;
    }
    return c;
}
}  // namespace

extern "C" {

NxgResolver* nxg_resolver_start(const char* ipv4, uint16_t port, uint16_t* bound_port,
                                uint64_t writer_ttl_secs, NetidxError* err) {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(port);
    if (!ipv4 || inet_pton(AF_INET, ipv4, &a.sin_addr) != 1) {
        rerr(err, "bad IPv4 address");
        return nullptr;
    }
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    const int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    socklen_t al = sizeof a;
    if (fd < 0 || bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0 || listen(fd, 64) != 0 ||
        getsockname(fd, reinterpret_cast<sockaddr*>(&a), &al) != 0) {
        rerr(err, "resolver listen: %s", strerror(errno));
        if (fd >= 0) close(fd);
        return nullptr;
    }
    NxgResolver* r = new NxgResolver();
    r->lfd = fd;
    r->self.ip = ntohl(a.sin_addr.s_addr);
    r->self.port = ntohs(a.sin_port);
    r->ttl = writer_ttl_secs;
    if (bound_port) *bound_port = r->self.port;
    r->acceptor = std::thread([r] {
        while (!r->stop) {
            const int c = accept(r->lfd, nullptr, nullptr);
            if (c < 0) {
                if (errno == EINTR) continue;
                break;  // the listener was shut down
            }
            const int one = 1;
            setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
            std::lock_guard<std::mutex> g(r->mu);
            r->reap();
            r->conns.emplace_back();
            NxgResolver::Conn* cn = &r->conns.back();
            cn->fd = c;
            cn->t = std::thread([r, cn, c] {
                r->serve(c);
                std::lock_guard<std::mutex> g2(r->mu);
                shutdown(c, SHUT_RDWR);
                close(c);
                cn->fd = -1;
                cn->done = true;
            });
        }
    });
    return r;
}

void nxg_resolver_stop(NxgResolver* r) {
    if (!r) return;
    r->stop = true;
    shutdown(r->lfd, SHUT_RDWR);
    close(r->lfd);
    if (r->acceptor.joinable()) r->acceptor.join();
    std::list<NxgResolver::Conn> cs;
    {
        std::lock_guard<std::mutex> g(r->mu);
        for (auto& c : r->conns)
            if (c.fd >= 0) shutdown(c.fd, SHUT_RDWR);  // each thread closes its own socket
        cs.splice(cs.end(), r->conns);
    }
    for (auto& c : cs)
        if (c.t.joinable()) c.t.join();
    delete r;
}

uint64_t nxg_resolver_n_published(NxgResolver* r) {
    if (!r) return 0;
    std::lock_guard<std::mutex> g(r->mu);
    return r->published.size();
}

NxgResolverClient* nxg_resolver_connect_write(const char* ipv4, uint16_t port,
                                              uint32_t write_ipv4, uint16_t write_port,
                                              uint64_t* ttl_out, NetidxError* err) {
    // ClientHello::WriteOnly(ClientHelloWrite { write_addr, auth: Anonymous, priority: Normal })
    Out f;
    put_addr(f, Addr4{write_ipv4, write_port});
    f.bytes(unit(0).data(), 2);
    f.bytes(unit(1).data(), 2);
    NxgResolverClient* c = client_hello(ipv4, port, wrap(1, wrap_struct(f.b)), true, err);
    if (c && ttl_out) *ttl_out = c->ttl;
    return c;
}

NxgResolverClient* nxg_resolver_connect_read(const char* ipv4, uint16_t port, NetidxError* err) {
    // ClientHello::ReadOnly(AuthRead::Anonymous)
    return client_hello(ipv4, port, wrap(0, unit(0)), false, err);
}

void nxg_resolver_client_close(NxgResolverClient* c) {
    if (!c) return;
    close(c->fd);
    delete c;
}

bool nxg_resolver_publish(NxgResolverClient* c, const char* path, uint64_t path_len,
                          NetidxError* err) {
    if (!c || !c->write || (!path && path_len)) {
        rerr(err, "bad argument");
        return false;
    }
    Out f;
    f.var(path_len);
    f.bytes(path, path_len);
    std::vector<uint8_t> m;
    if (!send_frame(c->fd, wrap(0, f.b)) || !recv_frame(c->fd, m)) {  // ToWrite::Publish
        rerr(err, "publish: connection lost");
        return false;
    }
    In in(m.data(), m.size());
    size_t end;
    uint32_t v;
    if (!in.wrapped(end) || !in.u8(v) || v != 0) {  // FromWrite::Published
        rerr(err, "publish: the resolver refused the path");
        return false;
    }
    return true;
}

bool nxg_resolver_resolve(NxgResolverClient* c, const char* path, uint64_t path_len,
                          NxgResolved* out, NetidxError* err) {
    if (!c || c->write || !out || (!path && path_len)) {
        rerr(err, "bad argument");
        return false;
    }
    memset(out, 0, sizeof *out);
    Out f;
    f.var(path_len);
    f.bytes(path, path_len);
    std::vector<uint8_t> m;
    if (!send_frame(c->fd, wrap(0, f.b)) || !recv_frame(c->fd, m)) {  // ToRead::Resolve
        rerr(err, "resolve: connection lost");
        return false;
    }
    struct P {
        uint64_t id;
        Addr4 addr;
    };
    std::vector<P> described;
    In in(m.data(), m.size());
    while (in.left()) {
        size_t end, e2;
        uint32_t v;
        if (!in.wrapped(end) || !in.u8(v) || !in.wrapped(e2)) break;
        if (v == 0) {  // FromRead::Publisher
            Addr4 res, addr;
            uint64_t id;
            if (!get_addr(in, res) || !in.var(id) || !get_addr(in, addr)) break;
            described.push_back(P{id, addr});
        } else if (v == 1) {  // FromRead::Resolved
            Addr4 res;
            uint64_t n, ts, flags, perm;
            if (!get_addr(in, res) || !in.var(n)) break;
            std::vector<uint64_t> ids;
            for (uint64_t k = 0; k < n; k++) {
                size_t e3;
                uint64_t id;
                if (!in.wrapped(e3) || !in.var(id)) return rerr(err, "resolve: bad reply"), false;
                ids.push_back(id);
                in.i = e3;
            }
            if (!in.be(ts, 8) || !in.be(flags, 4) || !in.be(perm, 4)) break;
            out->resolver_ipv4 = res.ip;
            out->resolver_port = res.port;
            out->n_publishers = (uint32_t)ids.size();
            out->timestamp = ts;
            out->flags = (uint32_t)flags;
            out->permissions = (uint32_t)perm;
            for (const P& p : described)
                if (!ids.empty() && p.id == ids[0]) {
                    out->publisher_id = p.id;
                    out->publisher_ipv4 = p.addr.ip;
                    out->publisher_port = p.addr.port;
                }
            return true;
        } else {  // Denied / Error / Referral: not resolvable here
            rerr(err, "resolve: the resolver answered with FromRead variant %u", v);
            return false;
        }
        in.i = end;
    }
    rerr(err, "resolve: bad reply");
    return false;
}

}  // extern "C"
