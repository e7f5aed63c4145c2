// tools/ws_echo.cpp -- loopback WebSocket echo over POSIX TCP (BASELINE C1 and
// the north star's host-memory end-to-end rate), with the server's receive
// path on the GPU (fws_rx_session_feed: H2D, fused header parse + unmask, D2H,
// OnRecvData's part replay) or on the real reference's OnRecvData
// (oracle/_ref/libfwsref.so, dlopen'ed; bench.py's CPU-baseline leg only).
//
// Shape of the reference's tests/new-ws-echo harness:
//  * client (test_ws_client.cpp:100-125, 187-280): sends a masked BIN message,
//    waits for the echo, measures the round trip and (rx + tx) goodput;
//  * server (test_ws_server.cpp:185-240): copies each on_read part into the
//    connection's message buffer and, at msg_end, writes it back as one
//    unmasked server frame of the message's opcode;
//  * reads of at most MAX_READABLE_SIZE_ONE_TIME = 2 MiB into a buffer at
//    start_pos 32 (constants.h:49-53, floop.h:664-665), one epoll loop thread
//    (FLoop, one loop per thread).
// Differences, stated: one process (server thread + one thread per client),
// `--window W` messages in flight per client (W = 1 is the reference's
// ping-pong), and every echoed payload is compared with what was sent.
//
// Output: one JSON line on stdout (goodput, msg/s, RTT quantiles, verified).
#include <arpa/inet.h>
#include <fcntl.h>
#include <dlfcn.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "fws_gpu.h"

namespace {

constexpr size_t kReadMax = 2u << 20;   // MAX_READABLE_SIZE_ONE_TIME (constants.h:49-53)
constexpr size_t kPad = 32;             // DEFAULT_READ_BUF_PRE_PADDING_SIZE

using Clock = std::chrono::steady_clock;

struct Opts {
    std::string engine = "gpu";
    std::string ref_lib;
    int clients = 1;
    size_t msg_len = 4096;
    size_t msgs = 20000;        // per client, timed
    size_t warmup = 200;        // per client, before the timed messages (connection setup, first launches)
    int window = 1;
    int port = 0;
    int device = 0;
};

[[noreturn]] void die(const char *what, long v = 0) {
    std::fprintf(stderr, "ws_echo: %s (%ld, errno %d %s)\n", what, v, errno, std::strerror(errno));
    std::exit(2);
}

// ---- server engines: one OnRecvData per read, events in the 48-B layout both
// ---- fws_rx_event (include/fws_gpu.h) and the reference driver's RefEvent use.
struct Engine {
    virtual ~Engine() = default;
    virtual void *open_conn() = 0;                      // per-connection session
    virtual uint8_t *read_buf(void *conn) = 0;          // where the read lands (start_pos 32)
    virtual int feed(void *conn, size_t n, std::vector<fws_rx_event> &ev, uint64_t *n_ev) = 0;
    // the reads of every readable connection of one loop iteration at once
    // (fws_rx_mux); engines without it feed one read at a time
    virtual bool batched() const { return false; }
    virtual int feed_batch(void *const *conns, const size_t *n, uint32_t k, fws_rx_read_result *out) {
        (void)conns; (void)n; (void)k; (void)out;
        return -1;
    }
};

struct GpuConn {
    fws_rx_session *s = nullptr;
    uint8_t *mem = nullptr;
    std::vector<uint8_t> ctl;
};

struct GpuEngine : Engine {
    fws_gpu_ctx *ctx = nullptr;
    std::vector<std::unique_ptr<GpuConn>> conns;
    explicit GpuEngine(int device) {
        if (int r = fws_gpu_ctx_create(device, &ctx)) die("fws_gpu_ctx_create", r);
    }
    ~GpuEngine() override {
        for (auto &c : conns) {
            fws_rx_session_destroy(c->s);
            fws_gpu_host_unregister(c->mem);
            std::free(c->mem);
        }
        fws_gpu_ctx_destroy(ctx);
    }
    void *open_conn() override {
        auto c = std::make_unique<GpuConn>();
        if (int r = fws_rx_session_create(ctx, 1, &c->s)) die("fws_rx_session_create", r);
        c->mem = static_cast<uint8_t *>(std::aligned_alloc(4096, kPad + kReadMax + 4096));
        if (int r = fws_gpu_host_register(c->mem, kPad + kReadMax + 4096)) die("fws_gpu_host_register", r);
        c->ctl.resize(kReadMax + 256);
        conns.push_back(std::move(c));
        return conns.back().get();
    }
    uint8_t *read_buf(void *conn) override { return static_cast<GpuConn *>(conn)->mem + kPad; }
    int feed(void *conn, size_t n, std::vector<fws_rx_event> &ev, uint64_t *n_ev) override {
        auto *c = static_cast<GpuConn *>(conn);
        uint64_t used = 0;
        return fws_rx_session_feed(c->s, c->mem + kPad, n, n, ev.data(), ev.size(), n_ev, c->ctl.data(),
                                   c->ctl.size(), &used);
    }
};

// all connections in one fws_rx_mux: the reads of one epoll_wait round are
// decoded with one H2D copy, one launch and one D2H copy
struct MuxEngine : Engine {
    static constexpr uint32_t kSlots = 1024;
    fws_gpu_ctx *ctx = nullptr;
    fws_rx_mux *mux = nullptr;
    struct Conn {
        uint32_t slot;
        uint8_t *mem;
    };
    std::vector<std::unique_ptr<Conn>> conns;
    std::vector<fws_rx_read> reads;
    explicit MuxEngine(int device) {
        if (int r = fws_gpu_ctx_create(device, &ctx)) die("fws_gpu_ctx_create", r);
        if (int r = fws_rx_mux_create(ctx, kSlots, &mux)) die("fws_rx_mux_create", r);
    }
    ~MuxEngine() override {
        fws_rx_mux_destroy(mux);
        for (auto &c : conns) std::free(c->mem);
        fws_gpu_ctx_destroy(ctx);
    }
    void *open_conn() override {
        if (conns.size() >= kSlots) die("mux slots");
        auto c = std::make_unique<Conn>();
        c->slot = (uint32_t)conns.size();
        c->mem = static_cast<uint8_t *>(std::aligned_alloc(4096, kPad + kReadMax + 4096));
        conns.push_back(std::move(c));
        return conns.back().get();
    }
    uint8_t *read_buf(void *conn) override { return static_cast<Conn *>(conn)->mem + kPad; }
    int feed(void *conn, size_t n, std::vector<fws_rx_event> &ev, uint64_t *n_ev) override {
        fws_rx_read_result o;
        void *cs[1] = {conn};
        size_t ns[1] = {n};
        if (int r = feed_batch(cs, ns, 1, &o)) return r;
        *n_ev = std::min<uint64_t>(o.n_events, ev.size());
        std::memcpy(ev.data(), o.events, *n_ev * sizeof(fws_rx_event));
        return o.ret;
    }
    bool batched() const override { return true; }
    int feed_batch(void *const *cs, const size_t *n, uint32_t k, fws_rx_read_result *out) override {
        reads.resize(k);
        for (uint32_t i = 0; i < k; ++i) {
            auto *c = static_cast<Conn *>(cs[i]);
            reads[i] = fws_rx_read{c->slot, 0u, c->mem + kPad, n[i], n[i]};
        }
        return fws_rx_mux_feed(mux, reads.data(), k, out);
    }
};

struct RefEngine : Engine {
    void *lib = nullptr;
    void *(*new_)(void) = nullptr;
    uint8_t *(*buf_)(void *, size_t) = nullptr;
    int (*feed_)(void *, size_t, void *, size_t, size_t *) = nullptr;
    explicit RefEngine(const std::string &path) {
        lib = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (!lib) die(dlerror());
        new_ = reinterpret_cast<void *(*)(void)>(dlsym(lib, "ref_session_new"));
        buf_ = reinterpret_cast<uint8_t *(*)(void *, size_t)>(dlsym(lib, "ref_session_read_buf"));
        feed_ = reinterpret_cast<int (*)(void *, size_t, void *, size_t, size_t *)>(
            dlsym(lib, "ref_session_feed_inplace"));
        if (!new_ || !buf_ || !feed_) die("reference driver lacks the echo entry points");
    }
    void *open_conn() override {
        void *h = new_();
        if (!h) die("ref_session_new");
        buf_(h, kReadMax);
        return h;
    }
    uint8_t *read_buf(void *conn) override { return buf_(conn, kReadMax); }
    int feed(void *conn, size_t n, std::vector<fws_rx_event> &ev, uint64_t *n_ev) override {
        size_t k = 0;
        const int r = feed_(conn, n, ev.data(), ev.size(), &k);
        *n_ev = k;
        return r;
    }
};

// ---- server: one epoll loop thread ----
struct SrvConn {
    int fd = -1;
    void *eng = nullptr;
    std::vector<uint8_t> msg;       // the connection's message buffer (test_ws_server.cpp:203-206)
    uint32_t opcode = 2;
};

size_t server_hdr(uint8_t *h, uint32_t opcode, uint64_t len) {   // SendFrame, server side (w_socket.h:832-944)
    h[0] = uint8_t(0x80u | opcode);
    if (len < 126) { h[1] = uint8_t(len); return 2; }
    if (len < 65536) { h[1] = 126; h[2] = uint8_t(len >> 8); h[3] = uint8_t(len); return 4; }
    h[1] = 127;
    for (int i = 0; i < 8; ++i) h[2 + i] = uint8_t(len >> (56 - 8 * i));
    return 10;
}

void write_all(int fd, const iovec *iov_in, int n) {
    iovec iov[2];
    std::memcpy(iov, iov_in, sizeof(iovec) * n);
    int i = 0;
    while (i < n) {
        ssize_t w = ::writev(fd, iov + i, n - i);
        if (w < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN) { pollfd p{fd, POLLOUT, 0}; ::poll(&p, 1, 1000); continue; }
            die("server writev");
        }
        while (i < n && size_t(w) >= iov[i].iov_len) { w -= ssize_t(iov[i].iov_len); ++i; }
        if (i < n) { iov[i].iov_base = static_cast<uint8_t *>(iov[i].iov_base) + w; iov[i].iov_len -= size_t(w); }
    }
}

struct ServerStats {
    uint64_t reads = 0, read_bytes = 0, feed_ns = 0, batches = 0;
    int err = 0;
};

void server_loop(int lfd, int n_clients, Engine &eng, std::atomic<bool> &stop, ServerStats &st) {
    int ep = ::epoll_create1(0);
    epoll_event lev{};
    lev.events = EPOLLIN;
    lev.data.ptr = nullptr;
    ::epoll_ctl(ep, EPOLL_CTL_ADD, lfd, &lev);
    std::vector<std::unique_ptr<SrvConn>> conns;
    std::vector<fws_rx_event> ev(kReadMax / 3 + 64);
    std::vector<SrvConn *> ready;
    std::vector<void *> ready_eng;
    std::vector<size_t> ready_n;
    std::vector<fws_rx_read_result> results;
    // the server's on_read (test_ws_server.cpp:203-230): append each data part,
    // write the message back at msg_end
    auto echo = [&](SrvConn *c, const uint8_t *buf, const fws_rx_event *evp, uint64_t n_ev) {
        for (uint64_t j = 0; j < n_ev; ++j) {
            const fws_rx_event &e = evp[j];
            if (e.kind != 0 || e.is_ctl) continue;
            c->msg.insert(c->msg.end(), buf + e.data_off, buf + e.data_off + e.size);
            c->opcode = e.opcode;
            if (e.msg_end) {
                uint8_t h[10];
                iovec iov[2] = {{h, server_hdr(h, c->opcode, c->msg.size())}, {c->msg.data(), c->msg.size()}};
                write_all(c->fd, iov, c->msg.empty() ? 1 : 2);
                c->msg.clear();
            }
        }
    };
    epoll_event evs[1024];
    while (!stop.load(std::memory_order_relaxed)) {
        int k = ::epoll_wait(ep, evs, 1024, 20);
        for (int i = 0; i < k; ++i) {
            if (evs[i].data.ptr == nullptr) {
                int fd = ::accept(lfd, nullptr, nullptr);
                if (fd < 0) continue;
                int one = 1, big = 8 << 20;
                ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
                ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
                ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
                auto c = std::make_unique<SrvConn>();
                c->fd = fd;
                c->eng = eng.open_conn();
                epoll_event e{};
                e.events = EPOLLIN;
                e.data.ptr = c.get();
                ::epoll_ctl(ep, EPOLL_CTL_ADD, fd, &e);
                conns.push_back(std::move(c));
                continue;
            }
            auto *c = static_cast<SrvConn *>(evs[i].data.ptr);
            uint8_t *buf = eng.read_buf(c->eng);
            ssize_t r = ::recv(c->fd, buf, kReadMax, MSG_DONTWAIT);
            if (r <= 0) {
                if (r < 0 && (errno == EAGAIN || errno == EINTR)) continue;
                ::epoll_ctl(ep, EPOLL_CTL_DEL, c->fd, nullptr);
                continue;
            }
            ++st.reads;
            st.read_bytes += uint64_t(r);
            if (eng.batched()) {                   // decoded below with this round's other reads
                ready.push_back(c);
                ready_n.push_back(size_t(r));
                continue;
            }
            uint64_t n_ev = 0;
            const auto t0 = Clock::now();
            const int ret = eng.feed(c->eng, size_t(r), ev, &n_ev);
            st.feed_ns += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count());
            if (ret != 0) { st.err = ret; stop = true; break; }
            echo(c, buf, ev.data(), n_ev);
        }
        if (!ready.empty()) {
            ready_eng.clear();
            for (SrvConn *c : ready) ready_eng.push_back(c->eng);
            results.resize(ready.size());
            const auto t0 = Clock::now();
            const int rc = eng.feed_batch(ready_eng.data(), ready_n.data(), (uint32_t)ready.size(), results.data());
            st.feed_ns += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count());
            ++st.batches;
            if (rc != 0) { st.err = rc; stop = true; }
            for (size_t j = 0; j < ready.size() && rc == 0; ++j) {
                if (results[j].ret != 0) { st.err = results[j].ret; stop = true; break; }
                echo(ready[j], eng.read_buf(ready[j]->eng), results[j].events, results[j].n_events);
            }
            ready.clear();
            ready_n.clear();
        }
    }
    for (auto &c : conns) ::close(c->fd);
    ::close(ep);
    (void)n_clients;
}

// ---- client: nonblocking poll loop, `window` masked messages in flight ----
struct ClientResult {
    std::vector<uint32_t> rtt_ns;
    uint64_t tx = 0, rx = 0;
    bool ok = true;
    double t_first = 0, t_last = 0;   // seconds since the common epoch
};

void client_run(int port, const Opts &o, int id, Clock::time_point epoch, ClientResult &res) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(uint16_t(port));
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    int one = 1, big = 8 << 20;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
    ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
    if (::connect(fd, reinterpret_cast<sockaddr *>(&a), sizeof(a)) != 0) die("connect");
    const size_t L = o.msg_len;
    // payload pool: message i is pool[(i * 61) % 4096 ...], distinct per message and client
    std::vector<uint8_t> pool(L + 4096 * 8);
    uint64_t x = 0x9E3779B97F4A7C15ull * uint64_t(id + 1);
    for (auto &b : pool) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; b = uint8_t(x >> 24); }
    auto payload = [&](size_t i) { return pool.data() + ((i * 61u) % 4096u) * 8u; };
    const size_t hdr = L < 126 ? 6 : (L < 65536 ? 8 : 14);
    std::deque<Clock::time_point> sent_at;
    std::vector<uint8_t> out;
    size_t out_off = 0, n_sent = 0, n_recv = 0;
    std::vector<uint8_t> in(kReadMax * 2);
    size_t in_len = 0;
    res.rtt_ns.reserve(o.msgs);
    auto queue_msg = [&]() {
        const size_t base = out.size();
        out.resize(base + hdr + L);
        uint8_t *f = out.data() + base;
        f[0] = 0x82;                                     // FIN | BIN
        if (hdr == 6) f[1] = uint8_t(0x80 | L);
        else if (hdr == 8) { f[1] = 0x80 | 126; f[2] = uint8_t(L >> 8); f[3] = uint8_t(L); }
        else { f[1] = 0x80 | 127; for (int i = 0; i < 8; ++i) f[2 + i] = uint8_t(uint64_t(L) >> (56 - 8 * i)); }
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const uint32_t key = uint32_t(x);
        std::memcpy(f + hdr - 4, &key, 4);
        const uint8_t *p = payload(n_sent);
        uint8_t *d = f + hdr;
        const uint64_t k64 = (uint64_t(key) << 32) | key;   // client masking, ws_mask.h:15-29
        size_t i = 0;
        for (; i + 8 <= L; i += 8) { uint64_t w; std::memcpy(&w, p + i, 8); w ^= k64; std::memcpy(d + i, &w, 8); }
        for (; i < L; ++i) d[i] = p[i] ^ uint8_t(key >> (8 * (i & 3)));
        sent_at.push_back(Clock::now());
        if (n_sent == o.warmup) res.t_first = std::chrono::duration<double>(sent_at.back() - epoch).count();
        if (n_sent >= o.warmup) res.tx += L;
        ++n_sent;
    };
    ::fcntl(fd, F_SETFL, ::fcntl(fd, F_GETFL) | O_NONBLOCK);
    const size_t total = o.warmup + o.msgs;
    while (n_recv < total) {
        while (n_sent < total && n_sent - n_recv < size_t(o.window)) queue_msg();
        pollfd p{fd, short(POLLIN | (out_off < out.size() ? POLLOUT : 0)), 0};
        if (::poll(&p, 1, 5000) <= 0) { res.ok = false; break; }
        if ((p.revents & POLLOUT) && out_off < out.size()) {
            ssize_t w = ::send(fd, out.data() + out_off, out.size() - out_off, MSG_NOSIGNAL);
            if (w > 0) out_off += size_t(w);
            if (out_off == out.size()) { out.clear(); out_off = 0; }
        }
        if (p.revents & (POLLIN | POLLHUP | POLLERR)) {
            if (in_len == in.size()) in.resize(in.size() * 2);
            ssize_t r = ::recv(fd, in.data() + in_len, in.size() - in_len, 0);
            if (r == 0 || (r < 0 && errno != EAGAIN && errno != EINTR)) { res.ok = false; break; }
            if (r > 0) in_len += size_t(r);
            size_t pos = 0;
            for (;;) {   // server frames: unmasked, 2 / 4 / 10-B headers
                if (in_len - pos < 2) break;
                const uint8_t *h = in.data() + pos;
                uint64_t len = h[1] & 127u;
                size_t hl = 2;
                if (len == 126) { if (in_len - pos < 4) break; len = (uint64_t(h[2]) << 8) | h[3]; hl = 4; }
                else if (len == 127) {
                    if (in_len - pos < 10) break;
                    len = 0;
                    for (int i = 0; i < 8; ++i) len = (len << 8) | h[2 + i];
                    hl = 10;
                }
                if (in_len - pos < hl + len) break;
                const auto now = Clock::now();
                if (n_recv >= o.warmup) {
                    res.rtt_ns.push_back(uint32_t(std::min<int64_t>(
                        std::chrono::duration_cast<std::chrono::nanoseconds>(now - sent_at.front()).count(),
                        UINT32_MAX)));
                    res.rx += len;
                }
                sent_at.pop_front();
                if (len != L || h[0] != 0x82 || std::memcmp(h + hl, payload(n_recv), L) != 0) res.ok = false;
                ++n_recv;
                pos += hl + len;
                if (n_recv == total) res.t_last = std::chrono::duration<double>(now - epoch).count();
            }
            if (pos) { std::memmove(in.data(), in.data() + pos, in_len - pos); in_len -= pos; }
        }
    }
    if (n_recv < total) res.ok = false;
    ::close(fd);
}

double quantile(std::vector<uint32_t> &v, double q) {
    if (v.empty()) return 0;
    size_t i = std::min(v.size() - 1, size_t(q * double(v.size() - 1) + 0.5));
    return v[i] / 1000.0;
}

}  // namespace

int main(int argc, char **argv) {
    Opts o;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> std::string { if (i + 1 >= argc) die("missing value"); return argv[++i]; };
        if (a == "--engine") o.engine = next();
        else if (a == "--ref-lib") o.ref_lib = next();
        else if (a == "--clients") o.clients = std::atoi(next().c_str());
        else if (a == "--msg-len") o.msg_len = std::strtoull(next().c_str(), nullptr, 10);
        else if (a == "--msgs") o.msgs = std::strtoull(next().c_str(), nullptr, 10);
        else if (a == "--warmup") o.warmup = std::strtoull(next().c_str(), nullptr, 10);
        else if (a == "--window") o.window = std::atoi(next().c_str());
        else if (a == "--port") o.port = std::atoi(next().c_str());
        else if (a == "--device") o.device = std::atoi(next().c_str());
        else die(("unknown option " + a).c_str());
    }
    if (o.clients < 1 || o.window < 1 || o.msg_len == 0 || o.msg_len > (1u << 20) || o.msgs == 0) die("bad options");

    std::unique_ptr<Engine> eng;
    if (o.engine == "gpu") eng = std::make_unique<GpuEngine>(o.device);
    else if (o.engine == "gpu-mux") eng = std::make_unique<MuxEngine>(o.device);
    else if (o.engine == "ref") eng = std::make_unique<RefEngine>(o.ref_lib);
    else die("engine must be gpu, gpu-mux or ref");

    int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(uint16_t(o.port));
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (::bind(lfd, reinterpret_cast<sockaddr *>(&a), sizeof(a)) != 0) die("bind");
    if (::listen(lfd, 128) != 0) die("listen");
    socklen_t al = sizeof(a);
    ::getsockname(lfd, reinterpret_cast<sockaddr *>(&a), &al);
    const int port = ntohs(a.sin_port);

    std::atomic<bool> stop{false};
    ServerStats st;
    std::thread srv(server_loop, lfd, o.clients, std::ref(*eng), std::ref(stop), std::ref(st));
    const auto epoch = Clock::now();
    std::vector<ClientResult> res(o.clients);
    std::vector<std::thread> cl;
    for (int c = 0; c < o.clients; ++c) cl.emplace_back(client_run, port, std::cref(o), c, epoch, std::ref(res[c]));
    for (auto &t : cl) t.join();
    stop = true;
    srv.join();
    ::close(lfd);

    std::vector<uint32_t> rtt;
    uint64_t tx = 0, rx = 0;
    bool ok = st.err == 0;
    double t0 = 1e30, t1 = 0;
    for (auto &r : res) {
        rtt.insert(rtt.end(), r.rtt_ns.begin(), r.rtt_ns.end());
        tx += r.tx;
        rx += r.rx;
        ok = ok && r.ok;
        t0 = std::min(t0, r.t_first);
        t1 = std::max(t1, r.t_last);
    }
    std::sort(rtt.begin(), rtt.end());
    const double secs = std::max(t1 - t0, 1e-9);
    const double goodput_mbps = double(rx + tx) * 8.0 / secs / 1e6;   // test_ws_client.cpp:79-80
    std::printf("{\"engine\": \"%s\", \"clients\": %d, \"msg_len\": %zu, \"window\": %d, \"msgs_per_client\": %zu, \"warmup_per_client\": %zu, "
                "\"seconds\": %.4f, \"goodput_rx_tx_mbps\": %.1f, \"payload_GiB_per_s\": %.3f, \"msgs_per_s\": %.0f, "
                "\"rtt_us\": {\"min\": %.2f, \"p50\": %.2f, \"p99\": %.2f, \"p999\": %.2f, \"max\": %.2f}, "
                "\"server_reads\": %llu, \"server_bytes_per_read\": %.0f, \"server_feed_us_per_read\": %.2f, "
                "\"server_reads_per_batch\": %.2f, \"verified\": %s, \"server_ret\": %d}\n",
                o.engine.c_str(), o.clients, o.msg_len, o.window, o.msgs, o.warmup, secs, goodput_mbps,
                double(rx) / secs / double(1ull << 30), double(rtt.size()) / secs, quantile(rtt, 0), quantile(rtt, 0.5),
                quantile(rtt, 0.99), quantile(rtt, 0.999), quantile(rtt, 1.0), (unsigned long long)st.reads,
                st.reads ? double(st.read_bytes) / double(st.reads) : 0.0,
                st.reads ? double(st.feed_ns) / double(st.reads) / 1000.0 : 0.0,
                st.batches ? double(st.reads) / double(st.batches) : 1.0, ok ? "true" : "false", st.err);
    return ok ? 0 : 1;
}
