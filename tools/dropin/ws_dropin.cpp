// tools/dropin/ws_dropin.cpp -- the north star's drop-in check: a flashws
// echo server written against the reference's OWN, unchanged API (FLoop +
// WSServerSocket<false>, compiled from /root/reference/include by
// oracle/Makefile `dropin`, output in oracle/_ref/), whose receive decode goes
// to the MI355X with one added line, fws_amd::GpuRxHook::Enable (--gpu), and a
// load client on the reference's WSClientSocket<false>.
//
// server: the shape of tests/new-ws-echo's server (test_ws_server.cpp:185-241):
//   each on_read data part is appended to the connection's message buffer and
//   at msg_end the message is written back as one frame of its opcode
//   (WriteFrame, ws_server_socket.h:131-141); PONG parts are ignored. Prints
//   "listening <port>", then one JSON line when --conns connections closed:
//   messages echoed, the on_close (code, reason) log, GPU reads.
//   --commands (tests only): a message whose payload starts with "cmd:" is a
//   command -- "cmd:sleep:<ms>" (echoed; the loop's end-of-step callback then
//   sleeps, so the next step collects every read sent meanwhile),
//   "cmd:close-peers" (echoed; Close(1000, "peer") on every other connection),
//   "cmd:shutwr" (not echoed; shutdown(SHUT_WR) of this connection's TCP socket),
//   "cmd:noecho..." (counted, not echoed).
// --tls (both modes): wss:// -- WSServerSocket<true> / WSClientSocket<true> over
//   the reference's TLSSocket and SSLManager (server: --cert / --key files, no
//   peer verification); the server's hook is then fws_amd::GpuRxHookTls, which
//   decodes the reads OpenSSL decrypted.
// client: --clients connections in one FLoop, each sends --msgs messages of
//   --msg-len bytes (window 1, a PING every --ping-every messages), checks every
//   echoed byte against what it sent, then Close(1000, "bye"). One JSON line:
//   goodput (rx + tx, test_ws_client.cpp:79-80), RTT quantiles, verified.
//
// Test / measurement infrastructure: it compiles the reference's headers, so it
// is built only where /root/reference exists and lives in oracle/_ref/.
#include "flashws/flashws.h"
#include "flashws/net/floop.h"
#include "flashws/net/ws_client_socket.h"
#include "flashws/net/ws_server_socket.h"

#include "flashws_amd/gpu_floop.hpp"

#include <arpa/inet.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_set>
#include <vector>

namespace {

using Loop = fws::FLoop<fws::FlashAllocator<char>>;
using Clock = std::chrono::steady_clock;

struct Opts {
    std::string mode;
    bool tls = false;
    std::string cert, key;
    int port = 0;
    bool gpu = false;
    bool gpu_batch = false;             // --gpu-batch: GpuRxHook::EnableBatched
    int persistent = -1;                // --persistent N: the context's resident decode grid (N workgroups,
                                        //   0 = a launch per read; default: GpuContext's)
    int device = 0;
    int conns = 1;
    int clients = 1;
    size_t msg_len = 4096;
    size_t msgs = 1000;
    size_t warmup = 50;
    size_t ping_every = 0;
    int max_seconds = 60;
    bool commands = false;
};

[[noreturn]] void die(const char *what) {
    std::fprintf(stderr, "ws_dropin: %s (%s)\n", what, std::string(fws::GetErrorStrV()).c_str());
    std::exit(2);
}

// ------------------------------------------------------------------ server
constexpr size_t kHead = fws::constants::SUGGEST_RESERVE_WS_HDR_SIZE;

struct ConnCtx {
    fws::IOBuffer msg;
    uint32_t opcode;
};

struct Server {
    Opts o;
    Loop loop;
    uint64_t msgs = 0, bytes = 0;
    int closes = 0;
    std::vector<std::pair<uint32_t, std::string>> close_log;
    std::unordered_set<void *> live;   // user data constructed by on_new_connection
    std::vector<void *> socks;         // open WS sockets (--commands: close-peers)
    int sleep_ms = 0;                  // --commands: sleep at the end of this step

    static fws::IOBuffer NewMsg(size_t cap) {
        fws::IOBuffer b = fws::RequestBuf(kHead + cap);
        b.start_pos = kHead;
        b.size = 0;
        return b;
    }
};

template <bool kTls>
int RunServer(const Opts &o) {
    using WS = fws::WSServerSocket<kTls>;
    static Server srv;                         // reached from captureless-size lambdas
    srv.o = o;
    if (srv.loop.template Init<kTls>() < 0) die("FLoop::Init");
    if constexpr (kTls) {
        if (fws::SSLManager::instance().Init(false, o.cert.c_str(), o.key.c_str(), nullptr) < 0) die("SSLManager::Init");
    }
    WS ws{};
    if (ws.Init() < 0) die("WSServerSocket::Init");
    Server *S = &srv;
    ws.SetOnNewConnection([S](WS &w, std::string_view, std::string_view, std::string_view, std::string_view,
                              std::string_view, std::string_view &, std::string_view &, void *ud) {
        new (ud) ConnCtx{Server::NewMsg(1u << 16), 2u};
        S->live.insert(ud);
        S->socks.push_back(&w);
        return 0;
    });
    ws.SetOnRead([S](WS &s, uint32_t opcode, fws::IOBuffer &&part, bool, bool is_msg_end, bool is_ctl, void *ud) {
        if (is_ctl) return;                    // PONG parts: nothing to echo
        auto &c = *static_cast<ConnCtx *>(ud);
        const size_t need = size_t(c.msg.size) + size_t(part.size);
        if (kHead + need > c.msg.capacity) {   // grow the message buffer
            fws::IOBuffer big = Server::NewMsg(std::max(need, 2 * (c.msg.capacity - kHead)));
            std::memcpy(big.data + kHead, c.msg.data + c.msg.start_pos, size_t(c.msg.size));
            big.size = c.msg.size;
            c.msg = std::move(big);
        }
        std::memcpy(c.msg.data + c.msg.start_pos + c.msg.size, part.data + part.start_pos, size_t(part.size));
        c.msg.size += part.size;
        c.opcode = opcode;
        if (is_msg_end) {
            ++S->msgs;
            S->bytes += uint64_t(c.msg.size);
            const std::string_view m{reinterpret_cast<const char *>(c.msg.data + c.msg.start_pos), size_t(c.msg.size)};
            const bool cmd = S->o.commands && m.substr(0, 4) == "cmd:";
            bool echo = true;
            std::vector<WS *> peers;
            if (cmd && m.substr(4, 6) == "sleep:") S->sleep_ms = std::atoi(std::string(m.substr(10)).c_str());
            if (cmd && m.substr(4) == "close-peers")
                for (void *p : S->socks) if (p != &s) peers.push_back(static_cast<WS *>(p));
            if (cmd && m.substr(4) == "shutwr") {
                if constexpr (!kTls) s.under_socket().Shutdown(fws::TCPSocket::SHUT_WR_MODE);   // ws:// only
                echo = false;
            }
            if (cmd && m.substr(4, 6) == "noecho") echo = false;
            if (echo && s.WriteFrame(std::move(c.msg), fws::WSTxFrameType(c.opcode), true) < 0) die("WriteFrame");
            c.msg = Server::NewMsg(1u << 16);
            for (WS *p : peers) p->Close(fws::WS_NORMAL_CLOSE, "peer");
        }
    });
    ws.SetOnClose([S](WS &w, uint32_t code, std::string_view reason, void *ud) {
        S->socks.erase(std::remove(S->socks.begin(), S->socks.end(), static_cast<void *>(&w)), S->socks.end());
        S->close_log.emplace_back(code, std::string(reason));
        if (S->live.erase(ud)) std::destroy_at(static_cast<ConnCtx *>(ud));
        if (++S->closes >= S->o.conns) S->loop.StopRun();
    });

    if (o.commands) {
        // the application's end-of-step callback (the batched hook chains to it)
        srv.loop.SetOnEventFunc([S](Loop &) {
            if (S->sleep_ms > 0) {
                ::usleep(useconds_t(S->sleep_ms) * 1000u);
                S->sleep_ms = 0;
            }
        });
    }
    std::unique_ptr<fws_amd::GpuContext> gpu;
    std::unique_ptr<fws_amd::GpuRxHookT<kTls>> hook;
    if (o.gpu) {
        gpu = std::make_unique<fws_amd::GpuContext>(o.device);
        if (o.persistent >= 0) gpu->SetPersistent(uint32_t(o.persistent));
        hook = std::make_unique<fws_amd::GpuRxHookT<kTls>>(*gpu);
        if (o.gpu_batch) hook->EnableBatched(ws, srv.loop);   // (or: every read of a loop step in one GPU batch)
        else hook->Enable(ws);                 // the one added line
    }

    if (ws.StartListen("127.0.0.1", uint16_t(o.port), 128, fws::TCPSocket::REUSE_ADDR_MODE) < 0) die("listen");
    sockaddr_in a{};
    socklen_t al = sizeof(a);
    ::getsockname(ws.under_socket().fd(), reinterpret_cast<sockaddr *>(&a), &al);
    auto [add_ret, sp] = srv.loop.AddSocket(std::move(ws), sizeof(ConnCtx), true);
    (void)sp;
    if (add_ret < 0) die("AddSocket");
    std::printf("listening %d\n", int(ntohs(a.sin_port)));
    std::fflush(stdout);
    ::alarm(unsigned(o.max_seconds));
    srv.loop.Run();

    std::string log = "[";
    for (size_t i = 0; i < srv.close_log.size(); ++i) {
        std::string r;
        for (unsigned char ch : srv.close_log[i].second) {
            char hx[8];
            std::snprintf(hx, sizeof(hx), "%02x", ch);
            r += hx;
        }
        log += (i ? ", " : "") + std::string("[") + std::to_string(srv.close_log[i].first) + ", \"" + r + "\"]";
    }
    log += "]";
    if (hook && std::getenv("FWS_HOOK_PROF")) {
        const auto &pf = hook->step_prof();
        std::printf("{\"hook_prof\": {\"steps\": %llu, \"flushes\": %llu, \"reads\": %llu, \"loop_us\": %.1f, "
                    "\"mux_us\": %.1f, \"dispatch_us\": %.1f, \"step_end_us\": %.1f}}\n",
                    (unsigned long long)pf.steps, (unsigned long long)pf.flushes, (unsigned long long)pf.reads, pf.loop_us,
                    pf.mux_us, pf.dispatch_us, pf.step_end_us);
    }
    std::printf("{\"mode\": \"server\", \"tls\": %s, \"gpu\": %s, \"msgs\": %llu, \"bytes\": %llu, \"closes\": %d, "
                "\"close_log_hex\": %s, \"gpu_reads\": %llu, \"gpu_batches\": %llu, \"zc_slots\": %llu, \"deferred_chunks\": %llu}\n",
                kTls ? "true" : "false", o.gpu ? "true" : "false", (unsigned long long)srv.msgs, (unsigned long long)srv.bytes, srv.closes,
                log.c_str(), (unsigned long long)(hook ? hook->gpu_reads() : 0),
                (unsigned long long)(hook ? hook->gpu_batches() : 0),
                (unsigned long long)(hook ? hook->zero_copy_slots() : 0),
                (unsigned long long)(hook ? hook->deferred_chunks() : 0));
    std::fflush(stdout);
    if constexpr (kTls) std::_Exit(0);        // see RunClient: no static TLS teardown
    return 0;
}

// ------------------------------------------------------------------ client
struct CliCtx {
    int id = 0;
    size_t sent = 0, recvd = 0;
    std::vector<uint8_t> acc;
    Clock::time_point t_send;
    bool ping_out = false;
};

struct Client {
    Opts o;
    Loop loop;
    std::vector<uint8_t> pool;
    std::vector<uint32_t> rtt_ns;
    uint64_t rx = 0, tx = 0, pongs = 0;
    bool ok = true;
    int open = 0, closed = 0;
    Clock::time_point t0, t1;
    bool started = false;

    const uint8_t *payload(int id, size_t i) const { return pool.data() + ((i * 131 + size_t(id) * 977) % 4096); }
};

template <bool kTls>
int RunClient(const Opts &o) {
    using WC = fws::WSClientSocket<kTls>;
    static Client cli;
    cli.o = o;
    cli.pool.resize(o.msg_len + 4096);
    uint64_t x = 0x2545F4914F6CDD1Dull;
    for (auto &b : cli.pool) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; b = uint8_t(x >> 32); }
    if (cli.loop.template Init<kTls>() < 0) die("FLoop::Init");
    if constexpr (kTls) {
        if (fws::SSLManager::instance().Init(false, nullptr, nullptr, nullptr) < 0) die("SSLManager::Init");
    }
    Client *C = &cli;
    auto send_msg = [](Client *C, WC &w, CliCtx &c) {
        if (C->o.ping_every && c.sent % C->o.ping_every == C->o.ping_every - 1) {
            fws::IOBuffer p = fws::RequestBuf(kHead + 8);
            p.start_pos = kHead;
            std::memcpy(p.data + kHead, "ping1234", 8);
            p.size = 8;
            if (w.WriteFrame(std::move(p), fws::WS_PING_FRAME, true) < 0) die("WriteFrame ping");
        }
        fws::IOBuffer b = fws::RequestBuf(kHead + C->o.msg_len);
        b.start_pos = kHead;
        std::memcpy(b.data + kHead, C->payload(c.id, c.sent), C->o.msg_len);
        b.size = ssize_t(C->o.msg_len);
        if (c.sent == C->o.warmup && !C->started) { C->started = true; C->t0 = Clock::now(); }
        c.t_send = Clock::now();
        if (w.WriteFrame(std::move(b), fws::WS_BIN_FRAME, true) < 0) die("WriteFrame");
        ++c.sent;
    };
    for (int k = 0; k < o.clients; ++k) {
        WC w{};
        if (w.Init() < 0) die("WSClientSocket::Init");
        if (w.Connect("127.0.0.1", uint16_t(o.port), "/", "127.0.0.1") < 0 && errno != EINPROGRESS) die("Connect");
        w.SetOnOpen([C, send_msg](WC &w, std::string_view, std::string_view, void *ud) {
            ++C->open;
            send_msg(C, w, *static_cast<CliCtx *>(ud));
        });
        w.SetOnRead([C, send_msg](WC &w, uint32_t opcode, fws::IOBuffer &&part, bool, bool is_msg_end, bool is_ctl,
                                  void *ud) {
            auto &c = *static_cast<CliCtx *>(ud);
            if (is_ctl) {
                if (opcode == fws::WS_OPCODE_PONG) {
                    ++C->pongs;
                    if (part.size != 8 || std::memcmp(part.data + part.start_pos, "ping1234", 8) != 0) C->ok = false;
                }
                return;
            }
            c.acc.insert(c.acc.end(), part.data + part.start_pos, part.data + part.start_pos + part.size);
            if (!is_msg_end) return;
            const auto now = Clock::now();
            if (opcode != fws::WS_OPCODE_BIN || c.acc.size() != C->o.msg_len ||
                std::memcmp(c.acc.data(), C->payload(c.id, c.recvd), C->o.msg_len) != 0)
                C->ok = false;
            if (c.recvd >= C->o.warmup) {
                C->rtt_ns.push_back(uint32_t(std::min<int64_t>(
                    std::chrono::duration_cast<std::chrono::nanoseconds>(now - c.t_send).count(), UINT32_MAX)));
                C->rx += c.acc.size();
                C->tx += C->o.msg_len;
            }
            c.acc.clear();
            ++c.recvd;
            if (c.recvd < C->o.warmup + C->o.msgs) {
                send_msg(C, w, c);
            } else {
                C->t1 = now;
                w.Close(fws::WS_NORMAL_CLOSE, "bye");
            }
        });
        w.SetOnClose([C](WC &, uint32_t, std::string_view, void *) {
            if (++C->closed >= C->o.clients) C->loop.StopRun();
        });
        CliCtx ctx;
        ctx.id = k;
        auto [r, sp] = cli.loop.AddSocket(std::move(w), sizeof(CliCtx), false, std::move(ctx));
        (void)sp;
        if (r < 0) die("AddSocket");
    }
    ::alarm(unsigned(o.max_seconds));
    cli.loop.Run();
    auto &v = cli.rtt_ns;
    std::sort(v.begin(), v.end());
    auto q = [&](double p) { return v.empty() ? 0.0 : v[std::min(v.size() - 1, size_t(p * double(v.size() - 1) + 0.5))] / 1e3; };
    const double secs = std::max(std::chrono::duration<double>(cli.t1 - cli.t0).count(), 1e-9);
    const bool complete = v.size() == size_t(o.clients) * o.msgs;
    std::printf("{\"mode\": \"client\", \"clients\": %d, \"msg_len\": %zu, \"msgs_per_client\": %zu, "
                "\"seconds\": %.4f, \"goodput_rx_tx_mbps\": %.1f, \"msgs_per_s\": %.0f, "
                "\"rtt_us\": {\"p50\": %.2f, \"p99\": %.2f, \"max\": %.2f}, \"pongs\": %llu, \"verified\": %s}\n",
                o.clients, o.msg_len, o.msgs, secs, double(cli.rx + cli.tx) * 8.0 / secs / 1e6,
                double(v.size()) / secs, q(0.5), q(0.99), q(1.0), (unsigned long long)cli.pongs,
                (cli.ok && complete) ? "true" : "false");
    std::fflush(stdout);
    const int rc = (cli.ok && complete) ? 0 : 1;
    // the reference's TLS objects crash in static teardown at exit (with and
    // without the GPU hook): a wss process leaves without running destructors
    if constexpr (kTls) std::_Exit(rc);
    return rc;
}

}  // namespace

int main(int argc, char **argv) {
    Opts o;
    if (argc < 2) die("usage: ws_dropin server|client [options]");
    o.mode = argv[1];
    for (int i = 2; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> std::string { if (i + 1 >= argc) die("missing value"); return argv[++i]; };
        if (a == "--port") o.port = std::atoi(next().c_str());
        else if (a == "--tls") o.tls = true;
        else if (a == "--cert") o.cert = next();
        else if (a == "--key") o.key = next();
        else if (a == "--gpu") o.gpu = true;
        else if (a == "--gpu-batch") o.gpu = o.gpu_batch = true;
        else if (a == "--device") o.device = std::atoi(next().c_str());
        else if (a == "--persistent") o.persistent = std::atoi(next().c_str());
        else if (a == "--conns") o.conns = std::atoi(next().c_str());
        else if (a == "--clients") o.clients = std::atoi(next().c_str());
        else if (a == "--msg-len") o.msg_len = std::strtoull(next().c_str(), nullptr, 10);
        else if (a == "--msgs") o.msgs = std::strtoull(next().c_str(), nullptr, 10);
        else if (a == "--warmup") o.warmup = std::strtoull(next().c_str(), nullptr, 10);
        else if (a == "--ping-every") o.ping_every = std::strtoull(next().c_str(), nullptr, 10);
        else if (a == "--max-seconds") o.max_seconds = std::atoi(next().c_str());
        else if (a == "--commands") o.commands = true;
        else die(("unknown option " + a).c_str());
    }
    if (o.mode == "server") return o.tls ? RunServer<true>(o) : RunServer<false>(o);
    if (o.mode == "client") return o.tls ? RunClient<true>(o) : RunClient<false>(o);
    die("mode must be server or client");
}
