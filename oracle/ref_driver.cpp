// oracle/ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Thin extern "C" shim that drives the REAL flashws reference (header-only,
// compiled from /root/reference/include by oracle/Makefile into
// oracle/_ref/libfwsref.so). Used in this container to generate tests/golden/
// fixtures, and on the GPU box as the "reference" CPU baseline in bench.py.
// No reference source is copied: this file only instantiates the reference's
// own classes and functions.
//
// Drives the hot path exactly like the transport read lambda
// (ws_server_socket.h:171-197): WSocket::OnRecvData(IOBuffer&) on a
// WSServerSocket<false> whose under-socket is one end of a socketpair, so
// control replies (PONG / CLOSE echo, w_socket.h:662-696) are real writes that
// we read back.
//
// flashws.h may be included in exactly one TU (SURVEY §0 finding 2): this one.

#include "flashws/flashws.h"

#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>
#include <fcntl.h>
#include <chrono>
#include <cstring>
#include <vector>

namespace {

struct RefEvent {          // layout == orc_event (oracle/fws_oracle.h)
    uint32_t kind;
    uint32_t opcode;
    uint8_t is_ctl;
    uint8_t frame_end;
    uint8_t msg_end;
    uint8_t fin;
    uint32_t key;
    uint64_t size;
    uint64_t data_off;
    uint64_t ctl_off;
    uint64_t capacity;
};
static_assert(sizeof(RefEvent) == 48, "event layout");

struct RefState {          // exported carried RX state (w_socket.h:223-245)
    int32_t recv_status;
    uint32_t last_rx_mask_key;
    uint64_t unread_pl_len;
    uint8_t last_rx_opcode;
    uint8_t last_rx_control_opcode;
    uint8_t last_rx_fin_flag;
    uint8_t is_rx_control_frame;
    uint32_t last_rx_hdr_part_len;
};

struct Probe : fws::WSServerSocket<false> {
    using Base = fws::WSServerSocket<false>;
    using Base::OnRecvData;
    using Base::InitWSPart;
    using Base::server_status_;
    using Base::recv_status_;
    using Base::unread_pl_len_;
    using Base::last_rx_mask_key_;
    using Base::last_rx_opcode_;
    using Base::last_rx_control_opcode_;
    using Base::last_rx_fin_flag_;
    using Base::is_rx_control_frame_;
    using Base::last_rx_hdr_part_len_;
};

struct Session {
    Probe sock;
    int peer_fd = -1;
    // recording sinks for the current feed
    std::vector<RefEvent> events;
    std::vector<uint8_t> ctl;
    size_t read_start = 0;     // IOBuffer::start_pos of the current read
    uint64_t bytes_seen = 0;   // used by the timing loop
    bool timing = false;       // timing mode: count bytes only, no recording
    bool echo = false;         // echo harness: record parts, no socketpair drain per part
    fws::IOBuffer *rbuf = nullptr;   // echo harness: the session's pool read buffer
};

// Parse server TX frames written to the socketpair (server frames are unmasked;
// control payloads are <= 125 B so the header is 2 B; w_socket.h:832-944).
void DrainPeer(Session &s) {
    uint8_t buf[65536];
    std::vector<uint8_t> acc;
    for (;;) {
        ssize_t r = ::read(s.peer_fd, buf, sizeof(buf));
        if (r <= 0) break;
        acc.insert(acc.end(), buf, buf + r);
    }
    size_t p = 0;
    while (p + 2 <= acc.size()) {
        uint8_t b0 = acc[p], b1 = acc[p + 1];
        size_t len = b1 & 127u, h = 2;
        if (len == 126) { len = (size_t(acc[p + 2]) << 8) | acc[p + 3]; h = 4; }
        RefEvent e{};
        e.opcode = b0 & 15u;
        e.kind = (e.opcode == 10u) ? 1u : (e.opcode == 8u ? 5u : 6u);  // 1 PONG sent, 5 CLOSE echo
        e.is_ctl = 1; e.frame_end = 1; e.msg_end = 1; e.fin = b0 >> 7;
        e.size = len;
        e.ctl_off = s.ctl.size();
        s.ctl.insert(s.ctl.end(), acc.begin() + p + h, acc.begin() + p + h + len);
        s.events.push_back(e);
        p += h + len;
    }
}

}  // namespace

extern "C" {

// ---- seam 1: crypto/ws_mask.h ----
void ref_ws_mask_fast(uint8_t *src, size_t n, uint32_t key) { fws::WSMaskBytesFast(src, n, key); }
void ref_ws_mask_bytes(uint8_t *src, size_t n, uint32_t key) { fws::WSMaskBytes(src, n, key); }
void ref_mask1(uint8_t *src, size_t n, uint32_t key) { fws::detail::Mask1(src, n, key); }
void ref_mask_avx2(uint8_t *src, size_t n, uint32_t key) { fws::MaskAVX2(src, n, key); }
void ref_mask_large_chunk_avx2(uint8_t *src, size_t n, uint32_t key) { fws::MaskLargeChunkAVX2(src, n, key); }
uint32_t ref_rotr32(uint32_t v, uint32_t b) { return fws::RotateR(v, b); }

// ---- seam 2: WSocket::OnRecvData (server) ----
void *ref_session_new(void) {
    auto *s = new Session();
    int sv[2];
    if (::socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) { delete s; return nullptr; }
    int big = 4 << 20;
    ::setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
    ::setsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
    ::fcntl(sv[1], F_SETFL, ::fcntl(sv[1], F_GETFL) | O_NONBLOCK);
    s->peer_fd = sv[1];
    // fq_ptr_ must be initialised (tcp_socket.h:51 leaves it indeterminate).
    s->sock.under_socket().Init(sv[0], true, fws::NORMAL_SOCKET_STATUS, nullptr,
                                /*nonblock=*/true, /*no_delay=*/false, /*busy_poll=*/false);
    s->sock.InitWSPart();
    s->sock.server_status_ = decltype(s->sock.server_status_)(3);   // OPEN_STATUS
    s->sock.SetOnRead([s](Probe::Base &, uint32_t opcode, fws::IOBuffer &&buf, bool frame_end,
                          bool msg_end, bool is_ctl, void *) {
        if (s->timing) { s->bytes_seen += (uint64_t)buf.size; return; }
        if (!s->echo) DrainPeer(*s);         // replies written before this delivery
        RefEvent e{};
        e.kind = 0; e.opcode = opcode; e.is_ctl = is_ctl;
        e.frame_end = frame_end; e.msg_end = msg_end;
        e.size = (uint64_t)buf.size;
        if (!is_ctl) {
            e.data_off = buf.start_pos - s->read_start;
            e.capacity = buf.capacity - s->read_start;
        } else {
            e.ctl_off = s->ctl.size();
            if (buf.data && buf.size > 0)
                s->ctl.insert(s->ctl.end(), buf.data + buf.start_pos, buf.data + buf.start_pos + buf.size);
        }
        s->bytes_seen += (uint64_t)buf.size;
        s->events.push_back(e);
    });
    s->sock.SetOnClose([s](Probe::Base &, uint32_t code, std::string_view reason, void *) {
        DrainPeer(*s);                       // the CLOSE echo precedes on_close (w_socket.h:691-706)
        RefEvent e{};
        e.kind = 2; e.opcode = 8; e.is_ctl = 1; e.frame_end = 1; e.msg_end = 1; e.fin = 1;
        e.key = code;
        e.size = reason.size();
        e.ctl_off = s->ctl.size();
        s->ctl.insert(s->ctl.end(), reason.begin(), reason.end());
        s->events.push_back(e);
    });
    return s;
}

void ref_session_free(void *h) {
    auto *s = static_cast<Session *>(h);
    if (!s) return;
    // The Probe object is intentionally leaked: destroying a WSServerSocket
    // that was never attached to an FLoop double-frees inside the reference
    // (observed here; not on the decode path). Close both fds and recycle nothing.
    s->sock.under_socket().Close();
    ::close(s->peer_fd);
    s->events.clear(); s->events.shrink_to_fit();
    s->ctl.clear(); s->ctl.shrink_to_fit();
}

// Feed one read. The bytes are placed in a pool IOBuffer at start_pos 32
// (DEFAULT_READ_BUF_PRE_PADDING_SIZE, tcp read path floop.h:664-665) and
// OnRecvData runs on it. out_buf receives the buffer after decode (in-place
// unmask). Returns OnRecvData's return code.
int ref_session_feed(void *h, const uint8_t *data, size_t n, uint8_t *out_buf, size_t extra_cap,
                     void *events, size_t ev_cap, size_t *n_ev,
                     uint8_t *ctl_out, size_t ctl_cap, size_t *ctl_used) {
    auto *s = static_cast<Session *>(h);
    s->events.clear();
    s->ctl.clear();
    const size_t pad = fws::constants::DEFAULT_READ_BUF_PRE_PADDING_SIZE;
    size_t cap = pad + n + extra_cap;
    fws::IOBuffer io = fws::RequestBuf(cap);
    io.start_pos = pad;
    io.size = (ssize_t)n;
    if (n) std::memcpy(io.data + pad, data, n);
    s->read_start = pad;
    int ret = s->sock.OnRecvData(io);
    DrainPeer(*s);
    if (out_buf && n) std::memcpy(out_buf, io.data + pad, n);
    *n_ev = s->events.size();
    std::memcpy(events, s->events.data(), sizeof(RefEvent) * std::min(ev_cap, s->events.size()));
    *ctl_used = s->ctl.size();
    std::memcpy(ctl_out, s->ctl.data(), std::min(ctl_cap, s->ctl.size()));
    return ret;
}

void ref_session_state(void *h, RefState *out) {
    auto *s = static_cast<Session *>(h);
    out->recv_status = (int32_t)s->sock.recv_status_;
    out->last_rx_mask_key = s->sock.last_rx_mask_key_;
    out->unread_pl_len = s->sock.unread_pl_len_;
    out->last_rx_opcode = s->sock.last_rx_opcode_;
    out->last_rx_control_opcode = s->sock.last_rx_control_opcode_;
    out->last_rx_fin_flag = s->sock.last_rx_fin_flag_;
    out->is_rx_control_frame = s->sock.is_rx_control_frame_;
    out->last_rx_hdr_part_len = s->sock.last_rx_hdr_part_len_;
}

// CPU baseline: `iters` passes of OnRecvData over `stream` delivered as reads of
// `read_size` bytes (<= MAX_READABLE_SIZE_ONE_TIME, constants.h:49-53), in
// place in one pool buffer (the XOR unmask is an involution, so an even pass
// count restores the input). Returns elapsed seconds; *payload_bytes receives
// the bytes delivered to on_read(). Per-read IOBuffer views and per-part
// callbacks are exactly the reference's.
double ref_time_onrecv(const uint8_t *stream, size_t n, size_t read_size, int iters,
                       uint64_t *payload_bytes, int *ret_code) {
    auto *s = static_cast<Session *>(ref_session_new());
    const size_t pad = fws::constants::DEFAULT_READ_BUF_PRE_PADDING_SIZE;
    fws::IOBuffer big = fws::RequestBuf(pad + n + 64);
    std::memcpy(big.data + pad, stream, n);
    s->bytes_seen = 0;
    s->timing = true;
    *ret_code = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; it < iters; ++it) {
        for (size_t off = 0; off < n; off += read_size) {
            size_t len = std::min(read_size, n - off);
            fws::IOBuffer view(big.data, (ssize_t)len, pad + off, pad + off + len);
            int r = s->sock.OnRecvData(view);
            if (r < 0) *ret_code = r;
        }
    }
    auto t1 = std::chrono::steady_clock::now();
    *payload_bytes = s->bytes_seen;
    ref_session_free(s);
    return std::chrono::duration<double>(t1 - t0).count();
}

// All-core CPU baseline: the reference's own scaling model is one event loop
// (one process, or one F-Stack lcore) per core (SURVEY §2 "Parallelism",
// floop.h:331-345), and its BufferManager / MemPoolEnv singletons are not
// thread-safe (buffer_manager.h:9-34, flash_alloc.h:437), so process p decodes stream[begin[p], end[p]) (a range starting at a frame
// header) in its own forked process exactly as ref_time_onrecv does (its own
// copy in a pool buffer, one untimed pass, then `iters` timed passes). The
// children start together (a pipe barrier) and time themselves; returns the
// slowest child's seconds, *payload_bytes = the sum. Call it before the process
// initialises a GPU (the children never touch one).
double ref_time_onrecv_procs(const uint8_t *stream, const uint64_t *begin, const uint64_t *end, int nproc,
                             size_t read_size, int iters, uint64_t *payload_bytes, int *ret_code) {
    struct Slot { double secs; uint64_t bytes; int ret; int done; };
    auto *slots = static_cast<Slot *>(::mmap(nullptr, sizeof(Slot) * (size_t)nproc, PROT_READ | PROT_WRITE,
                                             MAP_SHARED | MAP_ANONYMOUS, -1, 0));
    *payload_bytes = 0;
    *ret_code = 0;
    if (slots == MAP_FAILED) return -1.0;
    std::memset(slots, 0, sizeof(Slot) * (size_t)nproc);
    int ready[2], go[2];
    if (::pipe(ready) != 0 || ::pipe(go) != 0) return -1.0;
    std::vector<pid_t> kids;
    for (int p = 0; p < nproc; ++p) {
        const pid_t pid = ::fork();
        if (pid < 0) break;
        if (pid == 0) {
            ::close(ready[0]);
            ::close(go[1]);
            const uint8_t *src = stream + begin[p];
            const size_t n = (size_t)(end[p] - begin[p]);
            auto *s = static_cast<Session *>(ref_session_new());
            const size_t pad = fws::constants::DEFAULT_READ_BUF_PRE_PADDING_SIZE;
            fws::IOBuffer big = fws::RequestBuf(pad + n + 64);
            std::memcpy(big.data + pad, src, n);
            s->timing = true;
            int rc = 0;
            auto pass = [&]() {
                for (size_t off = 0; off < n; off += read_size) {
                    size_t len = std::min(read_size, n - off);
                    fws::IOBuffer view(big.data, (ssize_t)len, pad + off, pad + off + len);
                    int r = s->sock.OnRecvData(view);
                    if (r < 0) rc = r;
                }
            };
            pass();                                     // untimed: page faults of the copy
            char c = 1;
            if (::write(ready[1], &c, 1) != 1) ::_exit(3);
            if (::read(go[0], &c, 1) != 1) ::_exit(3);
            s->bytes_seen = 0;
            auto t0 = std::chrono::steady_clock::now();
            for (int it = 0; it < iters; ++it) pass();
            auto t1 = std::chrono::steady_clock::now();
            slots[p].secs = std::chrono::duration<double>(t1 - t0).count();
            slots[p].bytes = s->bytes_seen;
            slots[p].ret = rc;
            slots[p].done = 1;
            ::_exit(0);
        }
        kids.push_back(pid);
    }
    ::close(ready[1]);
    ::close(go[0]);
    char c;
    for (size_t i = 0; i < kids.size(); ++i)
        if (::read(ready[0], &c, 1) != 1) break;
    for (size_t i = 0; i < kids.size(); ++i) {
        c = 1;
        if (::write(go[1], &c, 1) != 1) break;
    }
    for (pid_t k : kids) ::waitpid(k, nullptr, 0);
    ::close(ready[0]);
    ::close(go[1]);
    double worst = 0.0;
    for (int p = 0; p < nproc; ++p) {
        if (!slots[p].done || p >= (int)kids.size()) { worst = -1.0; break; }
        worst = std::max(worst, slots[p].secs);
        *payload_bytes += slots[p].bytes;
        if (slots[p].ret < 0) *ret_code = slots[p].ret;
    }
    ::munmap(slots, sizeof(Slot) * (size_t)nproc);
    return worst;
}

// Echo harness (tools/ws_echo.cpp, run by bench.py's CPU-baseline leg): the
// session's own pool read buffer, RequestBuf(pad + cap) with reads landing at
// start_pos 32 as the transport puts them (floop.h:664-665), and OnRecvData on
// a view of it without a copy. Events as ref_session_feed's; control replies
// stay unread on the socketpair (the echo sends no control frames).
uint8_t *ref_session_read_buf(void *h, size_t cap) {
    auto *s = static_cast<Session *>(h);
    const size_t pad = fws::constants::DEFAULT_READ_BUF_PRE_PADDING_SIZE;
    if (!s->rbuf) s->rbuf = new fws::IOBuffer(fws::RequestBuf(pad + cap + 64));
    s->echo = true;
    return s->rbuf->data + pad;
}

int ref_session_feed_inplace(void *h, size_t n, void *events, size_t ev_cap, size_t *n_ev) {
    auto *s = static_cast<Session *>(h);
    const size_t pad = fws::constants::DEFAULT_READ_BUF_PRE_PADDING_SIZE;
    s->events.clear();
    s->ctl.clear();
    s->read_start = pad;
    fws::IOBuffer view(s->rbuf->data, (ssize_t)n, pad, pad + n);
    int ret = s->sock.OnRecvData(view);
    *n_ev = s->events.size();
    std::memcpy(events, s->events.data(), sizeof(RefEvent) * std::min(ev_cap, s->events.size()));
    return ret;
}

// WSMaskBytesFast alone over a list of (offset, len, key) parts of `buf`.
double ref_time_mask_parts(uint8_t *buf, const uint64_t *offs, const uint64_t *lens,
                           const uint32_t *keys, size_t n_parts, int iters) {
    auto t0 = std::chrono::steady_clock::now();
    for (int it = 0; it < iters; ++it)
        for (size_t i = 0; i < n_parts; ++i) fws::WSMaskBytesFast(buf + offs[i], lens[i], keys[i]);
    auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// ---- client TX: WSClientSocket::WriteFrame -> WSocket::SendFrame (w_socket.h:832-944)
// The under-socket is one end of a socketpair; the frame bytes SendFrame writes
// (header built backwards into the IOBuffer's headroom, payload masked with a
// SemiSecureRand32 key, w_socket.h:858-866) are read back from the other end.
struct TxProbe : fws::WSClientSocket<false> {
    using Base = fws::WSClientSocket<false>;
    using Base::InitWSPart;
};
struct TxSrvProbe : fws::WSServerSocket<false> {
    using Base = fws::WSServerSocket<false>;
    using Base::InitWSPart;
};

struct TxSession {
    bool server = false;
    TxProbe cli;
    TxSrvProbe srv;
    int peer_fd = -1;
};

void *ref_tx_new(int is_server) {
    auto *s = new TxSession();
    s->server = is_server != 0;
    int sv[2];
    if (::socketpair(AF_UNIX, SOCK_STREAM, 0, sv) != 0) { delete s; return nullptr; }
    int big = 8 << 20;
    ::setsockopt(sv[0], SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
    ::setsockopt(sv[1], SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
    s->peer_fd = sv[1];
    if (s->server) {
        s->srv.under_socket().Init(sv[0], true, fws::NORMAL_SOCKET_STATUS, nullptr, false, false, false);
        s->srv.InitWSPart();
    } else {
        s->cli.under_socket().Init(sv[0], true, fws::NORMAL_SOCKET_STATUS, nullptr, false, false, false);
        s->cli.InitWSPart();
    }
    return s;
}

void ref_tx_free(void *h) {
    auto *s = static_cast<TxSession *>(h);
    if (!s) return;
    if (s->server) s->srv.under_socket().Close(); else s->cli.under_socket().Close();
    ::close(s->peer_fd);                        // the probes are leaked, as ref_session_free does
}

// One WriteFrame(payload, frame_type, last_frame_if_possible) -> SendFrame
// (w_socket.h:832-944); the frame bytes go to out (*out_len). Returns its value.
long ref_tx_write(void *h, const uint8_t *payload, size_t n, uint32_t frame_type, int last_frame_if_possible,
                  uint8_t *out, size_t out_cap, size_t *out_len) {
    auto *s = static_cast<TxSession *>(h);
    const size_t head = fws::constants::MAX_WS_FRAME_HEADER_SIZE;
    fws::IOBuffer io = fws::RequestBuf(head + n + 16);
    io.start_pos = head;
    io.size = (ssize_t)n;
    if (n) std::memcpy(io.data + head, payload, n);
    const size_t expect = (s->server ? fws::GetTxWSFrameHdrSize<true>(n) : fws::GetTxWSFrameHdrSize<false>(n)) + n;
    long ret = s->server
        ? (long)s->srv.WriteFrame(std::move(io), fws::WSTxFrameType(frame_type), last_frame_if_possible != 0)
        : (long)s->cli.WriteFrame(std::move(io), fws::WSTxFrameType(frame_type), last_frame_if_possible != 0);
    size_t got = 0;
    while (ret >= 0 && got < expect && got < out_cap) {
        ssize_t r = ::read(s->peer_fd, out + got, std::min(out_cap - got, expect - got));
        if (r <= 0) break;
        got += (size_t)r;
    }
    *out_len = got;
    return ret;
}

size_t ref_tx_hdr_size(size_t payload, int is_server) {
    return is_server ? fws::GetTxWSFrameHdrSize<true>(payload) : fws::GetTxWSFrameHdrSize<false>(payload);
}

}  // extern "C"
