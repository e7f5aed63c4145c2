// flashws_amd/gpu_floop.hpp -- opt-in MI355X receive decode for an UNCHANGED
// flashws server: one call on the listening fws::WSServerSocket<false> (ws://,
// GpuRxHook) or fws::WSServerSocket<true> (wss://, GpuRxHookTls), no change to
// any flashws header and none to the application's on_read / WriteFrame /
// on_close code.
//
//   #include "flashws/flashws.h"              // the app's one flashws TU
//   #include "flashws_amd/gpu_floop.hpp"
//   fws_amd::GpuContext gpu(0);
//   fws_amd::GpuRxHook hook(gpu);
//   ws_socket.SetOnNewConnection(...); ws_socket.SetOnRead(...); ws_socket.SetOnClose(...);
//   hook.Enable(ws_socket);                    // <- the only added line
//   loop.AddSocket(std::move(ws_socket), sizeof(Ctx), true); loop.Run();
//
// How it attaches. FLoop copies the listening socket's on_new_connection /
// on_read / on_write / on_close into every accepted socket
// (floop.h:367-390). Enable() wraps the first and the last: when a
// connection's handshake completes (on_new_connection, ws_server_socket.h:
// 320-536) the wrapper re-installs that socket's under-socket readable
// callback -- the one WSServerSocket::InitUnderOnReadImp sets
// (ws_server_socket.h:171-197) -- with a callback of the same shape: in
// OPEN_STATUS each read goes through fws_amd::GpuRxDecoder (H2D, fused header
// parse + unmask on the GPU, D2H, OnRecvData's part bookkeeping on the host)
// instead of WSocket::OnRecvData (w_socket.h:543-769); every other status is
// handed to the reference's own callback (saved at Enable). The decoded events
// drive exactly the reference's code paths:
//   data / PONG part -> on_read()(sock, opcode, IOBuffer, frame_end, msg_end, is_ctl, &sock + 1)
//                                                              (w_socket.h:713-747)
//   PING             -> SendControlMsg(PONG)                   (w_socket.h:662-666)
//   CLOSE            -> OnRecvCloseFrame, SendControlMsg(CLOSE) echo, close_code_,
//                       on_close()(sock, code, reason, ...)    (w_socket.h:667-710)
//   error < 0        -> Close(WS_ABNORMAL_CLOSE, error text) and close the TCP
//                       socket                                 (ws_server_socket.h:176-194)
// The protected members are reached through using-declarations in a derived
// access struct and pointers to members (no reference file is edited). The
// wrapped on_close retires the connection's decoder (freed at the next read).
//
// Batched (ws:// and wss://): EnableBatched(listen, loop) makes
// every OPEN connection's read of one FLoop::OneStep wait in a pending list
// (the reference decodes it inside the read loop, floop.h:661-703) and sends
// the reads of many connections to the GPU in one fws_rx_mux round trip (one
// H2D or none, one launch or resident-grid request, one D2H). Chunks of
// SetChunk() reads (default 16) go out as they fill, from inside the step's
// read loop, through fws_rx_mux_submit / _complete: a chunk decodes while the
// loop reads the next sockets, and a completed chunk's events are dispatched
// while the following chunk decodes. The rest goes at the end of the step (the
// loop's on_event callback, floop.h:743, which the hook wraps and chains to the
// application's); its events are dispatched there, in read order -- or, while
// the loop has events waiting, in the next step (SetDeferLastChunk, the
// default since r06; see there). A connection
// with a second read in the same step (a full read buffer, floop.h:670-672) or
// whose previous read is still in flight, whose peer closes in the step
// (on_eof), or which the loop closes in the step (the EOF / error branch,
// floop.h:715-730 -> on_close) has everything pending decoded and dispatched
// first, so each connection sees its events in order and before its EOF /
// on_close. Per connection the callbacks are the per-read path's; only their
// timing moves (to a chunk boundary or the end of the step). A read of a
// connection that an earlier read's callbacks
// closed in the same step goes to the reference's own readable callback, as on
// the per-read path. A protocol error closes the connection as the reference
// does and removes it from the loop (DeleteFd, as floop.h:672-674 does after a
// read). More connections than mux slots fall back to the per-read decoder.
//
// Zero copy (default on): each read buffer the loop hands over is a MemPool
// slot (RequestBuf, buffer_manager.h:90-95 -> MemPool::allocate, flash_alloc.h:
// 137-244: a power-of-two slot inside a block the pool never frees); the hook
// registers every slot it sees once (fws_gpu_host_register) over the extent
// the pool's own metadata records for it (a buffer the pool does not know is
// staged, never registered on a guess), and the GPU then
// decodes the read where it lies -- no copy into pinned staging and back
// (rx_session.cpp: reads whose parts start on the 16-B chunk grid and need no
// staged header bytes). SetZeroCopy(false) keeps every read staged.
//
// wss:// (SURVEY §8f rank 4): the under-socket is the reference's TLSSocket,
// whose readable callback (tls_on_readable_, tls_socket.h:206-209) receives
// the reads OpenSSL has already decrypted on the CPU (SSL_read loop,
// tls_socket.h:472-562); the hook replaces that callback the same way, so the
// GPU decodes the plaintext WebSocket stream and TLS stays in OpenSSL.
#pragma once

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string_view>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "gpu_ws.hpp"

namespace fws_amd {
namespace detail {

struct TcpAccess : fws::TCPSocket {
    using fws::TCPSocket::on_readable_;
};

struct TlsAccess : fws::TLSSocket {
    using fws::TLSSocket::tls_on_readable_;
    using fws::TLSSocket::tls_on_eof_;
};

struct TcpEofAccess : fws::TCPSocket {
    using fws::TCPSocket::on_eof_;
};

// the loop's end-of-OneStep callback (floop.h:743) and DeleteFd (floop.h:348)
template <class Loop>
struct LoopAccess : Loop {
    using Loop::on_event_;
    using Loop::DeleteFd;
    using Loop::fq_;
};

// the under-socket's readable callback member (the one InitUnderOnReadImp sets)
template <bool kTls> struct UnderAccess;
template <> struct UnderAccess<false> {
    using Sock = fws::TCPSocket;
    using Func = fws::TCPSocket::OnReadableFunc;
    using EofFunc = fws::TCPSocket::OnEofFunc;
    static constexpr auto member = &TcpAccess::on_readable_;
    static constexpr auto eof_member = &TcpEofAccess::on_eof_;
};
template <> struct UnderAccess<true> {
    using Sock = fws::TLSSocket;
    using Func = fws::TLSSocket::TLSOnReadbleFunc;
    using EofFunc = fws::TLSSocket::TLSOnEofFunc;   // (called from the base's on_eof, tls_socket.h:468)
    static constexpr auto member = &TlsAccess::tls_on_readable_;
    static constexpr auto eof_member = &TlsAccess::tls_on_eof_;
};

template <bool kTls>
struct WsServerAccess : fws::WSServerSocket<kTls> {
    using S = fws::WSServerSocket<kTls>;
    using S::server_status_;
    using S::on_read;
    using S::on_close;
    using S::on_new_connection;
    using S::SendControlMsg;
    using S::HasRecvClose;
    using S::HasSentClose;
    using S::OnRecvCloseFrame;
    using S::close_code_;
    using S::has_called_on_close_;
    using S::in_shutting_down_;
    static constexpr auto kOpen = S::OPEN_STATUS;
    static constexpr auto kClosed = S::CLOSED_STATUS;
    static constexpr size_t kCtlHdr = fws::constants::WS_SERVER_TX_CONTROL_HDR_SIZE;
};

}  // namespace detail

template <bool kTls>
class GpuRxHookT {
public:
    using Sock = fws::WSServerSocket<kTls>;
    using A = detail::WsServerAccess<kTls>;
    using U = detail::UnderAccess<kTls>;
    using USock = typename U::Sock;

    explicit GpuRxHookT(GpuContext &ctx) : ctx_(ctx) {}
    GpuRxHookT(const GpuRxHookT &) = delete;
    GpuRxHookT &operator=(const GpuRxHookT &) = delete;

    // Call on the listening socket after the application set its callbacks and
    // before connections are accepted. The hook must outlive the loop.
    void Enable(Sock &listen) {
        user_new_conn_ = (listen.*(&A::on_new_connection))();
        user_close_ = (listen.*(&A::on_close))();
        ref_readable_ = static_cast<USock &>(listen.under_socket()).*(U::member);
        GpuRxHookT *self = this;
        listen.SetOnNewConnection([self](Sock &w, std::string_view uri, std::string_view host,
                                         std::string_view origin, std::string_view sub, std::string_view ext,
                                         std::string_view &rsub, std::string_view &rext, void *ud) {
            const int r = self->user_new_conn_(w, uri, host, origin, sub, ext, rsub, rext, ud);
            if (r >= 0) self->Attach(w);
            return r;
        });
        listen.SetOnClose([self](Sock &w, uint32_t code, std::string_view reason, void *ud) {
            if (self->DispatchBeforeClose(w)) return;   // its own CLOSE frame closed it, as on the per-read path
            self->Retire(w);
            self->user_close_(w, code, reason, ud);
        });
    }

    // Batched decode of each loop step's reads (ws:// and wss://; see the
    // header). Call after any SetOnEventFunc of the application (the hook
    // chains to it).
    template <class Loop>
    void EnableBatched(Sock &listen, Loop &loop, uint32_t max_conns = 1024) {
        Enable(listen);
        if (fws_rx_mux_create(ctx_.get(), max_conns, &mux_) != 0) throw std::runtime_error("fws_rx_mux_create failed");
        for (uint32_t i = max_conns; i-- > 0;) free_slots_.push_back(i);
        using LA = detail::LoopAccess<Loop>;
        auto app_event = loop.*(&LA::on_event_);      // the application's (or the loop's no-op)
        Loop *lp = &loop;
        app_on_event_ = [app_event, lp]() mutable { app_event(*lp); };
        delete_fd_ = [lp](void *p) { (lp->*(&LA::DeleteFd))(p, false); };
        GpuRxHookT *self = this;
        prof_on_ = std::getenv("FWS_HOOK_PROF") != nullptr;
        if (const char *c = std::getenv("FWS_HOOK_CHUNK")) chunk_ = (uint32_t)std::strtoul(c, nullptr, 10);
        if (const char *c = std::getenv("FWS_HOOK_DEFER")) defer_ = std::strtoul(c, nullptr, 10) != 0;
#ifndef FWS_ENABLE_FSTACK
        // "does the loop have events waiting?": a zero-timeout wait on the loop's own
        // queue. epoll and poll are level-triggered here (fevent.h: no EPOLLET), so
        // the events it sees are reported again to the next OneStep.
        loop_ready_ = [lp]() {
            fws::FEvent ev[1];
            const timespec ts{0, 0};
            return fws::FEventWait(lp->*(&LA::fq_), nullptr, 0, ev, 1, &ts) > 0;
        };
#endif
        loop.SetOnEventFunc([self](Loop &) {
            if (self->prof_on_) self->ProfStep(true);
            self->StepEnd();
            self->DeleteDeferred();
            self->app_on_event_();
            if (self->prof_on_) self->ProfStep(false);
        });
    }

    ~GpuRxHookT() {
        if (mux_ && fl_active_) (void)CompleteInflight();   // (its reads' buffers go with pending state)
        if (mux_) fws_rx_mux_destroy(mux_);
        for (uint8_t *p : registered_) (void)fws_gpu_host_unregister(p);
    }

    // Register the read buffers for in-place decode (default), or not. Only
    // buffers the reference's MemPool allocated (RequestBuf) are registered, each
    // over the slot the pool recorded for it (PoolSlot); any other IOBuffer is
    // staged through pinned memory as with SetZeroCopy(false).
    void SetZeroCopy(bool on) { zero_copy_ = on; }

    // Batched path: the reads of a step go to the GPU in chunks of this many as
    // they arrive (each chunk's round trip overlaps the step's later reads and
    // the previous chunk's dispatch); 0 = one batch at the end of the step.
    // Default kDefaultChunk; env FWS_HOOK_CHUNK at EnableBatched.
    void SetChunk(uint32_t reads) { chunk_ = reads; }

    // Batched path, on by default (off: SetDeferLastChunk(false) or env
    // FWS_HOOK_DEFER=0 at EnableBatched): at the end of
    // a step the last chunk goes to the GPU and, while it decodes, the hook asks
    // the loop's queue for events (a zero-timeout wait); if some are waiting it
    // returns and the chunk's events are dispatched in the next step (at its
    // first full chunk, a read of one of its connections, or its end), so its
    // round trip overlaps that step's reads. With nothing waiting it polls the
    // chunk to completion and dispatches it at once, so a deferred chunk never
    // waits on a blocking epoll. Per connection the order of events is the
    // per-read path's; what moves is the step in which the last chunk's
    // callbacks run (after the application's end-of-step callback of the step
    // that read them). Not available on F-stack (the whole step is flushed).
    void SetDeferLastChunk(bool on) { defer_ = on; }
    bool defer_last_chunk() const { return defer_; }
    uint64_t deferred_chunks() const { return deferred_chunks_; }

    size_t connections() const { return conns_.size(); }
    uint64_t gpu_reads() const { return gpu_reads_; }
    uint64_t gpu_batches() const { return gpu_batches_; }
    size_t zero_copy_slots() const { return registered_.size(); }   // MemPool slots decoded in place

    // Step profile of the batched path (env FWS_HOOK_PROF set at EnableBatched;
    // tools): loop steps, flushes, reads, and the wall time of the loop's own
    // part of the steps (epoll + reads, between two end-of-step callbacks), of
    // the mux rounds and of the event dispatch (the application's callbacks).
    struct StepProf {
        uint64_t steps = 0, flushes = 0, reads = 0;
        double loop_us = 0, mux_us = 0, dispatch_us = 0, step_end_us = 0;
    };
    const StepProf &step_prof() const { return prof_; }

private:
    static constexpr uint32_t kNoSlot = 0xFFFFFFFFu;
    static constexpr uint32_t kDefaultChunk = 16;
    struct Conn {
        Sock *ws;
        std::unique_ptr<GpuRxDecoder<fws::IOBuffer>> dec;   // per-read path (no mux slot)
        uint32_t slot = kNoSlot;                           // batched path: fws_rx_mux slot
        bool pending = false;                              // a read of this step waits in pending_
        bool inflight = false;                             // a read of it is in the submitted batch
        typename U::EofFunc ref_eof;                       // the under-socket's own on_eof
    };
    struct Pending {
        USock *u;
        fws::IOBuffer buf;
        void *ud;
    };

    // Maps decoded events onto the reference's own members (see the header).
    struct Sink {
        Sock &s;
        void on_read(uint32_t op, fws::IOBuffer &&b, bool fe, bool me, bool ctl) {
            (s.*(&A::on_read))()(s, op, std::move(b), fe, me, ctl, &s + 1);
        }
        fws::IOBuffer control_buf(std::string_view p) {
            fws::IOBuffer b = fws::RequestBuf(std::max(fws::constants::WS_MAX_CONTROL_FRAME_SIZE,
                                                       A::kCtlHdr + p.size()));
            b.start_pos = A::kCtlHdr;
            if (!p.empty()) std::memcpy(b.data + b.start_pos, p.data(), p.size());
            b.size = (ssize_t)p.size();
            return b;
        }
        void on_ping(std::string_view p) { (s.*(&A::SendControlMsg))(control_buf(p), fws::WS_PONG_FRAME); }
        void on_close(uint32_t code, std::string_view p) {
            const std::string_view reason = p.size() >= 2 ? p.substr(2) : std::string_view{};
            if (!(s.*(&A::HasRecvClose))()) {
                if ((s.*(&A::OnRecvCloseFrame))() < 0) return;
            }
            if (!(s.*(&A::HasSentClose))()) (s.*(&A::SendControlMsg))(control_buf(p), fws::WS_CLOSE_FRAME);
            s.*(&A::close_code_) = static_cast<fws::WSStatusCode>(code);
            if (!(s.*(&A::has_called_on_close_))) {
                s.*(&A::has_called_on_close_) = true;
                (s.*(&A::on_close))()(s, code, reason, &s + 1);
            }
        }
        fws::IOBuffer request_buf(size_t n) {
            fws::IOBuffer b = fws::RequestBuf(std::max(fws::constants::WS_MAX_CONTROL_FRAME_SIZE, A::kCtlHdr + n));
            b.start_pos = A::kCtlHdr;
            return b;
        }
    };

    void Attach(Sock &w) {
        auto &c = conns_[&w.under_socket()];
        c.ws = &w;
        if (c.slot != kNoSlot) free_slots_.push_back(c.slot);   // a stale entry at a reused address
        c.slot = kNoSlot;
        c.dec.reset();
        c.pending = false;
        if (mux_ && !free_slots_.empty() && fws_rx_mux_reset(mux_, free_slots_.back()) == 0) {
            c.slot = free_slots_.back();
            free_slots_.pop_back();
        } else {
            c.dec = std::make_unique<GpuRxDecoder<fws::IOBuffer>>(ctx_);
        }
        GpuRxHookT *self = this;
        w.under_socket().SetOnReadable([self](USock &u, fws::IOBuffer &&buf, void *ud) {
            self->OnReadable(u, std::move(buf), ud);
        });
        if (c.slot != kNoSlot) {
            auto &eof = static_cast<USock &>(w.under_socket()).*(U::eof_member);
            c.ref_eof = eof;
            eof = [self](USock &t, void *ud) { self->OnEof(t, ud); };
        }
    }

    // The wrapped on_close. A read of this connection still pending in the step
    // is decoded and dispatched first: the reference has already delivered it
    // inside the read loop (floop.h:661-703) when the same step's EOF / error
    // branch closes the socket (floop.h:715-730: DeleteFd(true) -> Close ->
    // on_close), so on_read comes before on_close as there. That flush runs
    // inside the loop's DeleteFd: it neither closes this socket again nor
    // removes any socket from the loop then (DeleteDeferred does, at the end of
    // the step; a DeleteFd nested in DeleteFd could move the map entry the outer
    // call still holds).
    //
    // The socket can close before a read it already handed over is dispatched:
    // the TLS socket closes on the peer's close_notify or an SSL error right
    // after delivering the read (tls_socket.h:507-559), the loop's error branch
    // on a reset, and a batched read waits for its chunk (or, deferred, for the
    // next step). The reference decodes that read before the close, so a CLOSE
    // frame in it reaches on_close with its own code and reason and the
    // under-socket's close then finds on_close called (w_socket.h:407-414).
    // The wrapped on_close therefore dispatches such reads first with
    // has_called_on_close_ cleared; if they called on_close (a CLOSE frame),
    // that was the connection's on_close and the under-socket's 1006 one is
    // dropped, else the flag is restored and the close goes on as before.
    bool DispatchBeforeClose(Sock &w) {
        auto it = conns_.find(&w.under_socket());
        if (it == conns_.end() || retiring_ != nullptr || !(it->second.pending || it->second.inflight)) return false;
        w.*(&A::has_called_on_close_) = false;
        retiring_ = static_cast<USock *>(&w.under_socket());
        Flush();
        retiring_ = nullptr;
        if (w.*(&A::has_called_on_close_)) return true;   // on_close ran (and retired the connection)
        w.*(&A::has_called_on_close_) = true;
        return false;
    }

    void Retire(Sock &w) {
        auto it = conns_.find(&w.under_socket());
        if (it == conns_.end()) return;
        if ((it->second.pending || it->second.inflight) && retiring_ == nullptr) {
            retiring_ = static_cast<USock *>(&w.under_socket());
            Flush();
            retiring_ = nullptr;
            it = conns_.find(&w.under_socket());
            if (it == conns_.end()) return;
        }
        if (it->second.dec) retired_.push_back(std::move(it->second.dec));   // may be mid-dispatch: freed at the next read
        if (it->second.slot != kNoSlot) free_slots_.push_back(it->second.slot);
        conns_.erase(it);
    }

    // The peer closed (floop.h:678-690): this connection's pending read is
    // decoded first, then the under-socket's own on_eof runs.
    void OnEof(USock &t, void *ud) {
        auto it = conns_.find(&t);
        if (it == conns_.end()) return;              // retired: its socket is being torn down
        typename U::EofFunc ref = it->second.ref_eof;
        if (it->second.pending || it->second.inflight) Flush();
        if (ref) ref(t, ud);
    }

    // A batch of reads on its way through the mux: submitted (fws_rx_mux_submit),
    // then completed (results) and dispatched.
    struct Batch {
        std::vector<Pending> items;
        std::vector<fws_rx_read> reads;
        std::vector<uint32_t> idx;                   // reads[k] -> items index
        std::vector<fws_rx_read_result> res;
        int rc = 0;
    };

    // pending_ -> the submitted batch (none may be in flight)
    void SubmitPending() {
        if (pending_.empty()) return;
        Batch &b = fl_;
        b = Batch{};
        b.items.swap(pending_);
        b.reads.reserve(b.items.size());
        for (uint32_t i = 0; i < b.items.size(); ++i) {
            auto it = conns_.find(b.items[i].u);
            if (it == conns_.end()) continue;
            it->second.pending = false;
            it->second.inflight = true;
            fws::IOBuffer &buf = b.items[i].buf;
            b.reads.push_back(fws_rx_read{it->second.slot, 0u, buf.data + buf.start_pos, (uint64_t)buf.size,
                                          (uint64_t)(buf.capacity - buf.start_pos)});
            b.idx.push_back(i);
        }
        const auto t0 = prof_on_ ? Clock::now() : Clock::time_point{};
        b.rc = b.reads.empty() ? 0 : fws_rx_mux_submit(mux_, b.reads.data(), (uint32_t)b.reads.size());
        if (prof_on_) prof_.mux_us += std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
        if (!b.reads.empty()) ++gpu_batches_;
        fl_active_ = true;
    }

    // the submitted batch, waited for; no batch is in flight afterwards
    Batch CompleteInflight() {
        Batch b = std::move(fl_);
        fl_ = Batch{};
        fl_active_ = false;
        const auto t0 = prof_on_ ? Clock::now() : Clock::time_point{};
        b.res.resize(b.reads.size());
        if (!b.reads.empty() && b.rc == 0) b.rc = fws_rx_mux_complete(mux_, b.res.data());
        if (prof_on_) prof_.mux_us += std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
        for (uint32_t k = 0; k < b.reads.size(); ++k) {
            auto it = conns_.find(b.items[b.idx[k]].u);
            if (it != conns_.end()) it->second.inflight = false;
        }
        return b;
    }

    // A completed batch's events, read by read in read order (ws_server_socket.h:
    // 172-196 per read).
    void Dispatch(Batch &b) {
        const auto t0 = prof_on_ ? Clock::now() : Clock::time_point{};
        for (size_t k = 0; k < b.reads.size(); ++k) {
            Pending &p = b.items[b.idx[k]];
            auto it = conns_.find(p.u);               // an earlier read's callbacks may have closed it
            if (it == conns_.end()) continue;
            Sock &sock = *it->second.ws;
            // closed by an earlier read's callbacks (an application closing another
            // connection): the read goes to the reference's own callback, as on the
            // per-read path -- in a closing state it does not decode the bytes (the
            // mux has unmasked them in place), it closes the TCP socket
            // (ws_server_socket.h:187-194)
            if ((sock.*(&A::server_status_)) != A::kOpen) {
                if (p.u == retiring_) continue;      // inside its own Close already
                ref_readable_(*p.u, std::move(p.buf), p.ud);
                if (!p.u->is_open()) DeleteFd(p.u);
                continue;
            }
            ++gpu_reads_;
            const uint32_t slot = it->second.slot;
            int ret = b.rc;
            if (b.rc == 0) {
                ret = b.res[k].ret;
                Sink sink{sock};
                GpuRxDecoder<fws::IOBuffer>::DispatchEvents(p.buf, b.res[k].events, b.res[k].n_events, b.res[k].ctl,
                                                            sink);
            }
            Finish(sock, *p.u, ret, [&]() {
                uint32_t op = 0;
                (void)fws_rx_mux_error(mux_, slot, &op);
                return op;
            }, true);
        }
        if (prof_on_) {
            ++prof_.flushes;
            prof_.reads += b.reads.size();
            prof_.dispatch_us += std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
        }
    }

    // One step of the pipeline: the batch in flight completes, the pending reads
    // go to the GPU, and the completed batch's events are dispatched while they
    // decode. Connections of the two batches are disjoint (a connection's next
    // read waits until its previous one is dispatched), so each connection
    // still sees its events in read order.
    void Advance() {
        if (!fl_active_) {
            SubmitPending();
            return;
        }
        Batch c = CompleteInflight();
        SubmitPending();
        Dispatch(c);
    }

    // Every pending and in-flight read decoded and dispatched, in order.
    void Flush() {
        while (fl_active_ || !pending_.empty()) Advance();
    }

    // The end of a loop step: Flush, or (SetDeferLastChunk) the step's last
    // chunk submitted and left in flight while the loop has events waiting.
    void StepEnd() {
        if (!defer_ || !loop_ready_) {
            Flush();
            return;
        }
        if (!pending_.empty()) Advance();            // the chunk before it completes and dispatches first
        while (fl_active_) {
            const int rd = fws_rx_mux_ready(mux_);
            if (rd != 0) {                           // decoded (or an error, which complete reports)
                Batch c = CompleteInflight();
                Dispatch(c);
                return;
            }
            if (loop_ready_()) {                     // reads are waiting: the next step dispatches it
                ++deferred_chunks_;
                return;
            }
        }
    }

    // end-of-step callback entry (begin) and exit: the loop's own part of a step
    // is the time from one exit to the next entry
    void ProfStep(bool begin) {
        const auto now = Clock::now();
        if (begin) {
            if (prof_.steps) prof_.loop_us += std::chrono::duration<double, std::micro>(now - prof_t_).count();
            ++prof_.steps;
        } else {
            prof_.step_end_us += std::chrono::duration<double, std::micro>(now - prof_b_).count();
        }
        (begin ? prof_b_ : prof_t_) = now;
    }

    // After a read's events: a protocol error closes the connection with the
    // reference's reason; a closed or failed socket's TCP socket is closed
    // (ws_server_socket.h:176-194) and, on the batched path, removed from the
    // loop as the read loop does after a read (floop.h:672-674).
    template <class ErrOp>
    void Finish(Sock &sock, USock &u, int ret, ErrOp &&err_opcode, bool batched) {
        if (ret < 0) {
            SetErrorText(ret, err_opcode());
            const std::string_view e = fws::GetErrorStrV();
            const size_t max_len = fws::constants::WS_MAX_CONTROL_FRAME_SIZE - A::kCtlHdr - 2U;
            sock.Close(fws::WS_ABNORMAL_CLOSE, std::string_view{e.data(), std::min(e.size(), max_len)});
        }
        if (&u == retiring_) return;                  // closing already (Retire)
        if (ret < 0 || ((sock.*(&A::server_status_)) == A::kClosed && !(sock.*(&A::in_shutting_down_)))) {
            sock.under_socket().Close();
            if (batched) DeleteFd(&u);
        }
    }

    // Remove a closed socket from the loop as the read loop does after a read
    // (floop.h:672-674); inside Retire's flush, at the end of the step instead.
    void DeleteFd(USock *u) {
        if (!delete_fd_ || u == retiring_) return;
        if (retiring_) deferred_.push_back(u);
        else delete_fd_(static_cast<void *>(u));
    }
    void DeleteDeferred() {
        std::vector<USock *> d;
        d.swap(deferred_);
        for (USock *u : d) delete_fd_(static_cast<void *>(u));   // FLoop::DeleteFd: a no-op if gone
    }

    // The pool's own record of a live allocation (register only what is
    // proven to be a MemPool slot): MemPool::allocate records every allocation of
    // >= 1 KiB in mem_meta_map_ with its size class (flash_alloc.h:145-157, 201-212),
    // and the slot is power2 = 1 << log2 bytes of memory_buffers_[log2], which the
    // pool never frees (only deallocate's index stack changes, :286-321). A buffer
    // that is not in the map (not from RequestBuf, buffer_manager.h:90-95) is staged.
    struct PoolSlot : fws::MemPool {
        static bool Extent(const void *p, size_t &bytes) {
            fws::MemPool &pool = fws::MemPoolEnv::instance();
            const auto &meta = pool.*(&PoolSlot::mem_meta_map_);   // protected: via a pointer to member
            const auto it = meta.find(const_cast<void *>(p));
            if (it == meta.end() || it->second.log2 >= 48) return false;
            bytes = size_t(1) << it->second.log2;
            return true;
        }
    };

    // A read buffer's MemPool slot, registered once over its exact extent (the
    // pool never frees its blocks, so the registration stays valid and the range
    // never changes owner outside the pool).
    void EnsureRegistered(const fws::IOBuffer &b) {
        if (!zero_copy_ || !b.data || b.capacity < 4096) return;
        if (registered_.count(b.data) || unregistrable_.count(b.data)) return;
        size_t slot = 0;
        if (PoolSlot::Extent(b.data, slot) && slot >= b.capacity && fws_gpu_host_register(b.data, slot) == 0)
            registered_.insert(b.data);
        else
            unregistrable_.insert(b.data);               // staged from then on
    }

    // ws_server_socket.h:172-196 with OnRecvData on the GPU.
    void OnReadable(USock &u, fws::IOBuffer &&buf, void *ud) {
        retired_.clear();
        auto it = conns_.find(&u);
        if (it == conns_.end() || (it->second.ws->*(&A::server_status_)) != A::kOpen) {
            ref_readable_(u, std::move(buf), ud);
            return;
        }
        EnsureRegistered(buf);
        if (it->second.slot != kNoSlot) {            // batched: decoded with its chunk or at the end of the step
            if (it->second.pending || it->second.inflight) {   // its previous read goes first
                Flush();
                it = conns_.find(&u);
                if (it == conns_.end() || (it->second.ws->*(&A::server_status_)) != A::kOpen) {
                    ref_readable_(u, std::move(buf), ud);    // as the top of this function does
                    return;
                }
            }
            it->second.pending = true;
            pending_.push_back(Pending{&u, std::move(buf), ud});
            // a full chunk goes to the GPU now, so its round trip overlaps the
            // step's remaining reads (and the previous chunk's dispatch)
            if (chunk_ && pending_.size() >= chunk_) Advance();
            return;
        }
        Sock &sock = *it->second.ws;
        GpuRxDecoder<fws::IOBuffer> *dec = it->second.dec.get();   // `it` may be erased by on_close
        ++gpu_reads_;
        const int ret = dec->OnRecvData(buf, Sink{sock});
        Finish(sock, u, ret, [&]() { return dec->error_opcode(); }, false);
    }

    // The error texts ParseFrameHdr sets (w_socket.h:452, 468, 494-496); -3 sets none.
    static void SetErrorText(int ret, uint32_t opcode) {
        char t[160];
        switch (ret) {
        case FWS_ERR_OPCODE: std::snprintf(t, sizeof(t), "Opcode %u is not valid", opcode); break;
        case FWS_ERR_RSV: std::snprintf(t, sizeof(t), "rev bits are not zero"); break;
        case FWS_ERR_TOO_LARGE:
            std::snprintf(t, sizeof(t), "payload length larger thanconstants::MAX_WS_FRAME_SIZE %zu",
                          fws::constants::MAX_WS_FRAME_SIZE);
            break;
        case FWS_ERR_CONTROL_FRAME: std::snprintf(t, sizeof(t), "Control frame over 125 B"); break;
        case FWS_ERR_NOT_MASKED: return;
        default: std::snprintf(t, sizeof(t), "GPU receive decode failed (%d)", ret); break;
        }
        fws::SetErrorString(t, std::strlen(t) + 1);
    }

    GpuContext &ctx_;
    typename Sock::WsOnNewConnectionFunc user_new_conn_;
    typename Sock::WSOnCloseFunc user_close_;
    typename U::Func ref_readable_;
    std::unordered_map<USock *, Conn> conns_;
    std::vector<std::unique_ptr<GpuRxDecoder<fws::IOBuffer>>> retired_;
    uint64_t gpu_reads_ = 0, gpu_batches_ = 0;
    // batched path
    fws_rx_mux *mux_ = nullptr;
    std::vector<uint32_t> free_slots_;
    std::vector<Pending> pending_;
    Batch fl_;                                         // the submitted batch
    bool fl_active_ = false;
    uint32_t chunk_ = kDefaultChunk;                   // reads per submitted chunk within a step (0: per step)
    bool defer_ = true;                                // SetDeferLastChunk
    uint64_t deferred_chunks_ = 0;                     // step ends that left their last chunk in flight
    std::function<bool()> loop_ready_;                 // the loop's queue has events (zero-timeout wait)
    std::function<void()> app_on_event_;
    std::function<void(void *)> delete_fd_;
    USock *retiring_ = nullptr;                        // Retire's flush in progress for this socket
    // zero copy: MemPool slots registered for in-place decode
    bool zero_copy_ = true;
    std::unordered_set<uint8_t *> registered_, unregistrable_;
    std::vector<USock *> deferred_;                    // DeleteFd at the end of the step
    // step profile (FWS_HOOK_PROF)
    using Clock = std::chrono::steady_clock;
    bool prof_on_ = false;
    StepProf prof_;
    Clock::time_point prof_t_, prof_b_;
};

using GpuRxHook = GpuRxHookT<false>;      // ws://
using GpuRxHookTls = GpuRxHookT<true>;    // wss://

}  // namespace fws_amd
