// flashws_amd/gpu_ws.hpp -- header-only C++ adapter that drops the MI355X
// decode path (libfws_gpu.so, include/fws_gpu.h) into flashws's own frame and
// buffer API. It does not include flashws.h (that header links in only one
// TU, SURVEY §0 finding 2): the reference types are template parameters.
//
//   seam 1  fws::WSMaskBytesFast(src, size, mask)         crypto/ws_mask.h:175
//           -> fws_amd::WSMaskBytesFastDevice(dev_src, size, mask, stream)
//   seam 2  WSocket<...>::OnRecvData(IOBuffer&)            net/w_socket.h:543-769
//           -> fws_amd::GpuRxDecoder::OnRecvData(io_buf, sink)
//
// GpuRxDecoder keeps the reference's on_read() contract (w_socket.h:82-84):
// the sink receives (opcode, IOBuffer view aliasing io_buf, is_frame_end,
// is_msg_end, is_control) in the reference's order; PING payloads are handed
// back for the PONG reply and CLOSE frames with their status code, exactly
// where the reference calls SendControlMsg / on_close (w_socket.h:661-711).
// Return values are the reference's ParseFrameHdr codes (0 or negative).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string_view>
#include <utility>
#include <vector>

#include "../fws_gpu.h"

namespace fws_amd {

// seam 1: in-place XOR unmask of device memory (any alignment, any size).
inline int WSMaskBytesFastDevice(void *dev_src, size_t size, uint32_t mask, void *hip_stream = nullptr) {
    return fws_gpu_mask(dev_src, size, mask, hip_stream);
}

// RAII device context (one per host thread / FLoop, floop.h:331-345). Server
// reads are decoded by the persistent receive decode by default (a resident
// grid of kDefaultPersistent workgroups while reads keep coming, gone after
// 250 us without one; push mode on large-BAR devices: DESIGN.md §4.5): the
// environment variable FWS_RX_PERSISTENT=N sets the workgroups, 0 a kernel
// launch per read; SetPersistent() changes it later.
class GpuContext {
public:
    static constexpr uint32_t kDefaultPersistent = 16;
    explicit GpuContext(int device = 0, uint64_t max_frames = 0, uint64_t max_stream_bytes = 0) {
        if (fws_gpu_ctx_create(device, &ctx_) != 0) throw std::runtime_error("fws_gpu_ctx_create failed");
        if ((max_frames || max_stream_bytes) && fws_gpu_ctx_reserve(ctx_, max_frames, max_stream_bytes) != 0) {
            fws_gpu_ctx_destroy(ctx_);
            throw std::runtime_error("fws_gpu_ctx_reserve failed");
        }
        const char *e = std::getenv("FWS_RX_PERSISTENT");
        const long w = e && *e ? std::strtol(e, nullptr, 10) : (long)kDefaultPersistent;
        if (w > 0 && fws_gpu_ctx_set_rx_persistent(ctx_, (uint32_t)(w < 1024 ? w : 1024)) != 0) {
            fws_gpu_ctx_destroy(ctx_);
            throw std::runtime_error("fws_gpu_ctx_set_rx_persistent failed");
        }
    }
    ~GpuContext() { fws_gpu_ctx_destroy(ctx_); }
    GpuContext(const GpuContext &) = delete;
    GpuContext &operator=(const GpuContext &) = delete;
    fws_gpu_ctx *get() const { return ctx_; }
    // the persistent receive decode (fws_gpu_ctx_set_rx_persistent): reads
    // decoded by a resident grid of `workers` workgroups, no launch per read
    void SetPersistent(uint32_t workers) {
        if (fws_gpu_ctx_set_rx_persistent(ctx_, workers) != 0) throw std::runtime_error("set_rx_persistent failed");
    }

private:
    fws_gpu_ctx *ctx_ = nullptr;
};

// seam 2: OnRecvData over the GPU. IOBuffer is fws::IOBuffer (or any type with
// the same {data, size, start_pos, capacity} members and 4-arg constructor,
// base/buffer_manager.h:36-52). Sink must provide:
//   void on_read(uint32_t opcode, IOBuffer &&part, bool frame_end, bool msg_end, bool is_ctl);
//   void on_ping(std::string_view payload);               // reply PONG (w_socket.h:662-666)
//   void on_close(uint32_t code, std::string_view payload); // w_socket.h:667-710
//   IOBuffer request_buf(size_t n);                         // e.g. fws::RequestBuf (buffer_manager.h:90)
template <class IOBuffer>
class GpuRxDecoder {
public:
    explicit GpuRxDecoder(GpuContext &ctx) {
        if (fws_rx_session_create(ctx.get(), 1, &s_) != 0) throw std::runtime_error("fws_rx_session_create failed");
    }
    ~GpuRxDecoder() { fws_rx_session_destroy(s_); }
    GpuRxDecoder(const GpuRxDecoder &) = delete;
    GpuRxDecoder &operator=(const GpuRxDecoder &) = delete;

    template <class Sink>
    int OnRecvData(IOBuffer &io_buf, Sink &&sink) {
        uint8_t *data = io_buf.data + io_buf.start_pos;
        const uint64_t size = (uint64_t)io_buf.size;
        const uint64_t cap = io_buf.capacity - io_buf.start_pos;
        const fws_rx_event *ev = nullptr;
        const uint8_t *ctl = nullptr;
        uint64_t n_ev = 0, ctl_used = 0;
        // the session's own event / control sinks: sized by what the read holds
        const int ret = fws_rx_session_feed_view(s_, data, size, cap, &ev, &n_ev, &ctl, &ctl_used);
        DispatchEvents(io_buf, ev, n_ev, ctl, sink);
        return ret;
    }

    // One read's decoded events onto the sink, in order (OnRecvData's callbacks,
    // w_socket.h:629-747); also used for the reads of a batched feed (fws_rx_mux).
    template <class Sink>
    static void DispatchEvents(IOBuffer &io_buf, const fws_rx_event *ev, uint64_t n_ev, const uint8_t *ctl,
                               Sink &sink) {
        for (uint64_t i = 0; i < n_ev; ++i) {
            const fws_rx_event &e = ev[i];
            const std::string_view payload((const char *)ctl + e.ctl_off, e.kind == 0 && !e.is_ctl ? 0 : e.size);
            if (e.kind == 1) {
                sink.on_ping(payload);
            } else if (e.kind == 2) {
                sink.on_close(e.code, payload);
            } else if (!e.is_ctl) {
                // aliasing view of the (now unmasked) read buffer, w_socket.h:715-728
                sink.on_read(e.opcode,
                             IOBuffer(io_buf.data, (ssize_t)e.size, io_buf.start_pos + e.data_off,
                                      io_buf.start_pos + e.capacity),
                             e.frame_end != 0, e.msg_end != 0, false);
            } else {
                // PONG payload: copied into a fresh buffer (the reference hands over
                // its control buffer buf_, w_socket.h:729-731)
                IOBuffer b = sink.request_buf(payload.size());
                for (size_t k = 0; k < payload.size(); ++k) b.data[b.start_pos + k] = (uint8_t)payload[k];
                b.size = (ssize_t)payload.size();
                sink.on_read(e.opcode, std::move(b), e.frame_end != 0, e.msg_end != 0, true);
            }
        }
    }

    // The opcode of the frame the last failing read stopped at (for the
    // reference's error text, w_socket.h:452).
    uint32_t error_opcode() const {
        uint32_t op = 0;
        (void)fws_rx_session_error(s_, &op);
        return op;
    }

private:
    fws_rx_session *s_ = nullptr;
};

// SendFrame over the GPU for one connection (w_socket.h:832-944): frames are
// queued with the reference's WriteFrame arguments and sent as one batch;
// the wire bytes of the whole batch come back in `wire`. A client encoder
// masks with the keys it is given (the reference draws SemiSecureRand32,
// w_socket.h:860). Opcode / FIN sequencing carries across batches.
class GpuTxEncoder {
public:
    GpuTxEncoder(GpuContext &ctx, bool is_server) {
        if (fws_tx_session_create(ctx.get(), is_server ? 1 : 0, &s_) != 0)
            throw std::runtime_error("fws_tx_session_create failed");
    }
    ~GpuTxEncoder() { fws_tx_session_destroy(s_); }
    GpuTxEncoder(const GpuTxEncoder &) = delete;
    GpuTxEncoder &operator=(const GpuTxEncoder &) = delete;

    // WriteFrame(buf, frame_type, last_frame_if_possible) for a payload that
    // stays valid until Flush().
    void Queue(const uint8_t *payload, uint64_t len, uint32_t frame_type, bool last, uint32_t key = 0) {
        ptrs_.push_back(payload);
        lens_.push_back(len);
        types_.push_back(frame_type);
        last_.push_back(last ? 1 : 0);
        keys_.push_back(key);
    }

    // Frames queued since the last Flush, as wire bytes; 0 or an FWS_ERR_* code.
    int Flush(std::vector<uint8_t> &wire) {
        uint64_t need = 0;
        for (uint64_t l : lens_) need += l + 14;
        wire.resize(need);
        uint64_t len = 0;
        const int r = fws_tx_session_send(s_, ptrs_.data(), lens_.data(), types_.data(), last_.data(), keys_.data(),
                                          (uint32_t)ptrs_.size(), wire.data(), need, &len);
        wire.resize(r == 0 ? len : 0);
        ptrs_.clear();
        lens_.clear();
        types_.clear();
        last_.clear();
        keys_.clear();
        return r;
    }

private:
    fws_tx_session *s_ = nullptr;
    std::vector<const uint8_t *> ptrs_;
    std::vector<uint64_t> lens_;
    std::vector<uint32_t> types_;
    std::vector<uint8_t> last_;
    std::vector<uint32_t> keys_;
};

}  // namespace fws_amd
