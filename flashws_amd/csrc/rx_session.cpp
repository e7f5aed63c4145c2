// rx_session.cpp -- fws_rx_session: WSocket::OnRecvData (net/w_socket.h:543-769)
// for host read buffers, with the byte work on the GPU.
//
// Per read: the continuation of a frame in progress is unmasked with the
// carried (rotated) key, the rest of the read -- prefixed with any header
// bytes staged from the previous read -- is parsed and unmasked (one launch of
// k_decode_one for reads whose header stream fits the small-read kernel, else
// fws_gpu_decode_stream), the unmasked bytes end up in the caller's buffer --
// in place when it lies in registered host memory (fws_gpu_host_register),
// else through pinned staging or device copies -- and the host replays the reference's
// per-part bookkeeping over the decoded frame list (no byte parsing, no XOR on
// the host) to produce the exact on_read() / PONG / CLOSE event sequence and
// carried RX state (w_socket.h:223-245). Host code only; server side only
// (client RX has no unmask and is out of scope).
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <vector>

#include "fws_internal.h"

namespace {

constexpr int kWaitHead = 0, kWaitPayload = 1;   // w_socket.h:225-228
// reads in registered host memory up to this size are decoded in place (one
// workgroup streams them over PCIe); larger ones take the device path
constexpr uint64_t kInPlaceMax = 256u << 10;

inline uint32_t rotr(uint32_t v, uint32_t b) {     // base/constexpr_math.h:67-82
    b &= 31u;
    return (v >> b) | (v << ((32u - b) & 31u));
}

}  // namespace

struct fws_rx_session {
    fws_gpu_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;
    // carried RX state, w_socket.h:223-245
    int recv_status = kWaitHead;
    uint64_t unread = 0;
    uint32_t key = 0;
    uint8_t last_op = 0, last_ctl_op = 0, last_fin = 0;
    bool is_ctl = false;
    uint32_t part_len = 0;
    uint8_t hdr[14] = {};
    // control payload staging (buf_), w_socket.h:637-658
    uint8_t ctl[128] = {};
    uint32_t ctl_size = 0;
    bool ctl_alloc = false;
    // device side
    uint8_t *dA = nullptr, *dB = nullptr;
    uint64_t capA = 0, capB = 0;
    fws_frame_info *dframes = nullptr;
    uint32_t fcap = 0;
    fws_decode_result *dres = nullptr;
    // pinned landing area: the decode result and the first kSpec frames come
    // back with the bytes, before the one synchronize; larger reads copy the
    // rest after it
    static constexpr uint32_t kSpec = 1024;
    static_assert(kSpec > kSmallFrames, "small-read frames land in the pinned block");
    static constexpr uint64_t kResPad = 64;
    // reads up to kZcMax bytes are staged by the host into pinned memory the
    // kernels work on directly (no copy-engine transfers; one copy of the
    // result block back)
    static constexpr uint64_t kZcMax = 16u << 10;
    uint8_t *hstage = nullptr;
    uint32_t *hflag = nullptr;         // host_done flag of the one-launch paths (coherent pinned word)
    uint32_t seq = 0;
    fws_decode_result *hres = nullptr;
    fws_frame_info *hframes = nullptr;
    uint32_t hfcap = 0;
    std::vector<uint8_t> stream_host;
    // event sinks of the current feed
    fws_rx_event *ev = nullptr;
    uint64_t ev_cap = 0, n_ev = 0;
    uint8_t *ctl_out = nullptr;
    uint64_t ctl_cap = 0, ctl_used = 0;

    // fws_rx_session_feed_view: the session's own growing sinks instead
    bool own = false;
    std::vector<fws_rx_event> own_ev;
    std::vector<uint8_t> own_ctl;
    // the last protocol error of a feed (fws_rx_session_error)
    int err_code = 0;
    uint32_t err_opcode = 0;
    bool borrowed_stream = false;     // a fws_rx_mux connection: the mux's stream

    void reset_state() {              // a new connection (w_socket.h:223-245 initial values)
        recv_status = kWaitHead;
        unread = 0;
        key = 0;
        last_op = last_ctl_op = last_fin = 0;
        is_ctl = false;
        part_len = 0;
        ctl_size = 0;
        ctl_alloc = false;
        err_code = 0;
        err_opcode = 0;
    }

    void push(const fws_rx_event &e) {
        if (own) own_ev.push_back(e);
        else if (n_ev < ev_cap) ev[n_ev] = e;
        ++n_ev;
    }
    uint64_t push_ctl(const uint8_t *p, uint64_t n) {
        const uint64_t off = ctl_used;
        if (own) own_ctl.insert(own_ctl.end(), p, p + n);
        else if (ctl_used + n <= ctl_cap) memcpy(ctl_out + ctl_used, p, n);
        ctl_used += n;
        return off;
    }

    // ParseFrameHdr's state side effects and result on <= 14 staged bytes
    // (w_socket.h:443-521); used only for a header left incomplete at the end
    // of a read and for the failing header of a protocol error.
    int host_parse(const uint8_t *d, uint64_t avail) {
        if (avail < 2) return 0;
        const uint32_t b0 = d[0], op = b0 & 15u;
        const bool valid = (op <= 2u) || (op >= 8u && op <= 10u);
        if (!valid) return FWS_ERR_OPCODE;
        if (op >> 3) { is_ctl = true; last_ctl_op = (uint8_t)op; }
        else if (op != 0u) last_op = (uint8_t)op;
        if (b0 & 112u) return FWS_ERR_RSV;
        const uint32_t b1 = d[1];
        const bool masked = b1 >> 7;
        uint64_t plen = b1 & 127u, n = 2;
        if (plen == 126u) {
            if (avail < 4) return 0;
            plen = ((uint64_t)d[2] << 8) | d[3];
            n = 4;
        } else if (plen == 127u) {
            if (avail < 10) return 0;
            plen = 0;
            for (int i = 0; i < 8; ++i) plen = (plen << 8) | d[2 + i];
            n = 10;
        }
        if (plen > (1ull << 32)) return FWS_ERR_TOO_LARGE;
        if (!masked) return FWS_ERR_NOT_MASKED;
        if (avail < n + 4) return 0;
        memcpy(&key, d + n, 4);
        return (int)(n + 4);
    }

    // The per-part tail of OnRecvData's loop body, w_socket.h:623-764.
    void part(uint8_t *buf, uint64_t size, uint64_t cap, uint64_t data, uint64_t avail, uint64_t remain,
              int status_at_part) {
        const bool frame_end = unread <= remain;
        const bool msg_end = last_fin && frame_end;
        const uint32_t opcode = is_ctl ? last_ctl_op : last_op;
        if (is_ctl && avail > 0) {                                    // :629-659
            if (status_at_part == kWaitHead || !ctl_alloc) { ctl_alloc = true; ctl_size = 0; }
            // control payloads are <= 125 B (checked at the header, feed_impl), so
            // this never clamps; the clamp keeps ctl_size inside the array regardless
            const uint64_t room = sizeof(ctl) - ctl_size;
            const uint64_t take = avail < room ? avail : room;
            memcpy(ctl + ctl_size, buf + data, take);
            ctl_size += (uint32_t)take;
        }
        if (frame_end && is_ctl) {                                   // :661-711
            const uint32_t n = ctl_alloc ? ctl_size : 0u;
            if (opcode == 9u) {
                fws_rx_event e{};
                e.kind = 1; e.opcode = 10; e.is_ctl = 1; e.frame_end = 1; e.msg_end = 1; e.fin = 1;
                e.size = n; e.data_off = data; e.ctl_off = push_ctl(ctl, n);
                push(e);
                ctl_alloc = false; ctl_size = 0;
            } else if (opcode == 8u) {
                fws_rx_event e{};
                e.kind = 2; e.opcode = 8; e.is_ctl = 1; e.frame_end = 1; e.msg_end = 1; e.fin = 1;
                e.code = n >= 2 ? ((uint32_t)ctl[0] << 8 | ctl[1]) : 1005u;
                e.size = n; e.data_off = data; e.ctl_off = push_ctl(ctl, n);
                push(e);
                ctl_alloc = false; ctl_size = 0;
            }
        }
        if (!is_ctl || opcode == 10u) {                               // :713-747
            fws_rx_event e{};
            e.kind = 0; e.opcode = opcode; e.is_ctl = is_ctl; e.frame_end = frame_end; e.msg_end = msg_end;
            if (!is_ctl) {
                e.size = avail;
                e.data_off = data;
                e.capacity = (data + avail == size) ? cap : data + avail;
            } else {
                const uint32_t n = ctl_alloc ? ctl_size : 0u;
                e.size = n; e.data_off = data; e.ctl_off = push_ctl(ctl, n);
                ctl_alloc = false; ctl_size = 0;
            }
            push(e);
        }
        unread -= avail;                                              // :750-764
        if (unread == 0 && is_ctl) is_ctl = false;
        if (!frame_end) {
            key = rotr(key, (uint32_t)(avail & 3u) * 8u);
            recv_status = kWaitPayload;
        } else {
            recv_status = kWaitHead;
        }
    }

    // bytes: device stream capacity; stage: the read goes through the pinned
    // staging area (size <= kZcMax, feed_impl)
    int ensure(uint64_t bytes, uint32_t nframes, bool stage) {
        hipError_t e = hipSuccess;
        if (bytes + 32 > capA) {
            if (dA) (void)hipFree(dA);
            if (dB) (void)hipFree(dB);
            capA = capB = (bytes + 32 + 4095) & ~4095ull;
            if ((e = hipMalloc((void **)&dA, capA)) != hipSuccess) return fws_hip_status(e);
            if ((e = hipMalloc((void **)&dB, capB)) != hipSuccess) return fws_hip_status(e);
        }
        if (nframes > fcap || !dres) {
            // one device block [result | frames], so a single copy brings back
            // the result and the first frames
            if (dres) (void)hipFree(dres);
            fcap = nframes > fcap ? nframes : fcap;
            if ((e = hipMalloc((void **)&dres, kResPad + (uint64_t)fcap * sizeof(fws_frame_info))) != hipSuccess)
                return fws_hip_status(e);
            dframes = (fws_frame_info *)((uint8_t *)dres + kResPad);
        }
        if (stage && !hstage && (e = hipHostMalloc((void **)&hstage, 2 * kZcMax + 64)) != hipSuccess)
            return fws_hip_status(e);
        if (!hflag) {
            if ((e = hipHostMalloc((void **)&hflag, 64, hipHostMallocCoherent)) != hipSuccess) return fws_hip_status(e);
            *hflag = 0;
            seq = 0;
        }
        return host_room(kSpec);
    }

    // pinned [result | frames] landing block for n frames
    int host_room(uint32_t n) {
        if (n <= hfcap) return 0;
        if (hres) (void)hipHostFree(hres);
        hres = nullptr;
        hframes = nullptr;
        hfcap = 0;
        hipError_t e = hipHostMalloc((void **)&hres, kResPad + (uint64_t)n * sizeof(fws_frame_info));
        if (e != hipSuccess) return fws_hip_status(e);
        hframes = (fws_frame_info *)((uint8_t *)hres + kResPad);
        hfcap = n;
        return 0;
    }
};

int fws_wait_flag(const volatile uint32_t *flag, uint32_t seq, hipStream_t s) {
    const uint32_t *f = (const uint32_t *)flag;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; ++i) {
        if (__atomic_load_n(f, __ATOMIC_ACQUIRE) == seq) return 0;
        if ((i & 255u) == 255u && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) break;
#if defined(__x86_64__) || defined(__i386__)
        __builtin_ia32_pause();
#elif defined(__aarch64__)
        __asm__ __volatile__("yield");
#endif
    }
    // a long decode (or a failed launch): block on the stream instead of spinning
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess) return fws_hip_status(e);
    return __atomic_load_n(f, __ATOMIC_ACQUIRE) == seq ? 0 : FWS_ERR_INTERNAL;
}

extern "C" {

int fws_rx_session_create(fws_gpu_ctx *ctx, int is_server, fws_rx_session **out) {
    if (!ctx || !out) return FWS_ERR_INVALID;
    *out = nullptr;
    if (!is_server) return FWS_ERR_INVALID;      // client RX (no unmask) is not on this path
    int r = fws_hip_status(hipSetDevice(ctx->device));
    if (r) return r;
    fws_rx_session *s = new fws_rx_session();
    s->ctx = ctx;
    if ((r = fws_hip_status(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)))) {
        delete s;
        return r;
    }
    *out = s;
    return 0;
}

void fws_rx_session_destroy(fws_rx_session *s) {
    if (!s) return;
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->dA) (void)hipFree(s->dA);
    if (s->dB) (void)hipFree(s->dB);
    if (s->dres) (void)hipFree(s->dres);
    if (s->hres) (void)hipHostFree(s->hres);
    if (s->hstage) (void)hipHostFree(s->hstage);
    if (s->hflag) (void)hipHostFree(s->hflag);
    if (s->stream && !s->borrowed_stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

int fws_rx_session_state(const fws_rx_session *s, fws_rx_state *out) {
    if (!s || !out) return FWS_ERR_INVALID;
    out->recv_status = s->recv_status;
    out->mask_key = s->key;
    out->unread_pl_len = s->unread;
    out->last_rx_opcode = s->last_op;
    out->last_rx_control_opcode = s->last_ctl_op;
    out->last_rx_fin_flag = s->last_fin;
    out->is_rx_control_frame = s->is_ctl ? 1 : 0;
    out->last_rx_hdr_part_len = s->part_len;
    return 0;
}

static int feed_impl(fws_rx_session *s, uint8_t *buf, uint64_t size, uint64_t buf_capacity);
static int replay(fws_rx_session *s, uint8_t *buf, uint64_t size, uint64_t buf_capacity, uint64_t u,
                  uint32_t part0, uint64_t rest, uint64_t L, const fws_decode_result &res,
                  const fws_frame_info *frames);

int fws_rx_session_feed(fws_rx_session *s, uint8_t *buf, uint64_t size, uint64_t buf_capacity,
                        fws_rx_event *events, uint64_t ev_cap, uint64_t *n_events,
                        uint8_t *ctl_out, uint64_t ctl_cap, uint64_t *ctl_used) {
    if (!s || (size && !buf) || !n_events || !ctl_used) return FWS_ERR_INVALID;
    s->own = false;
    s->ev = events; s->ev_cap = events ? ev_cap : 0; s->n_ev = 0;
    s->ctl_out = ctl_out; s->ctl_cap = ctl_out ? ctl_cap : 0; s->ctl_used = 0;
    s->err_code = 0;
    const int r = feed_impl(s, buf, size, buf_capacity);
    if (r < 0) s->err_code = r;
    *n_events = s->n_ev;
    *ctl_used = s->ctl_used;
    if (r == 0 && (s->n_ev > ev_cap || s->ctl_used > ctl_cap)) return FWS_ERR_CAPACITY;
    return r;
}

int fws_rx_session_feed_view(fws_rx_session *s, uint8_t *buf, uint64_t size, uint64_t buf_capacity,
                             const fws_rx_event **events, uint64_t *n_events, const uint8_t **ctl,
                             uint64_t *ctl_used) {
    if (!s || (size && !buf) || !events || !n_events || !ctl || !ctl_used) return FWS_ERR_INVALID;
    s->own = true;
    s->own_ev.clear();
    s->own_ctl.clear();
    s->n_ev = 0;
    s->ctl_used = 0;
    s->err_code = 0;
    const int r = feed_impl(s, buf, size, buf_capacity);
    if (r < 0) s->err_code = r;
    *events = s->own_ev.data();
    *n_events = s->own_ev.size();
    *ctl = s->own_ctl.data();
    *ctl_used = s->own_ctl.size();
    s->own = false;
    return r;
}

int fws_rx_session_error(const fws_rx_session *s, uint32_t *opcode) {
    if (!s) return FWS_ERR_INVALID;
    if (opcode) *opcode = s->err_opcode;
    return s->err_code;
}

static int feed_impl(fws_rx_session *s, uint8_t *buf, uint64_t size, uint64_t buf_capacity) {
    if (size == 0) return 0;
    int r;
    hipError_t e;
    hipStream_t st = s->stream;
    if ((r = fws_hip_status(hipSetDevice(s->ctx->device)))) return r;
    const uint32_t fcap = (uint32_t)((size + s->part_len) / 6 + 2);
    // staged reads (<= kZcMax) use [continuation | pad | header stream] in hstage:
    // at most kZcMax + 15 + 13 bytes of its 2 kZcMax + 64
    if ((r = s->ensure(size + 16, fcap, size <= fws_rx_session::kZcMax))) return r;

    // 1. continuation of the frame in progress (WAIT_FRAME_PAYLOAD, w_socket.h:607-617)
    uint64_t u = 0;
    fws_decode_result res{};
    const uint32_t spec = fcap < fws_rx_session::kSpec ? fcap : fws_rx_session::kSpec;
    if (s->recv_status == kWaitPayload) u = size < s->unread ? size : s->unread;
    const uint32_t part0 = s->part_len;
    const uint64_t rest = size - u;
    const uint64_t L = part0 + rest;
    // The header stream [staged header bytes | rest of the read] is decoded on
    // `hs`: streams of <= kSmallMax bytes by the one-launch small-read kernel
    // (declined for > kSmallFrames headers, then by the parallel decode),
    // longer ones by fws_gpu_decode_stream. The result block (result + the
    // first `spec` frames) comes back with one copy.
    auto launch = [&](uint8_t *hs, bool small) -> int {
        int rr = small ? fws_launch_decode_small(hs, L, s->dframes, fcap, s->dres, st)
                       : fws_gpu_decode_stream(s->ctx, hs, L, s->dframes, fcap, s->dres, nullptr, st);
        if (rr) return rr;
        return fws_hip_status(hipMemcpyAsync(s->hres, s->dres,
                                             fws_rx_session::kResPad + (uint64_t)spec * sizeof(fws_frame_info),
                                             hipMemcpyDeviceToHost, st));
    };
    const bool small = L <= kSmallMax;
    bool frames_here = false;                    // every frame record already in hframes
    // a read in registered host memory (fws_gpu_host_register: e.g. the MemPool
    // read buffers the drop-in hook registers) is decoded where it lies, when the
    // header stream needs no staged bytes in front and both parts start 16-B
    // aligned (the kernels' chunk grid)
    uint8_t *const dev = (part0 == 0 && size <= kInPlaceMax && small) ? fws_host_alias(buf, size) : nullptr;
    const bool in_place = dev && ((uintptr_t)dev & 15u) == 0 && (rest == 0 || ((uintptr_t)(dev + u) & 15u) == 0);
    if (in_place) {
        const uint32_t segcap = (uint32_t)(L / 6 + 2 < kSmallFrames ? L / 6 + 2 : kSmallFrames);
        if ((r = s->host_room(segcap > fws_rx_session::kSpec ? segcap : fws_rx_session::kSpec))) return r;
        fws_seg_desc d{};
        d.cont_off = 0;
        d.hs_off = u;
        d.u = (uint32_t)u;
        d.key = s->key;
        d.L = (uint32_t)(rest ? L : 0);
        d.fcap = segcap;
        const uint32_t seq = ++s->seq;
        fws_rx_service *const v = fws_ctx_rx_service(s->ctx);
        if (fws_rx_service_can_push(v, size)) {
            // the resident grid, the read pushed into its device staging; the decoded
            // bytes come back to the registered range itself
            if ((r = fws_rx_service_push(v, buf, size, dev, d, s->hframes, s->hres, s->hflag, seq))) return r;
        } else if (v) {                                                  // the resident grid, no launch
            if ((r = fws_rx_service_run(v, dev, nullptr, &d, 1, s->hframes, s->hres, s->hflag, seq))) return r;
        } else {
            if ((r = fws_launch_decode_one(dev, d, s->hframes, s->hres, st, s->hflag, seq))) return r;
            if ((r = fws_wait_flag(s->hflag, seq, st))) return r;
        }
        frames_here = true;
        if (rest && s->hres->status == FWS_SMALL_DECLINED) {
            if ((r = launch(dev + u, false))) return r;       // the parallel decode, in place
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return fws_hip_status(e);
            frames_here = false;
        }
    } else if (size <= fws_rx_session::kZcMax) {
        // tiny read: the host stages [continuation | 16-B pad | header stream]
        // in pinned memory; one launch (k_decode_one: the continuation unmask,
        // then the small-read decode) works on it there and writes the result
        // and the frame records straight into the pinned landing block -- no
        // copy-engine transfer and no second launch on the round trip
        uint8_t *cont = s->hstage;
        const uint64_t hs_off = (u + 15) & ~15ull;
        uint8_t *hs = s->hstage + hs_off;
        if (u) memcpy(cont, buf, u);
        if (rest) {
            if (part0) memcpy(hs, s->hdr, part0);
            memcpy(hs + part0, buf + u, rest);
        }
        const uint32_t segcap = (uint32_t)(L / 6 + 2 < kSmallFrames ? L / 6 + 2 : kSmallFrames);
        if ((r = s->host_room(segcap > fws_rx_session::kSpec ? segcap : fws_rx_session::kSpec))) return r;
        fws_seg_desc d{};
        d.cont_off = 0;
        d.hs_off = hs_off;
        d.u = (uint32_t)u;
        d.key = s->key;
        d.L = (uint32_t)(rest ? L : 0);
        d.fcap = segcap;
        d.fbase = 0;
        const uint32_t seq = ++s->seq;
        fws_rx_service *const v = fws_ctx_rx_service(s->ctx);
        const uint64_t span = rest ? hs_off + L : u;                     // the staged layout's bytes
        if (fws_rx_service_can_push(v, span)) {
            // pushed into the grid's device staging; the decoded bytes come back here
            if ((r = fws_rx_service_push(v, s->hstage, span, s->hstage, d, s->hframes, s->hres, s->hflag, seq)))
                return r;
        } else if (v) {
            if ((r = fws_rx_service_run(v, s->hstage, nullptr, &d, 1, s->hframes, s->hres, s->hflag, seq))) return r;
        } else {
            if ((r = fws_launch_decode_one(s->hstage, d, s->hframes, s->hres, st, s->hflag, seq))) return r;
            if ((r = fws_wait_flag(s->hflag, seq, st))) return r;
        }
        frames_here = true;
        if (rest && s->hres->status == FWS_SMALL_DECLINED) {
            // more than kSmallFrames headers: the parallel decode on the same bytes
            // (the continuation is unmasked already; the header stream untouched)
            if ((r = launch(hs, false))) return r;
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return fws_hip_status(e);
            frames_here = false;
        }
        if (u) memcpy(buf, cont, u);
        if (rest) memcpy(buf + u, hs + part0, rest);
    } else {
        if (u) {
            if ((e = hipMemcpyAsync(s->dA, buf, u, hipMemcpyHostToDevice, st)) != hipSuccess) return fws_hip_status(e);
            if ((r = fws_gpu_mask(s->dA, u, s->key, st))) return r;
            if ((e = hipMemcpyAsync(buf, s->dA, u, hipMemcpyDeviceToHost, st)) != hipSuccess) return fws_hip_status(e);
        }
        if (rest) {
            if (part0 && (e = hipMemcpyAsync(s->dB, s->hdr, part0, hipMemcpyHostToDevice, st)) != hipSuccess)
                return fws_hip_status(e);
            if ((e = hipMemcpyAsync(s->dB + part0, buf + u, rest, hipMemcpyHostToDevice, st)) != hipSuccess)
                return fws_hip_status(e);
            if ((r = launch(s->dB, small))) return r;
            if ((e = hipMemcpyAsync(buf + u, s->dB + part0, rest, hipMemcpyDeviceToHost, st)) != hipSuccess)
                return fws_hip_status(e);
        }
        if ((e = hipStreamSynchronize(st)) != hipSuccess) return fws_hip_status(e);
        if (rest && small && s->hres->status == FWS_SMALL_DECLINED) {
            // declined (nothing written): the parallel decode, and the bytes again
            if ((r = launch(s->dB, false))) return r;
            if ((e = hipMemcpyAsync(buf + u, s->dB + part0, rest, hipMemcpyDeviceToHost, st)) != hipSuccess)
                return fws_hip_status(e);
            if ((e = hipStreamSynchronize(st)) != hipSuccess) return fws_hip_status(e);
        }
    }
    if (rest) res = *s->hres;
    if (res.status == FWS_ERR_CAPACITY) return FWS_ERR_CAPACITY;
    if (res.n_frames > spec && !frames_here) {
        if ((r = s->host_room((uint32_t)res.n_frames))) return r;
        if ((e = hipMemcpy(s->hframes, s->dframes, (uint64_t)res.n_frames * sizeof(fws_frame_info),
                           hipMemcpyDeviceToHost)) != hipSuccess)
            return fws_hip_status(e);
    }
    return replay(s, buf, size, buf_capacity, u, part0, rest, L, res, s->hframes);
}

// Steps 3-4 of a feed, once the read's bytes are unmasked in buf: OnRecvData's
// loop replayed over the decoded frame list (res, frames: the header stream's
// decode; u continuation bytes, part0 staged header bytes, rest = size - u,
// L = part0 + rest).
static int replay(fws_rx_session *s, uint8_t *buf, uint64_t size, uint64_t buf_capacity, uint64_t u,
                  uint32_t part0, uint64_t rest, uint64_t L, const fws_decode_result &res,
                  const fws_frame_info *frames) {
    // 3. replay OnRecvData's loop over the decoded parts
    if (u) {
        s->part(buf, size, buf_capacity, 0, u, size, kWaitPayload);
    }
    if (!rest) return 0;   // the whole read was payload of the frame in progress
    // header stream coordinate x <-> read coordinate x - part0 + u
    for (uint32_t i = 0; i < res.n_frames; ++i) {
        const fws_frame_info &fi = frames[i];
        const uint32_t op = fi.opcode;
        // RFC 6455 §5.5: control frames carry <= 125 B. The reference only asserts
        // this in debug builds (w_socket.h:654) and otherwise copies past its 125-B
        // control buffer; the session refuses such a frame instead. A control frame
        // with FIN = 0 is handled as the reference handles it (PING answered, CLOSE
        // honoured at its frame end, w_socket.h:659-711, FIN not checked).
        if ((op >> 3) && fi.payload_len > 125u) {
            s->err_opcode = op;
            return FWS_ERR_CONTROL_FRAME;
        }
        if (op >> 3) { s->is_ctl = true; s->last_ctl_op = (uint8_t)op; }      // :455-464
        else if (op != 0u) s->last_op = (uint8_t)op;
        s->key = fi.key;
        s->part_len = 0;
        const uint64_t data = fi.hdr_off + fi.hdr_len - part0 + u;
        s->unread = fi.payload_len;
        s->last_fin = fi.fin;
        const uint64_t remain = size - data;
        const uint64_t avail = remain < fi.payload_len ? remain : fi.payload_len;
        s->part(buf, size, buf_capacity, data, avail, remain, kWaitHead);
    }
    // 4. the read ends inside a header, or at a protocol error (bookkeeping of
    //    the staged parse, w_socket.h:566-603)
    if (res.status < 0 || res.carry_hdr_len) {
        const uint64_t at = res.status < 0 ? res.err_off : L - res.carry_hdr_len;
        uint8_t win[14];
        uint64_t have = 0;
        for (; have < 14 && at + have < L; ++have) {
            const uint64_t x = at + have;
            win[have] = x < part0 ? s->hdr[x] : buf[x - part0 + u];
        }
        const int pr = s->host_parse(win, have);
        if (res.status < 0) {
            s->err_opcode = have ? (uint32_t)(win[0] & 15u) : 0u;
            return pr < 0 ? pr : res.status;
        }
        // incomplete: reference stages min(14 - part_len, bytes left) (:567-569, 592)
        const uint64_t staged_before = at < part0 ? part0 - at : 0;   // bytes of it from earlier reads
        const uint64_t from_read = L - at - staged_before;
        memmove(s->hdr, win, have);
        s->part_len = (uint32_t)(staged_before + from_read);
    }
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------- fws_rx_mux
// The reads of many connections in one round trip (the
// FLoop::OneStep shape, floop.h:661-703: every readable socket's read in one
// loop iteration). Per connection a fws_rx_session holds the carried state
// and replays OnRecvData's bookkeeping; the byte work of all reads is one
// pinned staging pass, one H2D copy, one launch (k_decode_segments: one
// workgroup per read) and one D2H copy. Reads a segment cannot take (a header
// stream over kSmallMax bytes or kSmallFrames headers, a read over
// kMuxMaxRead) go through the connection's own session afterwards.
struct fws_rx_mux {
    fws_gpu_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;
    std::vector<fws_rx_session *> conns;
    // pinned staging [segments] and its device copy
    uint8_t *hbuf = nullptr, *dbuf = nullptr;
    uint64_t bcap = 0;
    // pinned [descriptors | results | frames] and its device copy
    uint8_t *hmeta = nullptr, *dmeta = nullptr;
    uint64_t mcap = 0;
    std::vector<uint8_t> seen;        // per connection: fed in this call
    uint64_t zc_max = 0;              // batches up to this many bytes: kernels on the pinned buffers
    uint32_t *dctr = nullptr;         // host_done counter of the zero-copy launch (reset by its last workgroup)
    uint32_t *hflag = nullptr;        // and its flag (coherent pinned word)
    uint32_t seq = 0;
    // the submitted batch (fws_rx_mux_submit .. fws_rx_mux_complete)
    struct Plan {
        uint64_t u, rest, L, cont_off, hs_off;
        uint32_t part0, seg;                     // seg: index in the launch, or kNone (session path)
        uint8_t *dev;                            // decoded in place (registered host memory), or null
    };
    enum Wait { kWaitNone, kWaitService, kWaitFlag, kWaitStream };
    bool inflight = false;
    Wait wait = kWaitNone;
    std::vector<fws_rx_read> sub_reads;
    std::vector<Plan> sub_plan;
    uint64_t sub_desc_bytes = 0, sub_res_bytes = 0;
    uint32_t sub_seq = 0;
    fws_rx_service *sub_svc = nullptr;           // the service a kWaitService chunk was posted to

    int ensure(uint64_t bytes, uint64_t meta) {
        hipError_t e;
        if (bytes > bcap) {
            if (hbuf) (void)hipHostFree(hbuf);
            if (dbuf) (void)hipFree(dbuf);
            hbuf = dbuf = nullptr;
            bcap = (bytes + 65535) & ~65535ull;
            if ((e = hipHostMalloc((void **)&hbuf, bcap)) != hipSuccess) { bcap = 0; return fws_hip_status(e); }
            if ((e = hipMalloc((void **)&dbuf, bcap)) != hipSuccess) { bcap = 0; return fws_hip_status(e); }
        }
        if (meta > mcap) {
            if (hmeta) (void)hipHostFree(hmeta);
            if (dmeta) (void)hipFree(dmeta);
            hmeta = dmeta = nullptr;
            mcap = (meta + 65535) & ~65535ull;
            if ((e = hipHostMalloc((void **)&hmeta, mcap)) != hipSuccess) { mcap = 0; return fws_hip_status(e); }
            if ((e = hipMalloc((void **)&dmeta, mcap)) != hipSuccess) { mcap = 0; return fws_hip_status(e); }
        }
        return 0;
    }
};

namespace {
constexpr uint64_t kMuxMaxRead = 256u << 10;   // larger reads: the connection's session path
// Batches of at most this many staged bytes skip the copy engines: the segment
// kernel reads and writes the pinned staging over PCIe (env FWS_MUX_ZC_MAX
// overrides; 0 = always copy).
constexpr uint64_t kMuxZcMax = 256u << 10;
constexpr uint32_t kNone = 0xFFFFFFFFu;
inline uint64_t al16(uint64_t x) { return (x + 15) & ~15ull; }
}  // namespace

extern "C" {

int fws_rx_mux_create(fws_gpu_ctx *ctx, uint32_t n_conns, fws_rx_mux **out) {
    if (!ctx || !out || n_conns == 0) return FWS_ERR_INVALID;
    *out = nullptr;
    int r = fws_hip_status(hipSetDevice(ctx->device));
    if (r) return r;
    fws_rx_mux *m = new fws_rx_mux();
    m->ctx = ctx;
    if ((r = fws_hip_status(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking)))) {
        delete m;
        return r;
    }
    m->conns.resize(n_conns, nullptr);
    m->seen.resize(n_conns, 0);
    if ((r = fws_hip_status(hipMalloc((void **)&m->dctr, 64))) ||
        (r = fws_hip_status(hipMemset(m->dctr, 0, 64))) ||
        (r = fws_hip_status(hipHostMalloc((void **)&m->hflag, 64, hipHostMallocCoherent)))) {
        fws_rx_mux_destroy(m);
        return r;
    }
    *m->hflag = 0;
    const char *zc = getenv("FWS_MUX_ZC_MAX");
    m->zc_max = zc ? strtoull(zc, nullptr, 10) : kMuxZcMax;
    for (uint32_t i = 0; i < n_conns; ++i) {
        fws_rx_session *s = new fws_rx_session();
        s->ctx = ctx;
        s->stream = m->stream;
        s->borrowed_stream = true;
        m->conns[i] = s;
    }
    *out = m;
    return 0;
}

// A chunk posted to the context's service, done. If that service is gone
// (fws_gpu_ctx_set_rx_persistent between submit and complete), its teardown
// drained the grid, which served the request and set the flag: the flag
// alone tells.
static int mux_wait_service(fws_rx_mux *m) {
    fws_rx_service *v = m->ctx->svc;
    if (v && v == m->sub_svc) return fws_rx_service_wait(v, m->hflag, m->sub_seq);
    return __atomic_load_n(m->hflag, __ATOMIC_ACQUIRE) == m->sub_seq ? 0 : fws_wait_flag(m->hflag, m->sub_seq, m->stream);
}

void fws_rx_mux_destroy(fws_rx_mux *m) {
    if (!m) return;
    if (m->inflight && m->wait == fws_rx_mux::kWaitService)   // a posted request: served before the buffers go
        (void)mux_wait_service(m);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    for (fws_rx_session *s : m->conns) fws_rx_session_destroy(s);
    if (m->hbuf) (void)hipHostFree(m->hbuf);
    if (m->dbuf) (void)hipFree(m->dbuf);
    if (m->hmeta) (void)hipHostFree(m->hmeta);
    if (m->dmeta) (void)hipFree(m->dmeta);
    if (m->dctr) (void)hipFree(m->dctr);
    if (m->hflag) (void)hipHostFree(m->hflag);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

int fws_rx_mux_reset(fws_rx_mux *m, uint32_t conn) {
    if (!m || conn >= m->conns.size()) return FWS_ERR_INVALID;
    m->conns[conn]->reset_state();
    return 0;
}

int fws_rx_mux_state(const fws_rx_mux *m, uint32_t conn, fws_rx_state *out) {
    if (!m || conn >= m->conns.size()) return FWS_ERR_INVALID;
    return fws_rx_session_state(m->conns[conn], out);
}

int fws_rx_mux_error(const fws_rx_mux *m, uint32_t conn, uint32_t *opcode) {
    if (!m || conn >= m->conns.size()) return FWS_ERR_INVALID;
    return fws_rx_session_error(m->conns[conn], opcode);
}

int fws_rx_mux_submit(fws_rx_mux *m, const fws_rx_read *reads, uint32_t n) {
    if (!m || (n && !reads) || m->inflight) return FWS_ERR_INVALID;
    for (uint32_t i = 0; i < n; ++i) {
        const fws_rx_read &rd = reads[i];
        if (rd.conn >= m->conns.size() || (rd.size && !rd.buf) || m->seen[rd.conn]) {
            for (uint32_t j = 0; j < i; ++j) m->seen[reads[j].conn] = 0;
            return FWS_ERR_INVALID;              // unknown connection, or two reads of one in a call
        }
        m->seen[rd.conn] = 1;
    }
    for (uint32_t i = 0; i < n; ++i) m->seen[reads[i].conn] = 0;
    int r;
    if ((r = fws_hip_status(hipSetDevice(m->ctx->device)))) return r;

    // 1. plan: per read its continuation, header stream and frame slots
    using Plan = fws_rx_mux::Plan;
    std::vector<Plan> &plan = m->sub_plan;
    plan.resize(n);
    uint64_t bytes = 0, frames = 0;
    uint32_t nseg = 0;
    for (uint32_t i = 0; i < n; ++i) {
        fws_rx_session *s = m->conns[reads[i].conn];
        Plan &p = plan[i];
        const uint64_t size = reads[i].size;
        p.u = s->recv_status == kWaitPayload ? (size < s->unread ? size : s->unread) : 0;
        p.part0 = s->part_len;
        p.rest = size - p.u;
        p.L = p.rest ? p.part0 + p.rest : 0;
        p.seg = kNone;
        p.dev = nullptr;
        if (size == 0 || size > kMuxMaxRead || p.L > kSmallMax) continue;
        // in place when the read lies in registered host memory, needs no staged
        // header bytes, starts on the kernels' 16-B chunk grid and is either all
        // continuation or all header stream (a declined header stream is decoded
        // again by the session path, which must see the continuation still masked)
        uint8_t *dv = p.part0 == 0 && (p.u == 0 || p.rest == 0) ? fws_host_alias(reads[i].buf, size) : nullptr;
        if (dv && ((uintptr_t)dv & 15u) == 0) {
            p.dev = dv;
        } else {
            p.cont_off = bytes;
            p.hs_off = al16(bytes + p.u);
            bytes = al16(p.hs_off + p.L) + 16;   // + 16: the small decode reads one chunk past L
        }
        p.seg = nseg++;
        frames += p.L / 6 + 2 < kSmallFrames ? p.L / 6 + 2 : kSmallFrames;
    }
    const uint64_t desc_bytes = al16((uint64_t)nseg * sizeof(fws_seg_desc));
    const uint64_t res_bytes = al16((uint64_t)nseg * sizeof(fws_decode_result));
    fws_rx_mux::Wait wait = fws_rx_mux::kWaitNone;
    if (nseg) {
        if ((r = m->ensure(bytes ? bytes : 16, desc_bytes + res_bytes + frames * sizeof(fws_frame_info)))) return r;
        fws_seg_desc *hd = (fws_seg_desc *)m->hmeta;
        // the kernel's base: the pinned staging (zero-copy round) or its device copy
        const uintptr_t kbase = (uintptr_t)(bytes <= m->zc_max ? m->hbuf : m->dbuf);
        uint32_t fbase = 0;
        for (uint32_t i = 0; i < n; ++i) {
            const Plan &p = plan[i];
            if (p.seg == kNone) continue;
            fws_rx_session *s = m->conns[reads[i].conn];
            const uint8_t *buf = reads[i].buf;
            fws_seg_desc &d = hd[p.seg];
            if (p.dev) {                         // offsets from the base, modulo 2^64
                d.cont_off = (uint64_t)((uintptr_t)p.dev - kbase);
                d.hs_off = (uint64_t)((uintptr_t)(p.dev + p.u) - kbase);
            } else {
                if (p.u) memcpy(m->hbuf + p.cont_off, buf, p.u);
                if (p.rest) {
                    if (p.part0) memcpy(m->hbuf + p.hs_off, s->hdr, p.part0);
                    memcpy(m->hbuf + p.hs_off + p.part0, buf + p.u, p.rest);
                }
                d.cont_off = p.cont_off;
                d.hs_off = p.hs_off;
            }
            d.u = (uint32_t)p.u;
            d.key = s->key;
            d.L = (uint32_t)p.L;
            d.fcap = (uint32_t)(p.L / 6 + 2 < kSmallFrames ? p.L / 6 + 2 : kSmallFrames);
            d.fbase = fbase;
            d.pad = 0;
            fbase += d.fcap;
        }
        // 2. one round trip, not waited for here: H2D, the segments' decode, D2H --
        // or for a small batch the decode alone, on the pinned buffers
        hipStream_t st = m->stream;
        hipError_t e;
        if (bytes <= m->zc_max) {
            fws_decode_result *hr = (fws_decode_result *)(m->hmeta + desc_bytes);
            fws_frame_info *hf = (fws_frame_info *)(m->hmeta + desc_bytes + res_bytes);
            m->sub_seq = ++m->seq;
            // the resident grid when its workers cover the round (each takes its
            // segments one after another): 64 reads of 4 KiB took 36.3 us on 16
            // workers against 21.4 us for a launch with a workgroup per read
            // (tools/lat_feed.cpp, profiles/r05/lat_mux.jsonl)
            fws_rx_service *const v = fws_ctx_rx_service(m->ctx);
            if (v && nseg <= fws_rx_service_workers(v)) {
                if ((r = fws_rx_service_post(v, m->hbuf, (const fws_seg_desc *)m->hmeta, nseg, hf, hr, m->hflag,
                                             m->sub_seq)))
                    return r;
                wait = fws_rx_mux::kWaitService;
                m->sub_svc = v;
            } else {
                if ((r = fws_launch_decode_segments(m->hbuf, (const fws_seg_desc *)m->hmeta, nseg, hf, hr, st, m->dctr,
                                                    nseg, m->hflag, m->sub_seq)))
                    return r;
                wait = fws_rx_mux::kWaitFlag;
            }
        } else {
            fws_decode_result *dres = (fws_decode_result *)(m->dmeta + desc_bytes);
            fws_frame_info *dfr = (fws_frame_info *)(m->dmeta + desc_bytes + res_bytes);
            if ((e = hipMemcpyAsync(m->dbuf, m->hbuf, bytes, hipMemcpyHostToDevice, st)) != hipSuccess ||
                (e = hipMemcpyAsync(m->dmeta, m->hmeta, desc_bytes, hipMemcpyHostToDevice, st)) != hipSuccess)
                return fws_hip_status(e);
            if ((r = fws_launch_decode_segments(m->dbuf, (const fws_seg_desc *)m->dmeta, nseg, dfr, dres, st))) {
                (void)hipStreamSynchronize(st);  // nothing of this batch may still write the staging
                return r;
            }
            if ((e = hipMemcpyAsync(m->hbuf, m->dbuf, bytes, hipMemcpyDeviceToHost, st)) != hipSuccess ||
                (e = hipMemcpyAsync(m->hmeta + desc_bytes, m->dmeta + desc_bytes,
                                    res_bytes + frames * sizeof(fws_frame_info), hipMemcpyDeviceToHost, st)) != hipSuccess) {
                (void)hipStreamSynchronize(st);
                return fws_hip_status(e);
            }
            wait = fws_rx_mux::kWaitStream;
        }
    }
    m->sub_reads.assign(reads, reads + n);
    m->sub_desc_bytes = desc_bytes;
    m->sub_res_bytes = res_bytes;
    m->wait = wait;
    m->inflight = true;
    return 0;
}

int fws_rx_mux_ready(fws_rx_mux *m) {
    if (!m) return FWS_ERR_INVALID;
    if (!m->inflight) return 1;
    switch (m->wait) {
    case fws_rx_mux::kWaitService:                   // the grid (or its teardown) sets the flag last
    case fws_rx_mux::kWaitFlag: return __atomic_load_n(m->hflag, __ATOMIC_ACQUIRE) == m->sub_seq ? 1 : 0;
    case fws_rx_mux::kWaitStream: {
        const hipError_t e = hipStreamQuery(m->stream);
        return e == hipSuccess ? 1 : (e == hipErrorNotReady ? 0 : fws_hip_status(e));
    }
    case fws_rx_mux::kWaitNone: break;
    }
    return 1;
}

int fws_rx_mux_complete(fws_rx_mux *m, fws_rx_read_result *results) {
    if (!m || !m->inflight || (!m->sub_reads.empty() && !results)) return FWS_ERR_INVALID;
    m->inflight = false;
    int r = 0;
    switch (m->wait) {
    case fws_rx_mux::kWaitService: r = mux_wait_service(m); break;
    case fws_rx_mux::kWaitFlag: r = fws_wait_flag(m->hflag, m->sub_seq, m->stream); break;
    case fws_rx_mux::kWaitStream: r = fws_hip_status(hipStreamSynchronize(m->stream)); break;
    case fws_rx_mux::kWaitNone: break;
    }
    if (r) return r;

    // 3. per read: the bytes back, OnRecvData's bookkeeping, the events
    const uint32_t n = (uint32_t)m->sub_reads.size();
    const fws_rx_read *reads = m->sub_reads.data();
    const fws_rx_mux::Plan *plan = m->sub_plan.data();
    const uint64_t desc_bytes = m->sub_desc_bytes, res_bytes = m->sub_res_bytes;
    const fws_seg_desc *hd = (const fws_seg_desc *)m->hmeta;
    const fws_decode_result *hres = (const fws_decode_result *)(m->hmeta + desc_bytes);
    const fws_frame_info *hfr = (const fws_frame_info *)(m->hmeta + desc_bytes + res_bytes);
    for (uint32_t i = 0; i < n; ++i) {
        const fws_rx_read &rd = reads[i];
        const fws_rx_mux::Plan &p = plan[i];
        fws_rx_session *s = m->conns[rd.conn];
        s->own = true;
        s->own_ev.clear();
        s->own_ctl.clear();
        s->n_ev = 0;
        s->ctl_used = 0;
        s->err_code = 0;
        int ret;
        const fws_decode_result res = p.seg != kNone && p.rest ? hres[p.seg] : fws_decode_result{};
        if (p.seg == kNone || (p.rest && (res.status == FWS_SMALL_DECLINED || res.status == FWS_ERR_CAPACITY))) {
            ret = feed_impl(s, rd.buf, rd.size, rd.capacity);          // the session path, on the original bytes
        } else {
            if (!p.dev) {                                                // staged: the bytes back
                if (p.u) memcpy(rd.buf, m->hbuf + p.cont_off, p.u);
                if (p.rest) memcpy(rd.buf + p.u, m->hbuf + p.hs_off + p.part0, p.rest);
            }
            ret = replay(s, rd.buf, rd.size, rd.capacity, p.u, p.part0, p.rest, p.L, res, hfr + hd[p.seg].fbase);
        }
        if (ret < 0) s->err_code = ret;
        fws_rx_read_result &o = results[i];
        o.ret = ret;
        o.pad = 0;
        o.events = s->own_ev.data();
        o.n_events = s->own_ev.size();
        o.ctl = s->own_ctl.data();
        o.ctl_used = s->own_ctl.size();
        s->own = false;
    }
    return 0;
}

int fws_rx_mux_feed(fws_rx_mux *m, const fws_rx_read *reads, uint32_t n, fws_rx_read_result *results) {
    if (!m || (n && (!reads || !results))) return FWS_ERR_INVALID;
    const int r = fws_rx_mux_submit(m, reads, n);
    return r ? r : fws_rx_mux_complete(m, results);
}

}  // extern "C"
