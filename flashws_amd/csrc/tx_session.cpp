// tx_session.cpp -- fws_tx_session: WSocket::SendFrame (net/w_socket.h:832-944)
// for host payloads, the frame bytes built on the GPU.
//
// One call takes a connection's next n frames in order. The host does what
// SendFrame does outside the byte work: the opcode / FIN sequencing of the
// connection (last_msg_not_fin_, w_socket.h:845-848, 903-913, carried across
// calls) and the frame sizes (GetTxWSFrameHdrSize, w_socket.h:49-65). The
// payloads are gathered into a pinned staging buffer, copied to HBM with the
// descriptors, framed and masked by fws_gpu_encode_frames in one launch
// sequence, and the wire bytes come back into the caller's buffer. Host code.
#include <string.h>

#include <vector>

#include "fws_internal.h"

namespace {

inline uint64_t tx_hdr_size(uint64_t len, bool masked) {       // w_socket.h:49-65
    return 2u + (masked ? 4u : 0u) + (len < 126u ? 0u : (len <= 65535u ? 2u : 8u));
}

}  // namespace

struct fws_tx_session {
    fws_gpu_ctx *ctx = nullptr;
    hipStream_t stream = nullptr;
    bool is_server = false;
    uint8_t last_msg_not_fin = 0;                       // w_socket.h:903-913
    // pinned host staging and device buffers (grown on demand)
    uint8_t *h_src = nullptr, *h_out = nullptr;
    uint64_t h_src_cap = 0, h_out_cap = 0;
    fws_tx_desc *h_desc = nullptr;
    uint64_t h_desc_cap = 0;
    uint8_t *d_src = nullptr, *d_out = nullptr;
    uint64_t d_src_cap = 0, d_out_cap = 0;
    fws_tx_desc *d_desc = nullptr;
    uint64_t d_desc_cap = 0;
    uint64_t *d_len = nullptr;

    ~fws_tx_session() {
        if (h_src) (void)hipHostFree(h_src);
        if (h_out) (void)hipHostFree(h_out);
        if (h_desc) (void)hipHostFree(h_desc);
        if (d_src) (void)hipFree(d_src);
        if (d_out) (void)hipFree(d_out);
        if (d_desc) (void)hipFree(d_desc);
        if (d_len) (void)hipFree(d_len);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

template <typename T>
int grow_host(T **p, uint64_t *cap, uint64_t want) {
    if (want <= *cap && *p) return 0;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    const uint64_t n = want < 4096 ? 4096 : want + want / 4;
    int r = fws_hip_status(hipHostMalloc((void **)p, n * sizeof(T), hipHostMallocDefault));
    if (r == 0) *cap = n;
    return r;
}

template <typename T>
int grow_dev(T **p, uint64_t *cap, uint64_t want) {
    if (want <= *cap && *p) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const uint64_t n = want < 4096 ? 4096 : want + want / 4;
    int r = fws_hip_status(hipMalloc((void **)p, n * sizeof(T)));
    if (r == 0) *cap = n;
    return r;
}

}  // namespace

extern "C" {

int fws_tx_session_create(fws_gpu_ctx *ctx, int is_server, fws_tx_session **out) {
    if (!ctx || !out) return FWS_ERR_INVALID;
    *out = nullptr;
    int r = fws_hip_status(hipSetDevice(ctx->device));
    if (r) return r;
    fws_tx_session *s = new fws_tx_session();
    s->ctx = ctx;
    s->is_server = is_server != 0;
    if ((r = fws_hip_status(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking))) ||
        (r = fws_hip_status(hipMalloc((void **)&s->d_len, 16)))) {
        delete s;
        return r;
    }
    *out = s;
    return 0;
}

void fws_tx_session_destroy(fws_tx_session *s) { delete s; }

int fws_tx_session_send(fws_tx_session *s, const uint8_t *const *payloads, const uint64_t *lens,
                        const uint32_t *frame_types, const uint8_t *last, const uint32_t *keys, uint32_t n,
                        uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    if (!s || !out_len || (n && (!payloads || !lens || !frame_types || !last))) return FWS_ERR_INVALID;
    if (!s->is_server && n && !keys) return FWS_ERR_INVALID;
    *out_len = 0;
    if (n == 0) return 0;
    const bool masked = !s->is_server;
    uint64_t total = 0, src_total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (lens[i] && !payloads[i]) return FWS_ERR_INVALID;
        if (lens[i] > (1ull << 32)) return FWS_ERR_TOO_LARGE;   // MAX_WS_FRAME_SIZE, constants.h
        total += tx_hdr_size(lens[i], masked) + lens[i];
        src_total += lens[i];
    }
    *out_len = total;
    if (total > out_cap || (total && !out)) return FWS_ERR_CAPACITY;   // nothing sent, state unchanged
    int r;
    if ((r = fws_hip_status(hipSetDevice(s->ctx->device)))) return r;
    if ((r = grow_host(&s->h_src, &s->h_src_cap, src_total + 16)) || (r = grow_host(&s->h_out, &s->h_out_cap, total)) ||
        (r = grow_host(&s->h_desc, &s->h_desc_cap, n)) || (r = grow_dev(&s->d_src, &s->d_src_cap, src_total + 16)) ||
        (r = grow_dev(&s->d_out, &s->d_out_cap, total + 16)) || (r = grow_dev(&s->d_desc, &s->d_desc_cap, n)))
        return r;
    // sequencing and gather (the host side of SendFrame)
    uint8_t state = s->last_msg_not_fin;
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        fws_tx_desc &d = s->h_desc[i];
        fws_tx_next(frame_types[i], last[i], &state, &d.opcode, &d.fin);
        d.src_off = pos;
        d.len = lens[i];
        d.key = masked ? keys[i] : 0u;
        d.masked = masked ? 1 : 0;
        d.pad = 0;
        if (lens[i]) memcpy(s->h_src + pos, payloads[i], lens[i]);
        pos += lens[i];
    }
    hipStream_t st = s->stream;
    if ((r = fws_hip_status(hipMemcpyAsync(s->d_src, s->h_src, src_total ? src_total : 1, hipMemcpyHostToDevice, st))) ||
        (r = fws_hip_status(
             hipMemcpyAsync(s->d_desc, s->h_desc, (size_t)n * sizeof(fws_tx_desc), hipMemcpyHostToDevice, st))))
        return r;
    if ((r = fws_gpu_encode_frames(s->ctx, s->d_out, total, s->d_src, s->d_desc, n, s->d_len, st))) return r;
    if ((r = fws_hip_status(hipMemcpyAsync(s->h_out, s->d_out, total, hipMemcpyDeviceToHost, st))) ||
        (r = fws_hip_status(hipStreamSynchronize(st))))
        return r;
    memcpy(out, s->h_out, total);
    s->last_msg_not_fin = state;
    return 0;
}

int fws_tx_session_state(const fws_tx_session *s, uint8_t *last_msg_not_fin) {
    if (!s || !last_msg_not_fin) return FWS_ERR_INVALID;
    *last_msg_not_fin = s->last_msg_not_fin;
    return 0;
}

}  // extern "C"
