// rx_pipe.cpp -- fws_rx_pipe: batched, pipelined receive decode over host
// memory (the socket-side batching around FLoop::OneStep,
// floop.h:661-703, and the MemPool read blocks, flash_alloc.h:44-73).
//
// A server aggregates the reads of one event-loop step (many <= 2 MiB
// TCPSocket::Read buffers, tcp_socket.h:387-402) into one host batch and
// submits it; the pipe runs H2D copy -> fws_gpu_decode_stream (parallel header
// parse + unmask, optional UTF-8 flags) -> D2H copy of the unmasked bytes, the
// frame list and the result, on one of `depth` slots. Each slot owns a HIP
// stream, its device buffers and its own decode context, so batch i+1's H2D
// overlaps batch i's decode and D2H (PCIe is full duplex; copy engines run
// beside the compute queue). fws_rx_pipe_wait returns a batch's host-side
// results once its slot's event has completed. A submit into a busy slot
// waits for that slot first (back-pressure).
//
// The caller's batch buffer must stay valid until its wait returns; pinned
// memory (fws_gpu_host_register on a MemPool block, or hipHostMalloc) is
// needed for the copies to be asynchronous.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "fws_internal.h"

struct fws_rx_pipe_slot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    fws_gpu_ctx *ctx = nullptr;
    uint8_t *dwire = nullptr;
    fws_frame_info *dframes = nullptr;
    fws_decode_result *dres = nullptr;
    uint8_t *dutf8 = nullptr;
    fws_frame_info *hframes = nullptr;     // pinned
    fws_decode_result *hres = nullptr;     // pinned
    uint8_t *hutf8 = nullptr;              // pinned
    uint64_t ticket = ~0ull;               // batch in flight (or last completed)
    uint64_t copied = 0;                   // frame records (and flags) copied back with the batch
    bool busy = false;
};

struct fws_rx_pipe {
    int device = 0;
    uint64_t max_bytes = 0;
    uint32_t max_frames = 0;
    uint64_t est = 0;                      // frame records to copy back with the next batch
    bool utf8 = false;
    uint64_t next = 0;
    std::vector<fws_rx_pipe_slot> slots;
};

static void free_slot(fws_rx_pipe_slot &s) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.dwire) (void)hipFree(s.dwire);
    if (s.dframes) (void)hipFree(s.dframes);
    if (s.dres) (void)hipFree(s.dres);
    if (s.dutf8) (void)hipFree(s.dutf8);
    if (s.hframes) (void)hipHostFree(s.hframes);
    if (s.hres) (void)hipHostFree(s.hres);
    if (s.hutf8) (void)hipHostFree(s.hutf8);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.ctx) fws_gpu_ctx_destroy(s.ctx);
    s = fws_rx_pipe_slot{};
}

// Host ranges registered through fws_gpu_host_register (caller memory the GPU
// may read and write in place, e.g. the reference's MemPool read buffers), for
// the RX session and mux: a read that lies inside one is decoded where it is,
// without the pinned staging copies (fws_host_alias).
namespace {
struct HostRange {
    const uint8_t *host;
    uint64_t bytes;
    uint8_t *dev;
};
std::mutex g_reg_mu;
std::vector<HostRange> g_reg;          // sorted by host, disjoint
}  // namespace

void fws_host_registry_add(const uint8_t *host, uint64_t bytes, uint8_t *dev) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    const HostRange r{host, bytes, dev};
    g_reg.insert(std::upper_bound(g_reg.begin(), g_reg.end(), r,
                                  [](const HostRange &a, const HostRange &b) { return a.host < b.host; }),
                 r);
}

void fws_host_registry_remove(const uint8_t *host) {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    g_reg.erase(std::remove_if(g_reg.begin(), g_reg.end(), [&](const HostRange &r) { return r.host == host; }),
                g_reg.end());
}

uint8_t *fws_host_alias(const void *p, uint64_t n) {
    const uint8_t *q = (const uint8_t *)p;
    std::lock_guard<std::mutex> lk(g_reg_mu);
    auto it = std::upper_bound(g_reg.begin(), g_reg.end(), q,
                               [](const uint8_t *x, const HostRange &r) { return x < r.host; });
    if (it == g_reg.begin()) return nullptr;
    --it;
    const uint64_t off = (uint64_t)(q - it->host);
    if (q < it->host || off > it->bytes || n > it->bytes - off) return nullptr;
    return it->dev + off;
}

extern "C" {

int fws_gpu_host_register(void *host_ptr, uint64_t bytes) {
    if (!host_ptr || !bytes) return FWS_ERR_INVALID;
    hipError_t e = hipHostRegister(host_ptr, bytes, hipHostRegisterMapped);
    if (e != hipSuccess) return fws_hip_status(e);
    void *dev = nullptr;
    if ((e = hipHostGetDevicePointer(&dev, host_ptr, 0)) != hipSuccess || !dev) {
        (void)hipHostUnregister(host_ptr);
        return fws_hip_status(e != hipSuccess ? e : hipErrorInvalidValue);
    }
    fws_host_registry_add((const uint8_t *)host_ptr, bytes, (uint8_t *)dev);
    return 0;
}

int fws_gpu_host_unregister(void *host_ptr) {
    if (!host_ptr) return FWS_ERR_INVALID;
    fws_host_registry_remove((const uint8_t *)host_ptr);
    return fws_hip_status(hipHostUnregister(host_ptr));
}

void fws_rx_pipe_destroy(fws_rx_pipe *p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    for (auto &s : p->slots) free_slot(s);
    delete p;
}

int fws_rx_pipe_create(int device, uint64_t max_batch_bytes, uint32_t max_frames, uint32_t depth, int utf8,
                       fws_rx_pipe **out) {
    if (!out || depth == 0 || depth > 16 || max_batch_bytes == 0 || max_frames == 0) return FWS_ERR_INVALID;
    *out = nullptr;
    fws_rx_pipe *p = new fws_rx_pipe();
    p->device = device;
    p->max_bytes = max_batch_bytes;
    p->max_frames = max_frames;
    p->est = max_frames;
    p->utf8 = utf8 != 0;
    p->slots.resize(depth);
    int r = 0;
    for (auto &s : p->slots) {
        if ((r = fws_gpu_ctx_create(device, &s.ctx))) break;
        if ((r = fws_gpu_ctx_reserve(s.ctx, max_frames, max_batch_bytes))) break;
        hipError_t e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, hipEventDisableTiming);
        if (e == hipSuccess) e = hipMalloc((void **)&s.dwire, (max_batch_bytes + 15) & ~uint64_t(15));
        if (e == hipSuccess) e = hipMalloc((void **)&s.dframes, (uint64_t)max_frames * sizeof(fws_frame_info));
        if (e == hipSuccess) e = hipMalloc((void **)&s.dres, sizeof(fws_decode_result));
        if (e == hipSuccess) e = hipHostMalloc((void **)&s.hframes, (uint64_t)max_frames * sizeof(fws_frame_info));
        if (e == hipSuccess) e = hipHostMalloc((void **)&s.hres, sizeof(fws_decode_result));
        if (e == hipSuccess && p->utf8) e = hipMalloc((void **)&s.dutf8, max_frames);
        if (e == hipSuccess && p->utf8) e = hipHostMalloc((void **)&s.hutf8, max_frames);
        if ((r = fws_hip_status(e))) break;
    }
    if (r) {
        fws_rx_pipe_destroy(p);
        return r;
    }
    *out = p;
    return 0;
}

// Enqueue one batch (host bytes, unmasked in place once its wait returns).
int fws_rx_pipe_submit(fws_rx_pipe *p, uint8_t *batch, uint64_t len, uint64_t *ticket) {
    if (!p || !ticket || (len && !batch) || len > p->max_bytes) return FWS_ERR_INVALID;
    int r = fws_hip_status(hipSetDevice(p->device));
    if (r) return r;
    const uint64_t t = p->next;
    fws_rx_pipe_slot &s = p->slots[t % p->slots.size()];
    if (s.busy && (r = fws_hip_status(hipEventSynchronize(s.done)))) return r;   // back-pressure
    s.busy = true;
    s.ticket = t;
    hipError_t e = hipSuccess;
    if (len) e = hipMemcpyAsync(s.dwire, batch, len, hipMemcpyHostToDevice, s.stream);
    if ((r = fws_hip_status(e))) return r;
    if ((r = fws_gpu_decode_stream(s.ctx, s.dwire, len, s.dframes, p->max_frames, s.dres, s.dutf8, s.stream)))
        return r;
    if (len) e = hipMemcpyAsync(batch, s.dwire, len, hipMemcpyDeviceToHost, s.stream);
    // the frame list: the count is on the device until the wait, so a bounded
    // guess of it comes back with the batch (every frame has >= 6 header bytes;
    // the last batch's count plus a margin) and the wait copies any remainder
    uint64_t k = len / 6 + 1;
    if (k > p->est) k = p->est;
    if (k > p->max_frames) k = p->max_frames;
    s.copied = k;
    if (e == hipSuccess && k)
        e = hipMemcpyAsync(s.hframes, s.dframes, k * sizeof(fws_frame_info), hipMemcpyDeviceToHost, s.stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(s.hres, s.dres, sizeof(fws_decode_result), hipMemcpyDeviceToHost, s.stream);
    if (e == hipSuccess && p->utf8 && k)
        e = hipMemcpyAsync(s.hutf8, s.dutf8, k, hipMemcpyDeviceToHost, s.stream);
    if (e == hipSuccess) e = hipEventRecord(s.done, s.stream);
    if ((r = fws_hip_status(e))) return r;
    *ticket = t;
    p->next = t + 1;
    return 0;
}

// Wait for a submitted batch; its host-side results stay valid until the slot
// is reused (depth submits later).
int fws_rx_pipe_wait(fws_rx_pipe *p, uint64_t ticket, const fws_frame_info **frames, uint64_t *n_frames,
                     fws_decode_result *result, const uint8_t **utf8_ok) {
    if (!p || ticket >= p->next) return FWS_ERR_INVALID;
    fws_rx_pipe_slot &s = p->slots[ticket % p->slots.size()];
    if (s.ticket != ticket) return FWS_ERR_INVALID;             // slot already reused
    int r = fws_hip_status(hipEventSynchronize(s.done));
    if (r) return r;
    s.busy = false;
    const uint64_t n = s.hres->n_frames < p->max_frames ? s.hres->n_frames : p->max_frames;
    if (n > s.copied) {                                         // the guess fell short: the rest
        if ((r = fws_hip_status(hipSetDevice(p->device)))) return r;
        hipError_t e = hipMemcpyAsync(s.hframes + s.copied, s.dframes + s.copied,
                                      (n - s.copied) * sizeof(fws_frame_info), hipMemcpyDeviceToHost, s.stream);
        if (e == hipSuccess && p->utf8)
            e = hipMemcpyAsync(s.hutf8 + s.copied, s.dutf8 + s.copied, n - s.copied, hipMemcpyDeviceToHost, s.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(s.stream);
        if ((r = fws_hip_status(e))) return r;
        s.copied = n;
    }
    p->est = n + n / 8 + 64;
    if (result) *result = *s.hres;
    if (frames) *frames = s.hframes;
    if (n_frames) *n_frames = n;
    if (utf8_ok) *utf8_ok = s.hutf8;
    return 0;
}

}  // extern "C"
