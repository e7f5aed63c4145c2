// rx_service.cpp -- fws_rx_service: the host side of the persistent receive
// kernel (small_kernels.hip k_rx_service; protocol in fws_internal.h).
//
// A hooked read costs one kernel launch plus one PCIe round trip (DESIGN.md
// §4.5: ~6 us of a 4 KiB read's ~10 us). With the service the launch is gone
// from the steady state: the decode grid stays resident while reads keep
// coming (FLoop::OneStep's read loop, floop.h:661-703, hands over a read or a
// step's batch every few us), polls a mailbox in coherent pinned memory, and
// exits on its own after `linger` without a request -- so an idle process
// holds no CUs and no hardware queue, and the next request relaunches it.
// Requests are serialised per context (one mailbox); each is waited for by
// its flag before the next is published.
#include <string.h>

#include <chrono>
#include <mutex>

#include "fws_internal.h"

struct fws_rx_service {
    int device = 0;
    uint32_t workers = 0;
    uint64_t ticks_per_us = 100;      // wall_clock64 rate (s_memrealtime, 100 MHz on gfx9)
    hipStream_t stream = nullptr;
    fws_svc_mail *mail = nullptr;     // coherent pinned
    fws_svc_dev *dv = nullptr;
    std::mutex mu;
    uint64_t launches = 0, requests = 0;
};

namespace {
uint64_t g_linger_us = 250;            // idle time before the grid exits (tests shorten it)
constexpr uint64_t kLifeUs = 200000;   // and its longest stay: it leaves at the next idle moment
// phase trace (tools/lat_feed.cpp): the device's phase clocks (grids launched
// while it is on) and the host's publish / wait times, summed in ns
bool g_trace = false;
uint64_t g_host_ns[3];                 // requests, entry -> published, published -> flag seen
}  // namespace

// on: trace the grids launched from now on; out: [0..7] the device sums
// (small_kernels.hip g_svc_trace, wall-clock ticks), [8] ticks per us,
// [9..11] the host sums; every sum is zeroed after the copy
extern "C" __attribute__((visibility("default"))) int fws_internal_rx_service_trace(int on, int device,
                                                                                   unsigned long long *out12) {
    g_trace = on != 0;
    if (!out12) return 0;
    int r = fws_rx_service_trace_read(out12);
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess) khz = 0;
    out12[8] = (unsigned long long)khz / 1000u;
    for (int i = 0; i < 3; ++i) {
        out12[9 + i] = g_host_ns[i];
        g_host_ns[i] = 0;
    }
    return r;
}

extern "C" __attribute__((visibility("default"))) int fws_internal_set_rx_linger_us(int us) {
    const int old = (int)g_linger_us;
    if (us > 0) g_linger_us = (uint64_t)us;
    return old;
}

// launches and requests served by the context's service (tests)
extern "C" __attribute__((visibility("default"))) int fws_internal_rx_service_stats(fws_gpu_ctx *ctx,
                                                                                   uint64_t *out2) {
    if (!ctx || !out2) return FWS_ERR_INVALID;
    out2[0] = ctx->svc ? ctx->svc->launches : 0;
    out2[1] = ctx->svc ? ctx->svc->requests : 0;
    return 0;
}

fws_rx_service *fws_ctx_rx_service(fws_gpu_ctx *ctx) {
    if (!ctx || !ctx->svc_workers) return nullptr;
    if (ctx->svc) return ctx->svc;
    fws_rx_service *v = new fws_rx_service();
    v->device = ctx->device;
    v->workers = ctx->svc_workers;
    int khz = 0;
    bool ok = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device) == hipSuccess && khz > 0;
    if (ok) v->ticks_per_us = (uint64_t)khz / 1000u ? (uint64_t)khz / 1000u : 1u;
    ok = ok && hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipHostMalloc((void **)&v->mail, sizeof(fws_svc_mail), hipHostMallocCoherent) == hipSuccess;
    ok = ok && hipMalloc((void **)&v->dv, sizeof(fws_svc_dev)) == hipSuccess;
    if (!ok) {
        fws_rx_service_destroy(v);
        return nullptr;                // the per-read launch path stays in use
    }
    memset((void *)v->mail, 0, sizeof(fws_svc_mail));
    ctx->svc = v;
    return v;
}

void fws_rx_service_destroy(fws_rx_service *v) {
    if (!v) return;
    if (v->mail && v->stream) {
        std::lock_guard<std::mutex> lk(v->mu);
        uint64_t old = __atomic_load_n(&v->mail->state, __ATOMIC_ACQUIRE);
        if (old & 1u) {                // a grid is running: a quit request
            v->mail->req.kind = 1u;
            __atomic_store_n(&v->mail->tag, (old >> 1) + 1u, __ATOMIC_RELEASE);
            uint64_t e = old;
            (void)__atomic_compare_exchange_n(&v->mail->state, &e, (((old >> 1) + 1u) << 1) | 1u, false,
                                              __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);   // fails: it just stopped
        }
        (void)hipStreamSynchronize(v->stream);   // the grid has drained (quit or linger)
    }
    if (v->dv) (void)hipFree(v->dv);
    if (v->mail) (void)hipHostFree(v->mail);
    if (v->stream) (void)hipStreamDestroy(v->stream);
    delete v;
}

int fws_rx_service_run(fws_rx_service *v, uint8_t *base, const fws_seg_desc *descs, const fws_seg_desc *one,
                       uint32_t nseg, fws_frame_info *frames, fws_decode_result *res, uint32_t *flag,
                       uint32_t flag_seq) {
    if (!v || !nseg || !flag || (!descs && !one)) return FWS_ERR_INVALID;
    std::lock_guard<std::mutex> lk(v->mu);
    const bool tr = g_trace;
    std::chrono::steady_clock::time_point t0, t1;
    if (tr) t0 = std::chrono::steady_clock::now();
    fws_svc_req &q = v->mail->req;     // plain stores; the CAS / store below publishes them
    q.base = (uint64_t)(uintptr_t)base;
    q.descs = (uint64_t)(uintptr_t)descs;
    q.frames = (uint64_t)(uintptr_t)frames;
    q.res = (uint64_t)(uintptr_t)res;
    q.flag = (uint64_t)(uintptr_t)flag;
    q.nseg = nseg;
    q.flag_seq = flag_seq;
    q.kind = 0;
    if (!descs) q.one = *one;
    uint64_t old = __atomic_load_n(&v->mail->state, __ATOMIC_ACQUIRE);
    // the tag names the seq this request is published as (the poller reads the
    // line in one load and trusts the request only when the tag matches)
    __atomic_store_n(&v->mail->tag, (old >> 1) + 1u, __ATOMIC_RELEASE);
    bool published = false;
    if (old & 1u) {                    // a grid is running: hand it the request
        uint64_t e = old;
        published = __atomic_compare_exchange_n(&v->mail->state, &e, (((old >> 1) + 1u) << 1) | 1u, false,
                                                __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
        if (!published) old = e;       // it stopped in the meantime
    }
    ++v->requests;
    if (!published) {
        // no grid: publish the request as the next seq and launch one behind the
        // previous grid's exit (stream order), its device words zeroed first
        const uint32_t seq0 = (uint32_t)(old >> 1);
        __atomic_store_n(&v->mail->state, ((uint64_t)(seq0 + 1u) << 1) | 1u, __ATOMIC_SEQ_CST);
        int r = fws_hip_status(hipMemsetAsync(v->dv, 0, sizeof(fws_svc_dev), v->stream));
        if (!r)
            r = fws_launch_rx_service(v->mail, v->dv, seq0, v->workers, g_linger_us * v->ticks_per_us,
                                      kLifeUs * v->ticks_per_us, tr ? 1u : 0u, v->stream);
        if (r) {
            __atomic_store_n(&v->mail->state, (uint64_t)seq0 << 1, __ATOMIC_SEQ_CST);
            return r;
        }
        ++v->launches;
    }
    if (!tr) return fws_wait_flag(flag, flag_seq, v->stream);
    t1 = std::chrono::steady_clock::now();
    const int r = fws_wait_flag(flag, flag_seq, v->stream);
    const auto t2 = std::chrono::steady_clock::now();
    g_host_ns[0] += 1;
    g_host_ns[1] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    g_host_ns[2] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
    return r;
}

extern "C" {

int fws_gpu_ctx_set_rx_persistent(fws_gpu_ctx *ctx, uint32_t workers) {
    if (!ctx || workers > 1024u) return FWS_ERR_INVALID;
    int r = fws_hip_status(hipSetDevice(ctx->device));
    if (r) return r;
    if (ctx->svc && ctx->svc->workers != workers) {
        fws_rx_service_destroy(ctx->svc);
        ctx->svc = nullptr;
    }
    ctx->svc_workers = workers;
    return 0;
}

}  // extern "C"
