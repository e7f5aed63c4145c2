// rx_service.cpp -- fws_rx_service: the host side of the persistent receive
// kernel (small_kernels.hip k_rx_service; protocol in fws_internal.h).
//
// A hooked read costs one kernel launch plus one PCIe round trip (DESIGN.md
// §4.5: ~6 us of a 4 KiB read's ~10 us). With the service the launch is gone
// from the steady state: the decode grid stays resident while reads keep
// coming (FLoop::OneStep's read loop, floop.h:661-703, hands over a read or a
// step's batch every few us), polls a mailbox, and exits on its own after
// `linger` without a request -- so an idle process holds no CUs and no
// hardware queue, and the next request relaunches it. Requests are serialised
// per context (one mailbox); each is waited for by its flag before the next
// is published.
//
// Push mode (large-BAR devices): the mailbox the grid polls, and a staging
// area for one small read, live in fine-grained device memory that the CPU
// writes directly (write-combined stores, flushed by sfence). The grid then
// polls local memory instead of reading host memory over PCIe per poll, and a
// session's read arrives with its doorbell instead of being pulled by the
// kernel: a doorbell round trip of 3.05 against 4.85 us, and 3.44 against
// 5.99 us with 4 KiB pushed in and written back (tools/vram_probe.hip,
// profiles/r05/vram_probe.jsonl).
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>

#include "fws_internal.h"

struct fws_rx_service {
    int device = 0;
    uint32_t workers = 0;
    uint64_t ticks_per_us = 100;      // wall_clock64 rate (s_memrealtime, 100 MHz on gfx9)
    hipStream_t stream = nullptr;
    fws_svc_mail *mail = nullptr;     // coherent pinned: the running bit (and the request, pull mode)
    fws_svc_mail *vmail = nullptr;    // push mode: the polled line, in device memory (CPU-written only)
    uint8_t *vstage = nullptr;        // push mode: a pushed read's staging, after vmail
    bool push = false;
    fws_svc_dev *dv = nullptr;
    std::mutex mu;
    uint64_t launches = 0, requests = 0, pushes = 0;
    // a request published by fws_rx_service_post and not waited for yet: the
    // next request on the service waits for it first (one request at a time)
    uint32_t *pend_flag = nullptr;
    uint32_t pend_seq = 0;
};

namespace {
constexpr uint64_t kPushCap = (16u << 10) + 128u;   // a staged session read (kZcMax + pad + header bytes)
std::atomic<int> g_push{-1};           // -1: FWS_RX_PUSH (default on where the device has a large BAR)

// write-combined stores to device memory leave the CPU's buffers in order at a fence
inline void wc_flush() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_sfence();
#elif defined(__aarch64__)
    __asm__ __volatile__("dsb st" ::: "memory");
#else
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
#endif
}

std::atomic<uint64_t> g_linger_us{250};   // idle time before the grid exits (tests shorten it)
// the service stream's hardware queue. ROCclr keeps a pool of
// hardware queues per stream priority (GPU_MAX_HW_QUEUES each, 4 on the box)
// and maps streams onto them round robin; a queue shared by two streams runs
// its packets in order, so work queued there behind the resident grid would
// wait until the grid leaves (up to kLifeUs). 1 (default): a non-blocking
// stream of the highest priority -- a pool of its own, which the process's
// normal-priority streams (torch's, the pipes', the engine's) never share;
// 0: a plain non-blocking stream from the normal pool (r05); 2: a CU-masked
// stream (every CU: never pooled, but created blocking, so the legacy null
// stream waits for the lingering grid -- measured, not used).
std::atomic<int> g_svc_queue{1};
std::mutex g_create_mu;                   // ctx->svc is created once under it
constexpr uint64_t kLifeUs = 200000;   // and its longest stay: it leaves at the next idle moment
// phase trace (tools/lat_feed.cpp): the device's phase clocks (grids launched
// while it is on) and the host's publish / wait times, summed in ns
std::atomic<bool> g_trace{false};
std::atomic<uint64_t> g_host_ns[3];    // requests, entry -> published, published -> flag seen
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
    for (int i = 0; i < 3; ++i) out12[9 + i] = g_host_ns[i].exchange(0);
    return r;
}

extern "C" __attribute__((visibility("default"))) int fws_internal_set_rx_service_queue(int mode) {
    return g_svc_queue.exchange(mode >= 0 && mode <= 2 ? mode : 1);
}

extern "C" __attribute__((visibility("default"))) int fws_internal_set_rx_linger_us(int us) {
    const int old = (int)g_linger_us.load();
    if (us > 0) g_linger_us = (uint64_t)us;
    return old;
}

// launches and requests served by the context's service (tests); with a third
// word: the pushed reads among them
extern "C" __attribute__((visibility("default"))) int fws_internal_rx_service_stats(fws_gpu_ctx *ctx,
                                                                                   uint64_t *out2) {
    if (!ctx || !out2) return FWS_ERR_INVALID;
    out2[0] = ctx->svc ? ctx->svc->launches : 0;
    out2[1] = ctx->svc ? ctx->svc->requests : 0;
    return 0;
}
extern "C" __attribute__((visibility("default"))) int fws_internal_rx_service_pushes(fws_gpu_ctx *ctx,
                                                                                    uint64_t *out1) {
    if (!ctx || !out1) return FWS_ERR_INVALID;
    *out1 = ctx->svc ? ctx->svc->pushes : 0;
    return 0;
}

// push mode for services created from now on: 1 on (where the device has a
// large BAR), 0 off, -1 the FWS_RX_PUSH environment variable (default on)
extern "C" __attribute__((visibility("default"))) int fws_internal_set_rx_push(int on) {
    return g_push.exchange(on < 0 ? -1 : (on ? 1 : 0));
}

namespace {
// the service stream (g_svc_queue: 1 highest priority, 2 CU-masked, 0 pooled)
bool create_service_stream(fws_rx_service *v) {
    const int mode = g_svc_queue.load();
    if (mode == 1) {
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
            hipStreamCreateWithPriority(&v->stream, hipStreamNonBlocking, greatest) == hipSuccess)
            return true;
    } else if (mode == 2) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, v->device) == hipSuccess && cus > 0) {
            uint32_t mask[64] = {};
            const uint32_t words = ((uint32_t)cus + 31u) / 32u;
            if (words <= 64u) {
                for (int i = 0; i < cus; ++i) mask[i / 32] |= 1u << (i % 32);
                if (hipExtStreamCreateWithCUMask(&v->stream, words, mask) == hipSuccess) return true;
            }
        }
    }
    v->stream = nullptr;
    return hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) == hipSuccess;
}
}  // namespace

fws_rx_service *fws_ctx_rx_service(fws_gpu_ctx *ctx) {
    if (!ctx || !ctx->svc_workers) return nullptr;
    if (fws_rx_service *v = __atomic_load_n(&ctx->svc, __ATOMIC_ACQUIRE)) return v;
    // first use: created once (two threads feeding one context race here only)
    std::lock_guard<std::mutex> lk(g_create_mu);
    if (ctx->svc) return ctx->svc;
    fws_rx_service *v = new fws_rx_service();
    v->device = ctx->device;
    v->workers = ctx->svc_workers;
    int khz = 0;
    bool ok = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device) == hipSuccess && khz > 0;
    if (ok) v->ticks_per_us = (uint64_t)khz / 1000u ? (uint64_t)khz / 1000u : 1u;
    ok = ok && create_service_stream(v);
    ok = ok && hipHostMalloc((void **)&v->mail, sizeof(fws_svc_mail), hipHostMallocCoherent) == hipSuccess;
    ok = ok && hipMalloc((void **)&v->dv, sizeof(fws_svc_dev)) == hipSuccess;
    if (!ok) {
        fws_rx_service_destroy(v);
        return nullptr;                // the per-read launch path stays in use
    }
    memset((void *)v->mail, 0, sizeof(fws_svc_mail));
    int want = g_push;
    if (want < 0) {
        const char *e = getenv("FWS_RX_PUSH");
        want = !(e && e[0] == '0');
    }
    int large_bar = 0;
    if (want && hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, ctx->device) == hipSuccess &&
        large_bar) {
        void *p = nullptr;
        if (hipExtMallocWithFlags(&p, sizeof(fws_svc_mail) + kPushCap, hipDeviceMallocFinegrained) == hipSuccess) {
            // on the service's own stream: a device-wide synchronise would also wait for
            // every other stream, another context's resident grid included
            if (hipMemsetAsync(p, 0, sizeof(fws_svc_mail), v->stream) == hipSuccess &&
                hipStreamSynchronize(v->stream) == hipSuccess) {
                v->vmail = static_cast<fws_svc_mail *>(p);
                v->vstage = static_cast<uint8_t *>(p) + sizeof(fws_svc_mail);
                v->push = true;
            } else {
                (void)hipFree(p);      // pull mode
            }
        }
    }
    __atomic_store_n(&ctx->svc, v, __ATOMIC_RELEASE);
    return v;
}

uint32_t fws_rx_service_workers(const fws_rx_service *v) { return v ? v->workers : 0u; }

bool fws_rx_service_can_push(const fws_rx_service *v, uint64_t span) {
    return v && v->push && span <= kPushCap;
}

// Publishes the request written into line(v)->req as the next seq (tag, then
// the running bit's CAS on the pinned line; push mode: then the device line's
// state word) or launches a grid for it; the caller holds v->mu.
namespace {
fws_svc_mail *line(fws_rx_service *v) { return v->push ? v->vmail : v->mail; }

int publish(fws_rx_service *v, bool tr) {
    fws_svc_mail *const L = line(v);
    uint64_t old = __atomic_load_n(&v->mail->state, __ATOMIC_ACQUIRE);
    // the tag names the seq this request is published as (the poller reads the
    // line in one load and trusts the request only when the tag matches)
    if (v->push) {
        L->tag = (old >> 1) + 1u;
        wc_flush();                    // request, pushed bytes and tag before the state word
    } else {
        __atomic_store_n(&L->tag, (old >> 1) + 1u, __ATOMIC_RELEASE);
    }
    bool published = false;
    if (old & 1u) {                    // a grid is running: hand it the request
        uint64_t e = old;
        published = __atomic_compare_exchange_n(&v->mail->state, &e, (((old >> 1) + 1u) << 1) | 1u, false,
                                                __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST);
        if (!published) old = e;       // it stopped in the meantime (same seq, running bit clear)
    }
    const uint64_t next = (((old >> 1) + 1u) << 1) | 1u;
    if (published) {
        if (v->push) {                 // the running grid polls the device line
            L->state = next;
            wc_flush();
        }
        return 0;
    }
    // no grid: publish the request as the next seq and launch one behind the
    // previous grid's exit (stream order), its device words zeroed first
    const uint32_t seq0 = (uint32_t)(old >> 1);
    if (v->push) {
        L->state = next;
        wc_flush();
    }
    __atomic_store_n(&v->mail->state, next, __ATOMIC_SEQ_CST);
    int r = fws_hip_status(hipMemsetAsync(v->dv, 0, sizeof(fws_svc_dev), v->stream));
    if (!r)
        r = fws_launch_rx_service(v->mail, line(v), v->dv, seq0, v->workers, g_linger_us * v->ticks_per_us,
                                  kLifeUs * v->ticks_per_us, tr ? 1u : 0u, v->stream);
    if (r) {
        __atomic_store_n(&v->mail->state, (uint64_t)seq0 << 1, __ATOMIC_SEQ_CST);
        if (v->push) {
            L->state = (uint64_t)seq0 << 1;
            wc_flush();
        }
        return r;
    }
    ++v->launches;
    return 0;
}

// A request's flag. Not fws_wait_flag: its fallback after 200 us blocks on
// the stream, and the service stream stays busy while the grid lingers (up
// to kLifeUs), so a long request would be seen done only when the grid left.
// Here the spin turns into a polling sleep, and the stream is only queried:
// idle with the flag unset means the grid died or never ran (an error).
int wait_flag_svc(fws_rx_service *v, const uint32_t *flag, uint32_t seq) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0;; ++i) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return 0;
        if ((i & 255u) == 255u && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) break;
#if defined(__x86_64__) || defined(__i386__)
        __builtin_ia32_pause();
#endif
    }
    for (;;) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq) return 0;
        const hipError_t q = hipStreamQuery(v->stream);
        if (q == hipSuccess)                // the grid has left
            return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == seq ? 0 : FWS_ERR_INTERNAL;
        if (q != hipErrorNotReady) return fws_hip_status(q);
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// the posted request, if any, done (caller holds v->mu)
int drain(fws_rx_service *v) {
    if (!v->pend_flag) return 0;
    uint32_t *const f = v->pend_flag;
    v->pend_flag = nullptr;
    return wait_flag_svc(v, f, v->pend_seq);
}

int wait_traced(fws_rx_service *v, uint32_t *flag, uint32_t flag_seq, bool tr,
                std::chrono::steady_clock::time_point t0) {
    if (!tr) return wait_flag_svc(v, flag, flag_seq);
    const auto t1 = std::chrono::steady_clock::now();
    const int r = wait_flag_svc(v, flag, flag_seq);
    const auto t2 = std::chrono::steady_clock::now();
    g_host_ns[0].fetch_add(1, std::memory_order_relaxed);
    g_host_ns[1].fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count(),
                           std::memory_order_relaxed);
    g_host_ns[2].fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count(),
                           std::memory_order_relaxed);
    return r;
}
}  // namespace

void fws_rx_service_destroy(fws_rx_service *v) {
    if (!v) return;
    if (v->mail && v->stream) {
        std::lock_guard<std::mutex> lk(v->mu);
        (void)drain(v);                // a posted request is served before the quit
        const uint64_t old = __atomic_load_n(&v->mail->state, __ATOMIC_ACQUIRE);
        if (old & 1u) {                // a grid is running: a quit request
            fws_svc_mail *const L = line(v);
            L->req.kind = 1u;
            if (v->push) {
                L->tag = (old >> 1) + 1u;
                wc_flush();
            } else {
                __atomic_store_n(&L->tag, (old >> 1) + 1u, __ATOMIC_RELEASE);
            }
            uint64_t e = old;
            if (__atomic_compare_exchange_n(&v->mail->state, &e, (((old >> 1) + 1u) << 1) | 1u, false,
                                            __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST) &&
                v->push) {             // (a failed CAS: it just stopped)
                L->state = (((old >> 1) + 1u) << 1) | 1u;
                wc_flush();
            }
        }
        (void)hipStreamSynchronize(v->stream);   // the grid has drained (quit or linger)
    }
    if (v->dv) (void)hipFree(v->dv);
    if (v->vmail) (void)hipFree(v->vmail);
    if (v->mail) (void)hipHostFree(v->mail);
    if (v->stream) (void)hipStreamDestroy(v->stream);
    delete v;
}

namespace {
// the request of fws_rx_service_run / _post into the polled line (caller holds v->mu)
void fill_run(fws_rx_service *v, uint8_t *base, const fws_seg_desc *descs, const fws_seg_desc *one, uint32_t nseg,
              fws_frame_info *frames, fws_decode_result *res, uint32_t *flag, uint32_t flag_seq) {
    fws_svc_req &q = line(v)->req;     // plain stores; publish() orders them before the state word
    q.base = (uint64_t)(uintptr_t)base;
    q.descs = (uint64_t)(uintptr_t)descs;
    q.frames = (uint64_t)(uintptr_t)frames;
    q.res = (uint64_t)(uintptr_t)res;
    q.flag = (uint64_t)(uintptr_t)flag;
    q.out = 0;
    q.nseg = nseg;
    q.flag_seq = flag_seq;
    q.kind = 0;
    q.span = 0;
    if (!descs) q.one = *one;
    ++v->requests;
}
}  // namespace

int fws_rx_service_run(fws_rx_service *v, uint8_t *base, const fws_seg_desc *descs, const fws_seg_desc *one,
                       uint32_t nseg, fws_frame_info *frames, fws_decode_result *res, uint32_t *flag,
                       uint32_t flag_seq) {
    if (!v || !nseg || !flag || (!descs && !one)) return FWS_ERR_INVALID;
    std::lock_guard<std::mutex> lk(v->mu);
    if (int r = drain(v)) return r;
    const bool tr = g_trace;
    std::chrono::steady_clock::time_point t0;
    if (tr) t0 = std::chrono::steady_clock::now();
    fill_run(v, base, descs, one, nseg, frames, res, flag, flag_seq);
    if (int r = publish(v, tr)) return r;
    return wait_traced(v, flag, flag_seq, tr, t0);
}

int fws_rx_service_post(fws_rx_service *v, uint8_t *base, const fws_seg_desc *descs, uint32_t nseg,
                        fws_frame_info *frames, fws_decode_result *res, uint32_t *flag, uint32_t flag_seq) {
    if (!v || !nseg || !flag || !descs) return FWS_ERR_INVALID;
    std::lock_guard<std::mutex> lk(v->mu);
    if (int r = drain(v)) return r;
    fill_run(v, base, descs, nullptr, nseg, frames, res, flag, flag_seq);
    if (int r = publish(v, false)) return r;
    v->pend_flag = flag;
    v->pend_seq = flag_seq;
    return 0;
}

int fws_rx_service_wait(fws_rx_service *v, uint32_t *flag, uint32_t flag_seq) {
    if (!v || !flag) return FWS_ERR_INVALID;
    std::lock_guard<std::mutex> lk(v->mu);
    if (v->pend_flag == flag && v->pend_seq == flag_seq) return drain(v);
    // drained by a later request already: its flag is set
    return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == flag_seq ? 0 : wait_flag_svc(v, flag, flag_seq);
}

int fws_rx_service_push(fws_rx_service *v, const uint8_t *src, uint64_t span, uint8_t *out_dev, const fws_seg_desc &d,
                        fws_frame_info *frames, fws_decode_result *res, uint32_t *flag, uint32_t flag_seq) {
    if (!fws_rx_service_can_push(v, span) || !flag || !out_dev || (span && !src)) return FWS_ERR_INVALID;
    std::lock_guard<std::mutex> lk(v->mu);
    if (int r = drain(v)) return r;
    const bool tr = g_trace;
    std::chrono::steady_clock::time_point t0;
    if (tr) t0 = std::chrono::steady_clock::now();
    memcpy(v->vstage, src, span);      // the push: write-combined stores, flushed in publish()
    fws_svc_req &q = v->vmail->req;
    q.base = (uint64_t)(uintptr_t)v->vstage;
    q.descs = 0;
    q.frames = (uint64_t)(uintptr_t)frames;
    q.res = (uint64_t)(uintptr_t)res;
    q.flag = (uint64_t)(uintptr_t)flag;
    q.out = (uint64_t)(uintptr_t)out_dev;
    q.nseg = 1;
    q.flag_seq = flag_seq;
    q.kind = 2u;
    q.span = (uint32_t)span;
    q.one = d;
    ++v->requests;
    ++v->pushes;
    if (int r = publish(v, tr)) return r;
    return wait_traced(v, flag, flag_seq, tr, t0);
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
