// decode_engine.cpp -- fws_decode_engine: fws_gpu_decode_stream over many
// independent streams, pipelined on one device.
//
// A stream decode is two passes over the wire with a latency-bound resolve
// between them: k_scan (66 us on C3, ~4 TB/s of reads, VALU issue ~49 us of
// it), then k_merge -> k_link -> k_emit (~39 us of dependent round trips with
// few waves), then k_unmask_stream (HBM-bound). One call leaves the HBM mostly
// idle during the resolve. The engine keeps decodes in flight on two HIP
// streams, each with its own workspaces (a private fws_gpu_ctx per job slot),
// so one job's resolve overlaps another's streaming kernels.
//
// Schedules (fws_internal_set_engine_mode, measured on MI355X C3 batches,
// profiles/r04/engine/):
//   0 (default)  job j's whole decode on stream j % 2: 0.165 ms per batch (C3,
//                16 jobs per run; the bench's two contexts on two streams:
//                0.158-0.161).
//   1            split phases: every scan on stream X, every resolve + unmask
//                on stream Y, three jobs in flight (Y waits for scan(j), X
//                waits for job j's unmask before reusing its workspace for
//                j + 3): 0.201 ms -- a scan running beside an unmask slows
//                both (k_scan's own reads run at ~4 TB/s, so the two are not
//                issue- and HBM-bound complements), and the scans ahead of
//                the resolve take the CUs the unmask needs.
//   1 + CU partition (fws_internal_set_engine_scan_cus: X on that many CUs
//                spread over the index range, Y on the rest): 0.29-0.39 ms.
#include <hip/hip_runtime.h>

#include <cstring>
#include <new>

#include "fws_internal.h"

namespace {

constexpr int kSlots = 3;                  // workspaces (decodes in flight)

int g_engine_mode = 0;                     // tuning hook: the schedule (header comment)
uint32_t g_engine_scan_cus = 0;            // tuning hook: mode 1's CU partition (0: none)

}  // namespace

extern "C" __attribute__((visibility("default"))) int fws_internal_set_engine_mode(int m) {
    const int old = g_engine_mode;
    if (m == 0 || m == 1) g_engine_mode = m;
    return old;
}
extern "C" __attribute__((visibility("default"))) int fws_internal_set_engine_scan_cus(int cus) {
    const int old = (int)g_engine_scan_cus;
    g_engine_scan_cus = cus > 0 ? (uint32_t)cus : 0u;
    return old;
}

struct fws_decode_engine {
    int device = 0;
    fws_gpu_ctx *ctx[kSlots] = {};
    bool used[kSlots] = {};
    hipStream_t sx = nullptr, sy = nullptr;
    hipEvent_t ev_in = nullptr, ev_jx = nullptr, ev_jy = nullptr;   // run start, the two streams' ends
    hipEvent_t ev_scan[kSlots] = {}, ev_done[kSlots] = {};
    uint64_t max_frames = 0, max_bytes = 0;
    bool utf8_ready = false;
    uint32_t next = 0;                     // the next job's workspace
    int mode = 0;                          // the schedule this engine was created with
};

static void engine_free(fws_decode_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->sx) (void)hipStreamSynchronize(e->sx);
    if (e->sy) (void)hipStreamSynchronize(e->sy);
    for (int k = 0; k < kSlots; ++k) {
        if (e->ev_scan[k]) (void)hipEventDestroy(e->ev_scan[k]);
        if (e->ev_done[k]) (void)hipEventDestroy(e->ev_done[k]);
        fws_gpu_ctx_destroy(e->ctx[k]);
    }
    for (hipEvent_t ev : {e->ev_in, e->ev_jx, e->ev_jy})
        if (ev) (void)hipEventDestroy(ev);
    if (e->sx) (void)hipStreamDestroy(e->sx);
    if (e->sy) (void)hipStreamDestroy(e->sy);
    delete e;
}

// Workspaces in use: the default schedule (mode 0) alternates two, the
// split-phase schedule keeps kSlots decodes in flight (the third
// full-size workspace sat unused in mode 0).
static int engine_slots(const fws_decode_engine *e) { return e->mode == 0 ? 2 : kSlots; }

// Workspaces for jobs of up to `frames` frames / `bytes` bytes (and UTF-8
// seams): a growth drains the engine first (the workspaces may be in use).
static int engine_reserve(fws_decode_engine *e, uint64_t frames, uint64_t bytes, bool utf8) {
    if (frames <= e->max_frames && bytes <= e->max_bytes && (!utf8 || e->utf8_ready)) return 0;
    int r;
    if ((r = fws_hip_status(hipStreamSynchronize(e->sx))) || (r = fws_hip_status(hipStreamSynchronize(e->sy))))
        return r;
    const uint64_t f = frames > e->max_frames ? frames : e->max_frames;
    const uint64_t b = bytes > e->max_bytes ? bytes : e->max_bytes;
    if (f > 0xFFFFFFFFull) return FWS_ERR_CAPACITY;
    for (int k = 0; k < engine_slots(e); ++k) {
        if ((r = fws_gpu_ctx_reserve(e->ctx[k], f, b))) return r;
        if ((r = fws_decode_prepare(e->ctx[k], b, (uint32_t)f, utf8 || e->utf8_ready))) return r;
    }
    e->max_frames = f;
    e->max_bytes = b;
    e->utf8_ready = e->utf8_ready || utf8;
    return 0;
}

extern "C" {

int fws_decode_engine_create(int device, uint64_t max_frames, uint64_t max_stream_bytes, fws_decode_engine **out) {
    if (!out) return FWS_ERR_INVALID;
    *out = nullptr;
    fws_decode_engine *e = new (std::nothrow) fws_decode_engine();
    if (!e) return FWS_ERR_INTERNAL;
    e->device = device;
    e->mode = g_engine_mode;
    const uint32_t scan_cus = e->mode == 1 ? g_engine_scan_cus : 0u;
    int r = 0;
    for (int k = 0; k < kSlots && !r; ++k) r = fws_gpu_ctx_create(device, &e->ctx[k]);
    int cus = 0;
    if (!r) r = fws_hip_status(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    if (!r && scan_cus >= (uint32_t)cus) r = FWS_ERR_INVALID;
    if (!r && scan_cus > 0) {
        // CU i goes to the scan stream when floor((i + 1) s / C) > floor(i s / C):
        // s CUs spread evenly over the index range, the rest to the other stream
        uint32_t mx[64] = {}, my[64] = {};
        const uint32_t words = ((uint32_t)cus + 31u) / 32u;
        if (words > 64u) r = FWS_ERR_INVALID;
        for (uint32_t i = 0; !r && i < (uint32_t)cus; ++i) {
            const bool x = ((uint64_t)(i + 1) * scan_cus) / (uint32_t)cus > ((uint64_t)i * scan_cus) / (uint32_t)cus;
            (x ? mx : my)[i / 32] |= 1u << (i % 32);
        }
        if (!r) r = fws_hip_status(hipExtStreamCreateWithCUMask(&e->sx, words, mx));
        if (!r) r = fws_hip_status(hipExtStreamCreateWithCUMask(&e->sy, words, my));
    } else if (!r) {
        r = fws_hip_status(hipStreamCreateWithFlags(&e->sx, hipStreamNonBlocking));
        if (!r) r = fws_hip_status(hipStreamCreateWithFlags(&e->sy, hipStreamNonBlocking));
    }
    const unsigned evf = hipEventDisableTiming;
    if (!r) r = fws_hip_status(hipEventCreateWithFlags(&e->ev_in, evf));
    if (!r) r = fws_hip_status(hipEventCreateWithFlags(&e->ev_jx, evf));
    if (!r) r = fws_hip_status(hipEventCreateWithFlags(&e->ev_jy, evf));
    for (int k = 0; k < kSlots && !r; ++k) {
        r = fws_hip_status(hipEventCreateWithFlags(&e->ev_scan[k], evf));
        if (!r) r = fws_hip_status(hipEventCreateWithFlags(&e->ev_done[k], evf));
    }
    if (!r && (max_frames || max_stream_bytes)) r = engine_reserve(e, max_frames, max_stream_bytes, false);
    if (r) {
        engine_free(e);
        return r;
    }
    *out = e;
    return 0;
}

void fws_decode_engine_destroy(fws_decode_engine *e) { engine_free(e); }

// Queues every job on the engine's streams (after ev_in); returns the first
// failure, with the jobs before it queued.
static int engine_queue(fws_decode_engine *e, const fws_decode_job *jobs, uint32_t n) {
    int r;
    if (e->mode == 0) {
        // job j's whole decode on stream j % 2, workspace j % 2 (stream order
        // serialises the jobs that share a workspace). Left alone the two streams
        // fall into step (both scan, both resolve, both unmask: a kernel trace,
        // profiles/r04/engine/); making each scan wait for the previous job's scan,
        // so that scans alternate, measured slower (0.170-0.177 against
        // 0.165 ms, profiles/r04/engine/sweep_scan_order.jsonl)
        for (uint32_t j = 0; j < n; ++j) {
            const fws_decode_job &q = jobs[j];
            const uint32_t k = e->next;
            e->next = (k + 1) % 2;
            fws_gpu_ctx *c = e->ctx[k];
            hipStream_t st = k ? e->sy : e->sx;
            uint8_t *w = (uint8_t *)q.dev_wire;
            if ((r = fws_decode_prepare(c, q.len, q.cap, q.dev_utf8_ok != nullptr))) return r;   // sized: no allocation
            if ((r = fws_launch_decode(c, w, q.len, q.dev_frames, q.cap, q.dev_result, q.dev_utf8_ok, st))) return r;
            if ((r = fws_decode_unmask(c, w, q.len, q.dev_frames, q.cap, q.dev_utf8_ok, st))) return r;
        }
        return 0;
    }
    for (uint32_t j = 0; j < n; ++j) {
        const fws_decode_job &q = jobs[j];
        const uint32_t k = e->next;
        e->next = (k + 1) % kSlots;
        fws_gpu_ctx *c = e->ctx[k];
        uint8_t *w = (uint8_t *)q.dev_wire;
        if ((r = fws_decode_prepare(c, q.len, q.cap, q.dev_utf8_ok != nullptr))) return r;
        if (e->used[k] && (r = fws_hip_status(hipStreamWaitEvent(e->sx, e->ev_done[k], 0)))) return r;
        if ((r = fws_launch_decode_scan(c, w, q.len, e->sx))) return r;
        if ((r = fws_hip_status(hipEventRecord(e->ev_scan[k], e->sx)))) return r;
        if ((r = fws_hip_status(hipStreamWaitEvent(e->sy, e->ev_scan[k], 0)))) return r;
        if ((r = fws_launch_decode_resolve(c, w, q.len, q.dev_frames, q.cap, q.dev_result, q.dev_utf8_ok, e->sy)))
            return r;
        if ((r = fws_decode_unmask(c, w, q.len, q.dev_frames, q.cap, q.dev_utf8_ok, e->sy))) return r;
        if ((r = fws_hip_status(hipEventRecord(e->ev_done[k], e->sy)))) return r;
        e->used[k] = true;
    }
    return 0;
}

int fws_decode_engine_run(fws_decode_engine *e, const fws_decode_job *jobs, uint32_t n, void *stream) {
    if (!e || (n && !jobs)) return FWS_ERR_INVALID;
    hipStream_t s = (hipStream_t)stream;
    int r;
    if ((r = fws_hip_status(hipSetDevice(e->device)))) return r;
    // every argument checked (and the workspaces grown) before anything is queued
    uint64_t mf = 0, mb = 0;
    bool utf8 = false;
    for (uint32_t j = 0; j < n; ++j) {
        const fws_decode_job &q = jobs[j];
        if (!q.dev_result || (q.len && !q.dev_wire) || (q.cap && !q.dev_frames) || q.reserved) return FWS_ERR_INVALID;
        if (((uintptr_t)q.dev_wire & 15u) != 0) return FWS_ERR_INVALID;
        if (q.cap > mf) mf = q.cap;
        if (q.len > mb) mb = q.len;
        utf8 = utf8 || q.dev_utf8_ok;
    }
    if (n == 0) return 0;
    if ((r = engine_reserve(e, mf, mb, utf8))) return r;
    if ((r = fws_hip_status(hipEventRecord(e->ev_in, s))) || (r = fws_hip_status(hipStreamWaitEvent(e->sx, e->ev_in, 0))) ||
        (r = fws_hip_status(hipStreamWaitEvent(e->sy, e->ev_in, 0))))
        return r;
    r = engine_queue(e, jobs, n);
    // `stream` waits for both streams, also after a failure part-way (the jobs
    // queued before it still run)
    int j = fws_hip_status(hipEventRecord(e->ev_jx, e->sx));
    if (!j) j = fws_hip_status(hipEventRecord(e->ev_jy, e->sy));
    if (!j) j = fws_hip_status(hipStreamWaitEvent(s, e->ev_jx, 0));
    if (!j) j = fws_hip_status(hipStreamWaitEvent(s, e->ev_jy, 0));
    return r ? r : j;
}

}  // extern "C"
