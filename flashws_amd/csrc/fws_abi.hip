// fws_abi.hip -- the extern "C" entry points of libfws_gpu.so (include/fws_gpu.h).
// Host code: argument checks, workspace ownership, kernel launch sequencing.
#include <stdlib.h>
#include <string.h>

#include "fws_internal.h"

namespace {

template <typename T>
int dev_alloc(T **p, uint64_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    return fws_hip_status(hipMalloc((void **)p, count * sizeof(T)));
}

template <typename T>
void dev_free(T *&p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

void free_plan(fws_plan_ws &w) {
    dev_free(w.block_sums);
    dev_free(w.cbase);
    dev_free(w.unit_first);
    dev_free(w.unit_rec);
    dev_free(w.total);
    dev_free(w.status);
    dev_free(w.ticket);
    dev_free(w.mode);
    dev_free(w.tx_seam);
}

}  // namespace

int fws_ctx_ensure_plan(fws_gpu_ctx *ctx, uint64_t frames, uint64_t units) {
    if (frames <= ctx->cap_frames && units <= ctx->cap_units && ctx->plan.cbase) return 0;
    if (frames < ctx->cap_frames) frames = ctx->cap_frames;
    if (units < ctx->cap_units) units = ctx->cap_units;
    free_plan(ctx->plan);
    int r;
    if ((r = dev_alloc(&ctx->plan.block_sums, frames / 1024 + 2))) return r;
    if ((r = dev_alloc(&ctx->plan.cbase, frames + 2))) return r;
    if ((r = dev_alloc(&ctx->plan.unit_first, units + 2))) return r;
    if ((r = dev_alloc(&ctx->plan.unit_rec, 4 * (units + 2)))) return r;
    if ((r = dev_alloc(&ctx->plan.total, 2))) return r;
    if ((r = dev_alloc(&ctx->plan.status, frames / 8 + 2))) return r;
    if ((r = dev_alloc(&ctx->plan.ticket, 2))) return r;
    if ((r = dev_alloc(&ctx->plan.mode, sizeof(fws_plan_mode) / 8))) return r;
    if ((r = dev_alloc(&ctx->plan.tx_seam, 4 * (2 * frames + 2)))) return r;
    if ((r = fws_hip_status(hipMemset(ctx->plan.status, 0, (frames / 8 + 2) * 8)))) return r;
    if ((r = fws_hip_status(hipMemset(ctx->plan.ticket, 0, 8)))) return r;
    if ((r = fws_hip_status(hipMemset(ctx->plan.mode, 0, sizeof(fws_plan_mode))))) return r;
    ctx->plan.status_cap = frames / 8 + 2;             // k_tx_one: >= 8 frames per workgroup
    ctx->plan.epoch = 0;
    ctx->cap_frames = frames;
    ctx->cap_units = units;
    ctx->plan.unit_cap = units + 1;
    return 0;
}

// per-unit seam words of fws_gpu_unmask_sorted_utf8 for a span of `span` bytes
int fws_ctx_ensure_seam(fws_gpu_ctx *ctx, uint64_t span) {
    const uint64_t words = 2 * (span / 4096 + 2);
    if (words <= ctx->seam_cap) return 0;
    dev_free(ctx->seam);
    ctx->seam_cap = 0;
    if (int r = fws_hip_status(hipMalloc((void **)&ctx->seam, words * 4))) return r;
    ctx->seam_cap = words;
    return 0;
}

extern "C" {

// Test / tuning hook (not part of the ABI): the decode counters of the last
// decode on ctx (decode_common.h Counter), synchronously. 0 or an error.
__attribute__((visibility("default"))) int fws_internal_decode_counters(fws_gpu_ctx *ctx, uint32_t *out, int n) {
    if (!ctx || !out || n <= 0 || !ctx->dec.counters) return FWS_ERR_INVALID;
    if (n > 64) n = 64;
    return fws_hip_status(hipMemcpy(out, ctx->dec.counters, (size_t)n * 4, hipMemcpyDeviceToHost));
}

// Test hook (not part of the ABI): the last descriptor plan's fws_plan_mode
// words (byte_space, s0, first_po, last_pe, n_units), synchronously.
__attribute__((visibility("default"))) int fws_internal_plan_mode(fws_gpu_ctx *ctx, uint64_t *out5) {
    if (!ctx || !out5 || !ctx->plan.mode) return FWS_ERR_INVALID;
    return fws_hip_status(hipMemcpy(out5, ctx->plan.mode, 5 * 8, hipMemcpyDeviceToHost));
}

int fws_gpu_abi_version(void) { return FWS_GPU_ABI_VERSION; }

int fws_gpu_device_count(int *count) {
    if (!count) return FWS_ERR_INVALID;
    *count = 0;
    hipError_t e = hipGetDeviceCount(count);
    if (e == hipErrorNoDevice) { *count = 0; return 0; }
    return fws_hip_status(e);
}

int fws_gpu_ctx_create(int device, fws_gpu_ctx **out) {
    if (!out) return FWS_ERR_INVALID;
    *out = nullptr;
    int n = 0;
    int r = fws_gpu_device_count(&n);
    if (r) return r;
    if (device < 0 || device >= n) return FWS_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if ((r = fws_hip_status(hipGetDeviceProperties(&prop, device)))) return r;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return FWS_ERR_NO_DEVICE;
    if ((r = fws_hip_status(hipSetDevice(device)))) return r;
    fws_gpu_ctx *c = new fws_gpu_ctx();
    c->device = device;
    *out = c;
    return 0;
}

void fws_gpu_ctx_destroy(fws_gpu_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    fws_rx_service_destroy(ctx->svc);    // its grid drained before the buffers it names go
    ctx->svc = nullptr;
    free_plan(ctx->plan);
    dev_free(ctx->any_q);
    dev_free(ctx->any_cnt);
    fws_decode_ws &d = ctx->dec;
    dev_free(d.tile_count);
    dev_free(d.cnt_base);
    dev_free(d.stage_info);
    dev_free(d.spill_info);
    dev_free(d.tile_spill);
    dev_free(d.scan_dummy);
    dev_free(d.nres);
    dev_free(d.tails);
    dev_free(d.gnx);
    dev_free(d.tpk);
    dev_free(d.tmark);
    dev_free(d.comp);
    dev_free(d.st_nodes);
    dev_free(d.st_n);
    dev_free(d.st_nt);
    dev_free(d.st_entry);
    dev_free(d.st_fbase);
    dev_free(d.bg_nx);
    dev_free(d.bg_wt);
    dev_free(d.bg_lref);
    dev_free(d.bg_ptr);
    dev_free(d.bg_sc);
    dev_free(d.bg_mark);
    dev_free(ctx->seam);
    delete ctx;
}

int fws_gpu_ctx_reserve(fws_gpu_ctx *ctx, uint64_t max_frames, uint64_t max_stream_bytes) {
    if (!ctx) return FWS_ERR_INVALID;
    int r = fws_hip_status(hipSetDevice(ctx->device));
    if (r) return r;
    // chunks <= bytes / 16 + 2 per frame; units = chunks / 256
    const uint64_t units = (max_stream_bytes / 16 + 2 * max_frames) / 256 + 2;
    if ((r = fws_ctx_ensure_plan(ctx, max_frames, units))) return r;
    if (max_stream_bytes > ctx->cap_stream) ctx->cap_stream = max_stream_bytes;
    return fws_ctx_ensure_seam(ctx, ctx->cap_stream);
}


int fws_gpu_mask(void *dev_ptr, uint64_t n, uint32_t key, void *stream) {
    if (n && !dev_ptr) return FWS_ERR_INVALID;
    return fws_launch_mask_single(dev_ptr, n, key, 0u, (hipStream_t)stream);
}

int fws_gpu_unmask_plan(fws_gpu_ctx *ctx, const void *dev_base, const fws_frame_desc *dev_descs,
                        uint32_t n, void *stream) {
    if (!ctx || (n && (!dev_base || !dev_descs))) return FWS_ERR_INVALID;
    if (n == 0) return 0;
    if (ctx->cap_stream == 0 || n > ctx->cap_frames) return FWS_ERR_CAPACITY;
    if (int r = fws_hip_status(hipSetDevice(ctx->device))) return r;
    return fws_launch_plan((const uint8_t *)dev_base, dev_descs, n, nullptr, ctx->plan, (hipStream_t)stream);
}

int fws_gpu_unmask_run(fws_gpu_ctx *ctx, void *dev_base, const fws_frame_desc *dev_descs,
                       uint32_t n, void *stream) {
    if (!ctx || (n && (!dev_base || !dev_descs))) return FWS_ERR_INVALID;
    if (n == 0) return 0;
    if (ctx->cap_stream == 0 || n > ctx->cap_frames) return FWS_ERR_CAPACITY;
    if (int r = fws_hip_status(hipSetDevice(ctx->device))) return r;
    // the grid is sized from the reservation; a larger batch is still covered in
    // full (grid-stride loop, unit owners past the map's capacity are searched)
    const uint64_t max_chunks = ctx->cap_stream / 16 + 2ull * n;
    return fws_launch_unmask((uint8_t *)dev_base, dev_descs, n, nullptr, ctx->plan, max_chunks,
                             (hipStream_t)stream);
}

int fws_gpu_unmask_batch(fws_gpu_ctx *ctx, void *dev_base, const fws_frame_desc *dev_descs,
                         uint32_t n, void *stream) {
    if (fws_unmask_any_on()) {
        // one launch, descriptor-major (+ the queued pieces of regions over 64 KiB):
        // no plan; the same arguments and capacity checks as the planned form
        if (!ctx || (n && (!dev_base || !dev_descs))) return FWS_ERR_INVALID;
        if (n == 0) return 0;
        if (ctx->cap_stream == 0 || n > ctx->cap_frames) return FWS_ERR_CAPACITY;
        int r;
        if ((r = fws_hip_status(hipSetDevice(ctx->device))) || (r = fws_ctx_ensure_any(ctx))) return r;
        const uint32_t k = ctx->any_parity;
        ctx->any_parity ^= 1u;
        const uint32_t pg = ctx->any_qcap / 4u + 1u;
        return fws_launch_unmask_any((uint8_t *)dev_base, dev_descs, n, ctx->any_q, ctx->any_qcap, ctx->any_cnt + k,
                                     ctx->any_cnt + (k ^ 1u), pg < 2048u ? pg : 2048u, (hipStream_t)stream);
    }
    int r = fws_gpu_unmask_plan(ctx, dev_base, dev_descs, n, stream);
    if (r) return r;
    return fws_gpu_unmask_run(ctx, dev_base, dev_descs, n, stream);
}

}  // extern "C"

int fws_ctx_ensure_any(fws_gpu_ctx *ctx) {
    // pieces come from regions over 64 KiB: at most the reserved span / 64 KiB of
    // them (a batch past the reservation has its waves do their own pieces)
    const uint64_t want = ctx->cap_stream / (64u * 1024u) + 64u;
    const uint32_t cap = (uint32_t)(want < 0x7FFFFFFFull ? want : 0x7FFFFFFFull);
    if (ctx->any_q && ctx->any_qcap >= cap) return 0;
    hipError_t e = hipSuccess;
    if (ctx->any_q) {
        if ((e = hipDeviceSynchronize()) != hipSuccess) return fws_hip_status(e);   // (a regrowth: rare)
        (void)hipFree(ctx->any_q);
        ctx->any_q = nullptr;
    }
    if (!ctx->any_cnt) {
        if ((e = hipMalloc((void **)&ctx->any_cnt, 2 * sizeof(uint32_t))) != hipSuccess) return fws_hip_status(e);
        if ((e = hipMemset(ctx->any_cnt, 0, 2 * sizeof(uint32_t))) != hipSuccess) return fws_hip_status(e);
        ctx->any_parity = 0;
    }
    if ((e = hipMalloc((void **)&ctx->any_q, (uint64_t)cap * sizeof(uint64_t))) != hipSuccess) return fws_hip_status(e);
    ctx->any_qcap = cap;
    return 0;
}

extern "C" {

int fws_gpu_check_sorted(fws_gpu_ctx *ctx, const fws_frame_desc *dev_descs, uint32_t n, uint32_t *dev_bad,
                         void *stream) {
    if (!ctx || !dev_bad || (n && !dev_descs)) return FWS_ERR_INVALID;
    int r;
    if ((r = fws_hip_status(hipSetDevice(ctx->device)))) return r;
    return fws_launch_check_sorted(dev_descs, n, dev_bad, (hipStream_t)stream);
}

// FWS_CHECK_SORTED=1 in the environment: the sorted entry points check the
// contract first and refuse (FWS_ERR_INVALID, nothing written) a violating
// batch; this synchronises the stream (a debug mode, not for timing)
static int check_sorted_debug(fws_gpu_ctx *ctx, const fws_frame_desc *d, uint32_t n, hipStream_t s) {
    static const bool on = [] {
        const char *v = getenv("FWS_CHECK_SORTED");
        return v && v[0] && v[0] != '0';
    }();
    if (!on) return 0;
    uint32_t *bad = nullptr, h = 0;
    hipError_t e = hipMalloc((void **)&bad, sizeof(uint32_t));
    if (e != hipSuccess) return fws_hip_status(e);
    int r = fws_launch_check_sorted(d, n, bad, s);
    if (r == 0 && (e = hipMemcpyAsync(&h, bad, sizeof(h), hipMemcpyDeviceToHost, s)) != hipSuccess) r = fws_hip_status(e);
    if (r == 0 && (e = hipStreamSynchronize(s)) != hipSuccess) r = fws_hip_status(e);
    (void)hipFree(bad);
    if (r) return r;
    return h == 0xFFFFFFFFu ? 0 : FWS_ERR_INVALID;
}

int fws_gpu_unmask_sorted(fws_gpu_ctx *ctx, void *dev_base, const fws_frame_desc *dev_descs, uint32_t n,
                          void *stream) {
    if (!ctx || (n && (!dev_base || !dev_descs))) return FWS_ERR_INVALID;
    if (n == 0) return 0;
    int r;
    if ((r = fws_hip_status(hipSetDevice(ctx->device)))) return r;
    if ((r = check_sorted_debug(ctx, dev_descs, n, (hipStream_t)stream))) return r;
    // the grid only bounds the grid-stride loop: every unit of the span is visited at any grid
    const uint64_t span = ctx->cap_stream ? ctx->cap_stream : 4096ull * n;
    return fws_launch_unmask_sorted((uint8_t *)dev_base, dev_descs, n, span, (hipStream_t)stream);
}

int fws_gpu_unmask_sorted_utf8(fws_gpu_ctx *ctx, void *dev_base, const fws_frame_desc *dev_descs, uint32_t n,
                               uint8_t *dev_ok, void *stream) {
    if (!ctx || (n && (!dev_base || !dev_descs || !dev_ok))) return FWS_ERR_INVALID;
    if (n == 0) return 0;
    int r;
    if ((r = fws_hip_status(hipSetDevice(ctx->device)))) return r;
    if ((r = check_sorted_debug(ctx, dev_descs, n, (hipStream_t)stream))) return r;
    // span only sizes the grid (grid-stride: every unit is visited) and the seam
    // reservation; the kernels bound their seam words by ctx->seam_cap, so a batch
    // whose payload span exceeds it stays in bounds
    const uint64_t span = ctx->cap_stream ? ctx->cap_stream : 4096ull * n;
    if ((r = fws_ctx_ensure_seam(ctx, span))) return r;
    return fws_launch_unmask_sorted_utf8((uint8_t *)dev_base, dev_descs, n, span, dev_ok, ctx->seam, ctx->seam_cap,
                                         (hipStream_t)stream);
}

int fws_gpu_unmask_gather(fws_gpu_ctx *ctx, void *dev_dst, const void *dev_src, const fws_frame_desc *dev_descs,
                          uint32_t n, void *stream) {
    if (!ctx || (n && (!dev_dst || !dev_src || !dev_descs))) return FWS_ERR_INVALID;
    if (((uintptr_t)dev_dst & 15u) != 0) return FWS_ERR_INVALID;
    if (n == 0) return 0;
    if (ctx->cap_stream == 0 || n > ctx->cap_frames) return FWS_ERR_CAPACITY;
    if (int r = fws_hip_status(hipSetDevice(ctx->device))) return r;
    return fws_launch_gather((uint8_t *)dev_dst, (const uint8_t *)dev_src, dev_descs, n, ctx->plan, ctx->cap_stream,
                             (hipStream_t)stream);
}

int fws_gpu_validate_utf8(fws_gpu_ctx *ctx, const void *dev_base, const fws_frame_desc *dev_descs, uint32_t n,
                          uint8_t *dev_ok, void *stream) {
    if (!ctx || (n && (!dev_base || !dev_descs || !dev_ok))) return FWS_ERR_INVALID;
    if (int r = fws_hip_status(hipSetDevice(ctx->device))) return r;
    return fws_launch_utf8_descs((const uint8_t *)dev_base, dev_descs, n, dev_ok, (hipStream_t)stream);
}

int fws_gpu_decode_stream(fws_gpu_ctx *ctx, void *dev_wire, uint64_t len, fws_frame_info *dev_frames,
                          uint32_t cap, fws_decode_result *dev_result, uint8_t *dev_utf8_ok, void *stream) {
    if (!ctx || !dev_result || (len && !dev_wire) || (cap && !dev_frames)) return FWS_ERR_INVALID;
    if (((uintptr_t)dev_wire & 15u) != 0) return FWS_ERR_INVALID;   // tiles are staged with 16-B loads
    hipStream_t s = (hipStream_t)stream;
    int r;
    if ((r = fws_hip_status(hipSetDevice(ctx->device)))) return r;
    if (fws_resolve_mode() == 2 && len <= kSmallMax && !dev_utf8_ok) {
        // test hook: the RX session's one-launch small-read decode, with its
        // fallback taken synchronously as rx_session.cpp does
        if ((r = fws_launch_decode_small((uint8_t *)dev_wire, len, dev_frames, cap, dev_result, s))) return r;
        int32_t st = 0;
        if ((r = fws_hip_status(hipMemcpyAsync(&st, dev_result, 4, hipMemcpyDeviceToHost, s)))) return r;
        if ((r = fws_hip_status(hipStreamSynchronize(s)))) return r;
        if (st != FWS_SMALL_DECLINED) return 0;
    }
    if ((r = fws_decode_prepare(ctx, len, cap, dev_utf8_ok != nullptr))) return r;
    if ((r = fws_launch_decode(ctx, (uint8_t *)dev_wire, len, dev_frames, cap, dev_result, dev_utf8_ok, s)))
        return r;
    return fws_decode_unmask(ctx, (uint8_t *)dev_wire, len, dev_frames, cap, dev_utf8_ok, s);
}

}  // extern "C"

int fws_decode_prepare(fws_gpu_ctx *ctx, uint64_t len, uint32_t cap, bool utf8) {
    int r;
    if ((r = fws_decode_ensure(ctx, len, cap))) return r;
    const uint64_t units = (len / 16 + 2ull * cap) / 256 + 2;
    if ((r = fws_ctx_ensure_plan(ctx, cap, units))) return r;
    return utf8 ? fws_ctx_ensure_seam(ctx, len) : 0;
}

int fws_decode_unmask(fws_gpu_ctx *ctx, uint8_t *wire, uint64_t len, fws_frame_info *frames, uint32_t cap,
                      uint8_t *utf8_ok, hipStream_t s) {
    if (cap == 0 || len == 0) return 0;
    // the resolve left the device frame count, the stream-space unmask plan of the
    // decoded frames and (with utf8_ok) each frame's TEXT/FIN/complete preset;
    // the unmask checks UTF-8 while the payload is in registers
    const uint32_t *n_dev = ctx->dec.counters + kDecodeFramesCounter;
    return fws_launch_unmask_stream(wire, len, frames, cap, n_dev, ctx->plan.unit_first, utf8_ok, ctx->seam, s);
}

