// fws_internal.h -- host-side internals of libfws_gpu (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fws_gpu.h"

// Map a HIP error to the ABI's negative range (fws_gpu.h FWS_ERR_HIP_BASE).
static inline int fws_hip_status(hipError_t e) {
    return e == hipSuccess ? 0 : (FWS_ERR_HIP_BASE - (int)e);
}

// Device workspace for the chunk plan of one descriptor batch.
struct fws_plan_ws {
    uint64_t *block_sums = nullptr;   // ceil(n / 1024)
    uint64_t *cbase = nullptr;        // n + 1
    uint32_t *unit_first = nullptr;   // units (total chunks / 256) + 1
    uint64_t *total = nullptr;        // 1
    uint64_t unit_cap = 0;            // capacity of unit_first (writes are clamped)
};

// Stream-decode workspace (see decode_kernels.hip).
struct fws_decode_ws {
    uint64_t tile_bytes = 0;          // bytes per scan tile
    uint64_t max_tiles = 0;
    uint64_t max_surv = 0;            // capacity of the survivor arrays
    uint32_t *tile_count = nullptr;   // survivors per tile
    uint64_t *tile_base = nullptr;    // exclusive prefix of tile_count
    uint64_t *surv_pos = nullptr;     // survivor header offsets, sorted
    uint64_t *surv_next = nullptr;    // next header offset of each survivor
    uint32_t *jump = nullptr;         // [levels][max_surv] pointer-doubling tables
    uint32_t levels = 0;
    uint8_t *mark = nullptr;          // on-path flags
    uint64_t *mark_base = nullptr;    // exclusive prefix of marks
    uint32_t *counters = nullptr;     // misc device counters
    fws_frame_desc *descs = nullptr;  // payload regions of the decoded frames
};

struct fws_gpu_ctx {
    int device = 0;
    uint64_t cap_frames = 0;
    uint64_t cap_units = 0;
    uint64_t cap_stream = 0;
    fws_plan_ws plan;
    fws_decode_ws dec;
    void *pinned = nullptr;           // host staging for small readbacks
};

int fws_ctx_ensure_plan(fws_gpu_ctx *ctx, uint64_t frames, uint64_t units);

// unmask_kernels.hip
int fws_launch_mask_single(void *dev_ptr, uint64_t n, uint32_t key, uint32_t phase, hipStream_t s);
int fws_launch_plan(const uint8_t *base, const fws_frame_desc *d, uint32_t n, fws_plan_ws &ws,
                    hipStream_t s);
int fws_launch_unmask(uint8_t *base, const fws_frame_desc *d, uint32_t n, const fws_plan_ws &ws,
                      uint64_t max_chunks, hipStream_t s);
