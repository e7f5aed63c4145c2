// outplan_common.h -- the one-block body of the output-space plan (the
// out-of-place reassembly, fws_gpu_unmask_gather, and the TX frame builder,
// fws_gpu_encode_frames), for k_out_plan (outplan_kernels.hip).
// One thread per descriptor; the block scan of the output sizes and a
// decoupled look-back (plan_common.h) give base[f]; frame f owns the 4 KiB
// output units whose first byte lies in [base[f], base[f + 1]), written
// wave-cooperatively.
#pragma once
#include "fws_device.h"
#include "fws_internal.h"
#include "plan_common.h"

namespace fwsk {

struct OutPlanArgs {
    uint64_t *base;         // n + 1
    uint32_t *unit_first;   // output units
    uint64_t unit_cap;
    uint64_t *total;        // bytes to write (0 when they do not fit out_cap)
    uint64_t *out_len;      // TX: total, or ~0 when it exceeds out_cap; may be null
    uint64_t out_cap;
    uint64_t *status;
    uint32_t *ticket;
    uint32_t epoch;
};

__device__ __forceinline__ uint64_t out_size(const fws_frame_desc &d) { return d.payload_len; }
__device__ __forceinline__ uint64_t out_size(const fws_tx_desc &d) {   // w_socket.h:49-65
    return 2u + (d.masked ? 4u : 0u) + (d.len < 126u ? 0u : (d.len <= 65535u ? 2u : 8u)) + d.len;
}

// One frame per thread for the first kF threads (kF = 64 for batches of few
// frames -- C4: 1427 fragments of up to 1 MiB, 46 units each on average --
// so they still spread over many workgroups; 256 for large batches, where the
// look-back over fewer workgroups is the shorter chain). Then the four waves
// write the kF frames' unit-map runs, kF / 4 runs each, 64 entries per store.
template <typename Desc, int kF>
__device__ __forceinline__ void out_plan_block(const Desc *__restrict__ d, uint32_t n, const OutPlanArgs &a,
                                               uint32_t blk) {
    __shared__ uint64_t s_u0[kF];
    __shared__ uint32_t s_len[kF];
    __shared__ uint64_t s_wsum[kBlock / kWave];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const uint64_t f = uint64_t(blk) * kF + threadIdx.x;
    const bool mine = threadIdx.x < (uint32_t)kF, has = mine && f < n;
    const uint64_t sz = has ? out_size(d[f]) : 0;
    const uint64_t inc = wave_incl_scan64(sz, lane);
    if (lane == kWave - 1) s_wsum[w] = inc;
    __syncthreads();
    uint64_t run = inc - sz, agg = 0;
#pragma unroll
    for (int i = 0; i < kBlock / kWave; ++i) {
        run += i < w ? s_wsum[i] : 0;
        agg += s_wsum[i];
    }
    bool unused;
    run += block_lookback(a.status, blk, agg, true, a.epoch, &unused);
    if (mine) {
        uint64_t u0 = 0, ue = 0;
        if (has) {
            a.base[f] = run;
            u0 = (run + 4095u) / 4096u;
            ue = (run + sz + 4095u) / 4096u;
            if (f == n - 1) {
                const uint64_t tot = run + sz;
                const bool fits = tot <= a.out_cap;
                a.base[n] = tot;
                *a.total = fits ? tot : 0;            // nothing is written when it does not fit
                if (a.out_len) *a.out_len = fits ? tot : ~0ull;
            }
        }
        if (ue > a.unit_cap) ue = a.unit_cap;         // contract violation guard, never OOB
        s_u0[threadIdx.x] = u0;
        s_len[threadIdx.x] = ue > u0 ? (uint32_t)(ue - u0) : 0u;
    }
    // short runs (frames of a few KiB): each thread writes its own
    const uint32_t my_len = mine ? s_len[threadIdx.x] : 0u;
    if (__syncthreads_and(my_len <= 4u)) {
        for (uint32_t k = 0; k < my_len; ++k) a.unit_first[s_u0[threadIdx.x] + k] = (uint32_t)f;
        return;
    }
    constexpr uint32_t kPerWave = kF / (kBlock / kWave);
    for (uint32_t L = (uint32_t)w * kPerWave; L < (uint32_t)(w + 1) * kPerWave; ++L) {
        const uint32_t len = s_len[L];
        const uint64_t u0 = s_u0[L];
        const uint32_t fl = blk * kF + L;
        for (uint32_t k = (uint32_t)lane; k < len; k += kWave) a.unit_first[u0 + k] = fl;
    }
}

}  // namespace fwsk
