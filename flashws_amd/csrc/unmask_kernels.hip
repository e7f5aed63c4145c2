// unmask_kernels.hip -- descriptor-mode XOR unmask for gfx950.
//
// The hot loop of flashws's RX path is WSMaskBytesFast (crypto/ws_mask.h:175)
// called once per frame part from OnRecvData (net/w_socket.h:586,614). Here a
// whole batch of frame payloads is one launch: the payload bytes are cut into
// 16-byte aligned chunks, the chunk space of all frames is concatenated
// (exclusive prefix `cbase`, built by the two plan kernels), and every wave
// owns a 4 KiB unit of that space (64 lanes x 4 chunks), so any mix of frame
// sizes is load-balanced and every full chunk is one global_load_dwordx4 +
// v_xor + global_store_dwordx4 with the key broadcast in registers.
// HBM-bound: bytes = payload read + payload write (+ header bytes of partially
// covered chunks). No LDS, no MFMA.
#include "fws_device.h"
#include "fws_internal.h"

namespace fwsk {

// ---------------------------------------------------------------- plan
constexpr int kPlanItems = 4;                        // frames per thread
constexpr int kPlanTile = kBlock * kPlanItems;       // frames per block

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v, int lane) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        uint64_t t = __shfl_up(v, o, kWave);
        if (lane >= o) v += t;
    }
    return v;
}

// Block exclusive scan of one u64 per thread; returns the block total in *total.
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *total) {
    __shared__ uint64_t wsum[kBlock / kWave];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    uint64_t inc = wave_incl_scan(v, lane);
    if (lane == kWave - 1) wsum[w] = inc;
    __syncthreads();
    uint64_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < kBlock / kWave; ++i) {
        uint64_t s = wsum[i];
        off += (i < w) ? s : 0;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + inc - v;
}

__device__ __forceinline__ uint64_t desc_chunks(const uint8_t *base, const fws_frame_desc &d) {
    return chunks_of((uintptr_t)(base + d.payload_off), d.payload_len);
}

__global__ __launch_bounds__(kBlock) void k_plan_count(const uint8_t *base,
                                                       const fws_frame_desc *__restrict__ d,
                                                       uint32_t n, const uint32_t *__restrict__ n_dev,
                                                       uint64_t *__restrict__ block_sums) {
    if (n_dev && *n_dev < n) n = *n_dev;
    const uint64_t f0 = uint64_t(blockIdx.x) * kPlanTile + uint64_t(threadIdx.x) * kPlanItems;
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kPlanItems; ++i)
        if (f0 + i < n) s += desc_chunks(base, d[f0 + i]);
    uint64_t tot;
    block_excl_scan(s, &tot);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

// cbase[f] = chunks of frames [0, f); cbase[n] = total; unit_first[u] = frame
// holding chunk u * kUnitChunks; *total_out = total chunks.
__global__ __launch_bounds__(kBlock) void k_plan_scan(const uint8_t *base,
                                                      const fws_frame_desc *__restrict__ d, uint32_t n,
                                                      const uint32_t *__restrict__ n_dev,
                                                      const uint64_t *__restrict__ block_sums,
                                                      uint64_t *__restrict__ cbase,
                                                      uint32_t *__restrict__ unit_first,
                                                      uint64_t *__restrict__ total_out,
                                                      uint64_t unit_cap) {
    if (n_dev && *n_dev < n) n = *n_dev;
    __shared__ uint64_t s_prefix;
    // prefix of earlier blocks (n_blocks is small: n / 1024)
    uint64_t p = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += kBlock) p += block_sums[b];
    uint64_t dummy;
    uint64_t pe = block_excl_scan(p, &dummy);
    if (threadIdx.x == kBlock - 1) s_prefix = pe + p;
    __syncthreads();
    const uint64_t prefix = s_prefix;

    const uint64_t f0 = uint64_t(blockIdx.x) * kPlanTile + uint64_t(threadIdx.x) * kPlanItems;
    uint64_t c[kPlanItems];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kPlanItems; ++i) {
        c[i] = (f0 + i < n) ? desc_chunks(base, d[f0 + i]) : 0;
        s += c[i];
    }
    uint64_t tot;
    uint64_t run = prefix + block_excl_scan(s, &tot);
#pragma unroll
    for (int i = 0; i < kPlanItems; ++i) {
        const uint64_t f = f0 + i;
        if (f < n) {
            cbase[f] = run;
            if (c[i]) {
                uint64_t u = (run + kUnitChunks - 1) / kUnitChunks;
                uint64_t ue = (run + c[i] + kUnitChunks - 1) / kUnitChunks;
                if (ue > unit_cap) ue = unit_cap;   // contract violation guard, never OOB
                for (; u < ue; ++u) unit_first[u] = (uint32_t)f;
            }
            run += c[i];
            if (f == n - 1) {   // the thread holding the last frame has the grand total
                cbase[n] = run;
                *total_out = run;
            }
        }
    }
    if (n == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
        cbase[0] = 0;
        *total_out = 0;
    }
}

// ---------------------------------------------------------------- unmask
// One wave = one unit of kUnitChunks chunks. Loads for all U chunks of a lane
// are issued before any XOR/store so each lane keeps 64 B in flight.
template <bool kSingle>
__global__ __launch_bounds__(kBlock) void k_unmask(uint8_t *base, const fws_frame_desc *__restrict__ d,
                                                   uint32_t n, const uint32_t *__restrict__ n_dev,
                                                   const uint64_t *__restrict__ cbase,
                                                   const uint32_t *__restrict__ unit_first,
                                                   const uint64_t *__restrict__ total_ptr,
                                                   uint64_t unit_cap, fws_frame_desc single) {
    if (!kSingle && n_dev && *n_dev < n) n = *n_dev;
    if (n == 0) return;
    const uint64_t total = kSingle ? chunks_of((uintptr_t)(base + single.payload_off), single.payload_len)
                                   : *total_ptr;
    uint64_t n_units = (total + kUnitChunks - 1) / kUnitChunks;
    if (!kSingle && n_units > unit_cap) n_units = unit_cap;
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t nwaves = uint64_t(gridDim.x) * (kBlock / kWave);
    for (uint64_t u = uint64_t(blockIdx.x) * (kBlock / kWave) + threadIdx.x / kWave; u < n_units;
         u += nwaves) {
        uint32_t flo = 0, fhi = 0;
        if (!kSingle) {
            flo = unit_first[u];
            fhi = (u + 1 < n_units) ? unit_first[u + 1] : n - 1;
        }
        uintptr_t ca[kUnmaskU], lo[kUnmaskU], hi[kUnmaskU];
        uint32_t rk[kUnmaskU];
        bool live[kUnmaskU];
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            const uint64_t g = u * kUnitChunks + uint64_t(j) * kWave + lane;
            live[j] = g < total;
            fws_frame_desc fd = single;
            uint64_t cb = 0;
            if (!kSingle) {
                const uint32_t f = find_frame(cbase, flo, fhi, live[j] ? g : cbase[flo]);
                fd = d[f];
                cb = cbase[f];
            }
            const uintptr_t a0 = (uintptr_t)(base + fd.payload_off);
            lo[j] = a0;
            hi[j] = a0 + fd.payload_len;
            ca[j] = (a0 & ~uintptr_t(15)) + (uintptr_t)((g - cb) << 4);
            rk[j] = aligned_key(fd.key, fd.phase, a0);
        }
        u32x4 v[kUnmaskU];
        bool full[kUnmaskU];
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            full[j] = live[j] && ca[j] >= lo[j] && ca[j] + 16u <= hi[j];
            if (full[j]) v[j] = *reinterpret_cast<const u32x4 *>(ca[j]);
        }
#pragma unroll
        for (int j = 0; j < kUnmaskU; ++j) {
            if (full[j]) {
                *reinterpret_cast<u32x4 *>(ca[j]) = v[j] ^ rk[j];
            } else if (live[j]) {
                xor_partial_chunk(ca[j], lo[j], hi[j], rk[j]);
            }
        }
    }
}

}  // namespace fwsk

// ---------------------------------------------------------------- launchers
using namespace fwsk;

static int grid_for_units(uint64_t units) {
    // memory-bound: cap near 256 CUs x 8 blocks and grid-stride the rest
    uint64_t blocks = (units + (kBlock / kWave) - 1) / (kBlock / kWave);
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    return (int)blocks;
}

int fws_launch_mask_single(void *dev_ptr, uint64_t n, uint32_t key, uint32_t phase, hipStream_t s) {
    if (n == 0) return 0;
    fws_frame_desc one{0, n, key, phase};
    const uint64_t chunks = ((((uintptr_t)dev_ptr) + n + 15u) >> 4) - (((uintptr_t)dev_ptr) >> 4);
    const uint64_t units = (chunks + kUnitChunks - 1) / kUnitChunks;
    hipLaunchKernelGGL(k_unmask<true>, dim3(grid_for_units(units)), dim3(kBlock), 0, s,
                       (uint8_t *)dev_ptr, nullptr, 1u, nullptr, nullptr, nullptr, nullptr, 0ull, one);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_plan(const uint8_t *base, const fws_frame_desc *d, uint32_t n, const uint32_t *n_dev,
                    fws_plan_ws &ws, hipStream_t s) {
    const uint32_t nb = (n + kPlanTile - 1) / kPlanTile;
    hipLaunchKernelGGL(k_plan_count, dim3(nb), dim3(kBlock), 0, s, base, d, n, n_dev, ws.block_sums);
    hipLaunchKernelGGL(k_plan_scan, dim3(nb), dim3(kBlock), 0, s, base, d, n, n_dev, ws.block_sums, ws.cbase,
                       ws.unit_first, ws.total, ws.unit_cap);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_unmask(uint8_t *base, const fws_frame_desc *d, uint32_t n, const uint32_t *n_dev,
                      const fws_plan_ws &ws, uint64_t max_chunks, hipStream_t s) {
    const uint64_t units = (max_chunks + kUnitChunks - 1) / kUnitChunks;
    fws_frame_desc none{0, 0, 0, 0};
    hipLaunchKernelGGL(k_unmask<false>, dim3(grid_for_units(units)), dim3(kBlock), 0, s, base, d, n,
                       n_dev, ws.cbase, ws.unit_first, ws.total, ws.unit_cap, none);
    return fws_hip_status(hipGetLastError());
}
