// plan_common.h -- device helpers shared by the batch plans (k_plan,
// k_out_plan): a single-pass block scan with a decoupled look-back over
// epoch-tagged status words, and wave-cooperative unit-map fills.
#pragma once
#include "fws_device.h"

namespace fwsk {

// Look-back word: value (bits 0-44) | flag (45: "sorted" for k_plan) | state
// (46-47: 1 block aggregate, 2 inclusive prefix) | epoch (48-63, the call's
// tag: words of earlier calls are ignored, so nothing is cleared between calls).
constexpr uint64_t kLbValue = (1ull << 45) - 1;
constexpr uint64_t kLbSorted = 1ull << 45;
constexpr uint64_t kLbAgg = 1ull << 46, kLbPrefix = 2ull << 46;

__device__ __forceinline__ uint64_t lb_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v, int lane) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint64_t t = __shfl_up(v, o, kWave);
        if (lane >= o) v += t;
    }
    return v;
}

// The block's order for the look-back: blockIdx for grids that are co-resident
// (<= 1024 blocks of 256 threads), else an ordered ticket, so a block only
// waits on started blocks. Every thread of the block calls it.
__device__ __forceinline__ uint32_t plan_block_order(uint32_t *ticket) {
    __shared__ uint32_t s_blk;
    if (gridDim.x <= 1024u) return blockIdx.x;
    if (threadIdx.x == 0) s_blk = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t blk = s_blk;
    if (blk == gridDim.x - 1 && threadIdx.x == 0) *ticket = 0u;   // every ticket is taken
    return blk;
}

// Block blk's exclusive prefix of the values (agg = the block's sum, flag =
// its flag bit); *all_flag = AND of the flags of blocks 0..blk. Publishes the
// aggregate first, then reads up to 256 earlier blocks' words per round (one
// round covers a 256-block grid) and stops at the nearest inclusive prefix.
// Every thread of the block calls it; all get the result.
__device__ __forceinline__ uint64_t block_lookback(uint64_t *status, uint32_t blk, uint64_t agg, bool flag,
                                                   uint32_t epoch, bool *all_flag) {
    __shared__ uint32_t s_pstop[kBlock / kWave];
    __shared__ uint64_t s_lsum[kBlock / kWave];
    __shared__ uint32_t s_lbad[kBlock / kWave];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const uint64_t tag = (uint64_t)epoch << 48;
    if (threadIdx.x == 0) lb_store(status + blk, tag | (blk == 0 ? kLbPrefix : kLbAgg) | (flag ? kLbSorted : 0) | agg);
    uint64_t excl = 0;
    bool all = flag;
    for (int64_t j = (int64_t)blk - 1; j >= 0; j -= kBlock) {
        const int64_t idx = j - (int64_t)threadIdx.x;
        uint64_t st = tag | kLbPrefix | kLbSorted;     // before block 0: an empty prefix
        if (idx >= 0) {
            do {
                st = lb_load(status + idx);
            } while ((st >> 48) != epoch || (st & (3ull << 46)) == 0);
        }
        const uint64_t pm = __ballot((st & (3ull << 46)) == kLbPrefix);
        if (lane == 0) s_pstop[w] = pm ? (uint32_t)(w * kWave + __builtin_ctzll(pm)) : (uint32_t)kBlock;
        __syncthreads();
        uint32_t stop = kBlock;
#pragma unroll
        for (int i = 0; i < kBlock / kWave; ++i) stop = s_pstop[i] < stop ? s_pstop[i] : stop;
        const bool use = threadIdx.x <= stop && idx >= 0;
        uint64_t v = use ? (st & kLbValue) : 0;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
        const uint64_t vb = __ballot(use && !(st & kLbSorted));
        if (lane == 0) {
            s_lsum[w] = v;
            s_lbad[w] = vb != 0;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kBlock / kWave; ++i) {
            excl += s_lsum[i];
            all = all && !s_lbad[i];
        }
        __syncthreads();                               // s_pstop / s_lsum reused next round
        if (stop < (uint32_t)kBlock) break;
    }
    if (threadIdx.x == 0 && blk != 0)
        lb_store(status + blk, tag | kLbPrefix | (all ? kLbSorted : 0) | ((excl + agg) & kLbValue));
    *all_flag = all;
    return excl;
}

// Longest run of the wave.
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t t = (uint32_t)__shfl_xor(v, o, kWave);
        v = t > v ? t : v;
    }
    return v;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int k) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, k), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), k);
    return ((uint64_t)hi << 32) | lo;
}

constexpr uint32_t kRunInline = 64;     // runs up to this long: each lane writes its own

// For every lane's run [u0, u0 + len): fn(u) for each u, wave-cooperatively.
// When every run is short each lane walks its own; otherwise the lanes' runs
// are taken one at a time (fields broadcast by readlane, `get(L)` returns lane
// L's run context) and the whole wave writes it, 64 entries per step.
template <typename Get, typename Fn>
__device__ __forceinline__ void wave_for_runs(uint64_t u0, uint32_t len, Get get, Fn fn) {
    if (wave_max(len) <= kRunInline) {
        const auto ctx = get(-1);
        for (uint32_t k = 0; k < len; ++k) fn(ctx, u0 + k);
        return;
    }
    const int lane = threadIdx.x & (kWave - 1);
    for (int L = 0; L < kWave; ++L) {
        const uint32_t n = __builtin_amdgcn_readlane(len, L);
        if (n == 0) continue;
        const uint64_t b = readlane64(u0, L);
        const auto ctx = get(L);
        for (uint32_t k = (uint32_t)lane; k < n; k += kWave) fn(ctx, b + k);
    }
}

// map[u0 + k] = f for k < len, for every lane's run (wave_for_runs).
__device__ __forceinline__ void wave_fill_runs(uint32_t *map, uint64_t u0, uint32_t len, uint32_t f, int lane) {
    (void)lane;
    wave_for_runs(u0, len, [&](int L) { return L < 0 ? f : (uint32_t)__builtin_amdgcn_readlane(f, L); },
                  [&](uint32_t fl, uint64_t u) { map[u] = fl; });
}

// Entry u of a unit map (frame f owns the units whose first position lies in
// [prefix_f, prefix_{f+1}), positions in the prefix's units): the map itself
// where the plan wrote it (u < unit_cap), else the same answer by a binary
// search of the prefix (the last f < n with prefix_f <= pos), so a batch larger
// than the context's reservation is still covered in full.
__device__ __forceinline__ uint32_t unit_owner(const uint32_t *__restrict__ map, uint64_t unit_cap,
                                               const uint64_t *__restrict__ prefix, uint32_t n, uint64_t u,
                                               uint64_t pos) {
    if (u < unit_cap) return map[u];
    uint32_t lo = 0, hi = n;                          // prefix[lo] <= pos < prefix[hi] (prefix[n] = total)
    while (hi - lo > 1u) {
        const uint32_t mid = lo + (hi - lo) / 2u;
        if (prefix[mid] <= pos) lo = mid;
        else hi = mid;
    }
    return lo;
}

}  // namespace fwsk
