// tools/bw_probe3.hip -- r06 HBM ceiling probe (not part of the library): the
// in-place 16-B XOR of bw_probe2 (C2's 269 MB wire, 4 rotating buffers,
// nontemporal loads and stores) at 1, 2 and 4 units of 4 KiB per wave (all
// loads of a wave issued before its first store), and the 1-unit form with
// a dependent scalar load ahead of the data loads (the latency a descriptor
// lookup puts in front of a unit).
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/bw_probe3 tools/bw_probe3.hip && tools/bin/bw_probe3
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error %s line %d\n", #x, __LINE__); return 1; } } while (0)

// a 16-B store with an explicit cache policy (ST: 1 sc1, 2 sc0 sc1, 3 sc1 nt); the
// trailing s_nop covers the store-data hazard (the compiler pads nothing in asm)
template <int ST>
__device__ __forceinline__ void store_pol(g_u32x4 *p, u32x4 v) {
    if constexpr (ST == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (ST == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" :: "v"(p), "v"(v) : "memory");
}

// One unit's four 16-B loads with an explicit cache policy, issued and waited in
// one asm statement (the compiler does not count asm loads): LD 1 sc1 nt, 2 sc0
// nt, 3 sc0 sc1 nt, 4 sc1.
template <int LD>
__device__ __forceinline__ void load4_pol(const g_u32x4 *p0, const g_u32x4 *p1, const g_u32x4 *p2, const g_u32x4 *p3,
                                          u32x4 (&v)[4]) {
#define LD4(POL)                                                                                              \
    asm volatile("global_load_dwordx4 %0, %4, off " POL "\n\tglobal_load_dwordx4 %1, %5, off " POL           \
                 "\n\tglobal_load_dwordx4 %2, %6, off " POL "\n\tglobal_load_dwordx4 %3, %7, off " POL       \
                 "\n\ts_waitcnt vmcnt(0)"                                                                   \
                 : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])                                      \
                 : "v"(p0), "v"(p1), "v"(p2), "v"(p3)                                                      \
                 : "memory")
    if constexpr (LD == 1) LD4("sc1 nt");
    else if constexpr (LD == 2) LD4("sc0 nt");
    else if constexpr (LD == 3) LD4("sc0 sc1 nt");
    else LD4("sc1");
#undef LD4
}

template <int LD>
__global__ __launch_bounds__(256) void k_xor_ld(u32x4 *__restrict__ buf, uint64_t n16, uint32_t key) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t base = wave * 256;
    g_u32x4 *p = (g_u32x4 *)buf;
    uint64_t ii[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = base + j * 64 + lane;
        ii[j] = i < n16 ? i : 0;
    }
    u32x4 v[4];
    load4_pol<LD>(p + ii[0], p + ii[1], p + ii[2], p + ii[3], v);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = base + j * 64 + lane;
        if (i < n16) store_pol<3>(p + i, v[j] ^ key);
    }
}

// U units of 4 KiB per wave; DEP: 0 none, 1 one scalar load (a per-unit word) before
// the data loads; ST: 0 nontemporal stores, else store_pol<ST>
template <int U, int DEP, int ST = 0>
__global__ __launch_bounds__(256) void k_xor(u32x4 *__restrict__ buf, uint64_t n16, uint32_t key,
                                             const uint32_t *__restrict__ words) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t base = wave * 256 * U;
    uint32_t k = key;
    if (DEP) k ^= words[wave & 1023];
    g_u32x4 *p = (g_u32x4 *)buf;
    u32x4 v[4 * U];
#pragma unroll
    for (int j = 0; j < 4 * U; ++j) {
        const uint64_t i = base + j * 64 + lane;
        v[j] = __builtin_nontemporal_load(p + (i < n16 ? i : 0));
    }
#pragma unroll
    for (int j = 0; j < 4 * U; ++j) {
        const uint64_t i = base + j * 64 + lane;
        if (i < n16) {
            if constexpr (ST == 0) __builtin_nontemporal_store(v[j] ^ k, p + i);
            else store_pol<ST>(p + i, v[j] ^ k);
        }
    }
}

// Out of place with the source 8 B off the destination's 16-B grid (C4's and
// TX's shifted windows): dst chunk a = src bytes [a + 8, a + 24) ^ key.
// SH 0: two aligned default-policy loads per chunk (v1 of lane L = v0 of lane
// L + 1, served by the cache: k_gather_one's form); SH 1: one nontemporal load
// per chunk and v1 from the next lane by a DPP wave shift (lane 63: lane 0 of
// the next chunk, the unit's last one loaded); SH 2: SH 1 with default-policy loads.
__device__ __forceinline__ u32x4 shl_lane(const u32x4 &v) {   // lane L gets lane L + 1's value (wave_shl:1)
    return u32x4{(uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.x, 0x130, 0xF, 0xF, false),
                 (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.y, 0x130, 0xF, 0xF, false),
                 (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.z, 0x130, 0xF, 0xF, false),
                 (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.w, 0x130, 0xF, 0xF, false)};
}
__device__ __forceinline__ u32x4 bcast0(const u32x4 &v) {
    return u32x4{(uint32_t)__builtin_amdgcn_readlane((int)v.x, 0), (uint32_t)__builtin_amdgcn_readlane((int)v.y, 0),
                 (uint32_t)__builtin_amdgcn_readlane((int)v.z, 0), (uint32_t)__builtin_amdgcn_readlane((int)v.w, 0)};
}
template <int SH>
__global__ __launch_bounds__(256) void k_shift(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, uint64_t n16,
                                               uint32_t key) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t base = wave * 256;                 // in 16-B blocks; src has n16 + 1 blocks
    const g_u32x4 *s = (const g_u32x4 *)src;
    g_u32x4 *d = (g_u32x4 *)dst;
    u32x4 v0[4], v1[4];
    if (SH == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + j * 64 + lane;
            const uint64_t ii = i < n16 ? i : 0;
            uint64_t i1 = ii + 1;
            asm volatile("" : "+v"(i1));
            v0[j] = s[ii];
            v1[j] = s[i1];
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + j * 64 + lane;
            v0[j] = SH == 1 ? __builtin_nontemporal_load(s + (i < n16 ? i : 0)) : s[i < n16 ? i : 0];
        }
        u32x4 last = u32x4{0u, 0u, 0u, 0u};
        if (lane == 63) {
            const uint64_t i = base + 256;
            last = SH == 1 ? __builtin_nontemporal_load(s + (i <= n16 ? i : 0)) : s[i <= n16 ? i : 0];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            v1[j] = shl_lane(v0[j]);
            const u32x4 nx = j < 3 ? bcast0(v0[j < 3 ? j + 1 : 0]) : last;
            if (lane == 63) v1[j] = nx;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = base + j * 64 + lane;
        const u32x4 w = u32x4{v0[j].z, v0[j].w, v1[j].x, v1[j].y} ^ key;   // bytes 8..23
        if (i < n16) __builtin_nontemporal_store(w, d + i);
    }
}

static hipEvent_t e0, e1;

template <typename F>
static void timeit(const char *name, F launch, double bytes) {
    for (int i = 0; i < 8; ++i) launch(i & 3);
    hipError_t err = hipDeviceSynchronize();
    if (err == hipSuccess) err = hipGetLastError();
    if (err != hipSuccess) {
        printf("%-36s error %s\n", name, hipGetErrorString(err));
        return;
    }
    const int steps = 100;
    float t[5] = {};
    for (int r = 0; r < 5; ++r) {
        if (hipEventRecord(e0, 0) != hipSuccess) printf("record e0 failed\n");
        for (int i = 0; i < steps; ++i) launch(i & 3);
        if (hipEventRecord(e1, 0) != hipSuccess) printf("record e1 failed\n");
        if (hipEventSynchronize(e1) != hipSuccess) printf("sync failed\n");
        const hipError_t q = hipEventElapsedTime(&t[r], e0, e1);
        if (q != hipSuccess) printf("elapsed failed: %s\n", hipGetErrorString(q));
    }
    float best = t[0], sum = 0;
    for (int r = 0; r < 5; ++r) { best = t[r] < best ? t[r] : best; sum += t[r]; }
    printf("%-36s best %7.2f us  mean %7.2f us  %7.1f GB/s (best)\n", name, best * 1e3 / steps, sum / 5 * 1e3 / steps,
           bytes / (best * 1e3 / steps) / 1e3);
    fflush(stdout);
}

// Out of place, no shift: dst block i = src block i ^ key (nontemporal both ways)
__global__ __launch_bounds__(256) void k_copy_xor(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, uint64_t n16,
                                                  uint32_t key) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t base = wave * 256;
    u32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = base + j * 64 + lane;
        v[j] = __builtin_nontemporal_load((const g_u32x4 *)src + (i < n16 ? i : 0));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = base + j * 64 + lane;
        if (i < n16) __builtin_nontemporal_store(v[j] ^ key, (g_u32x4 *)dst + i);
    }
}

// r06 "oop" mode: the out-of-place forms with ONE source (re-read every step, as
// bench.py's C4 / TX did up to r06) against FOUR rotating sources (1 GiB, past
// the 256 MB Infinity Cache), beside the in-place XOR
static int oop_mode(u32x4 **bufs, uint64_t bytes, uint64_t n16) {
    u32x4 *srcs[4];
    for (int i = 0; i < 4; ++i) { CK(hipMalloc(&srcs[i], bytes + 64)); CK(hipMemset(srcs[i], 7 + i, bytes + 64)); }
    const double cb = 2.0 * bytes;
    const unsigned g1 = (unsigned)((n16 / 256 + 1 + 3) / 4);
    for (int rep = 0; rep < 2; ++rep) {
        timeit("in-place xor (4 buffers)", [&](int i) {
            k_xor<1, 0, 0><<<(unsigned)(((n16 + 255) / 256 + 3) / 4), 256>>>(bufs[i & 3], n16, 0x12345678u, nullptr);
        }, cb);
        timeit("copy xor, 1 src", [&](int i) { k_copy_xor<<<g1, 256>>>(srcs[0], bufs[i & 3], n16, 1u); }, cb);
        timeit("copy xor, 4 src", [&](int i) { k_copy_xor<<<g1, 256>>>(srcs[i & 3], bufs[i & 3], n16, 1u); }, cb);
        timeit("shift, 2 loads (cached), 1 src", [&](int i) { k_shift<0><<<g1, 256>>>(srcs[0], bufs[i & 3], n16, 1u); }, cb);
        timeit("shift, 2 loads (cached), 4 src", [&](int i) { k_shift<0><<<g1, 256>>>(srcs[i & 3], bufs[i & 3], n16, 1u); }, cb);
        timeit("shift, 1 nt load + DPP, 4 src", [&](int i) { k_shift<1><<<g1, 256>>>(srcs[i & 3], bufs[i & 3], n16, 1u); }, cb);
        timeit("shift, 1 cached load + DPP, 4 src", [&](int i) { k_shift<2><<<g1, 256>>>(srcs[i & 3], bufs[i & 3], n16, 1u); }, cb);
    }
    return 0;
}

int main(int argc, char **argv) {
    const bool oop = argc > 1 && argv[1][0] == 'o';
    const bool quick = argc > 1 && !oop;   // one variant, one repetition (counter passes)
    const uint64_t bytes = 268959744ull;
    const uint64_t n16 = bytes / 16;
    u32x4 *bufs[4];
    uint32_t *words;
    for (int i = 0; i < 4; ++i) { CK(hipMalloc(&bufs[i], bytes)); CK(hipMemset(bufs[i], i, bytes)); }
    CK(hipMalloc(&words, 4096));
    CK(hipMemset(words, 0, 4096));
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    if (oop) return oop_mode(bufs, bytes, n16);
    const double rw = 2.0 * bytes;
    for (int rep = 0; rep < (quick ? 1 : 2); ++rep) {
#define X(U, DEP, ST, NAME)                                                                                    \
        timeit(NAME, [&](int i) {                                                                              \
            const uint64_t waves = (n16 + 256 * U - 1) / (256 * U);                                            \
            k_xor<U, DEP, ST><<<(unsigned)((waves + 3) / 4), 256>>>(bufs[i & 3], n16, 0x12345678u, words);    \
        }, rw)
        X(1, 0, 0, "xor 1 unit/wave");
        if (quick) break;
        X(2, 0, 0, "xor 2 units/wave");
        X(4, 0, 0, "xor 4 units/wave");
        X(1, 1, 0, "xor 1 unit/wave, scalar dep first");
        X(1, 0, 1, "xor 1 unit/wave, sc1 stores");
        X(1, 0, 2, "xor 1 unit/wave, sc0 sc1 stores");
        X(1, 0, 3, "xor 1 unit/wave, sc1 nt stores");
#define XL(LD, NAME)                                                                                           \
        timeit(NAME, [&](int i) {                                                                              \
            k_xor_ld<LD><<<(unsigned)(((n16 + 255) / 256 + 3) / 4), 256>>>(bufs[i & 3], n16, 0x12345678u);       \
        }, rw)
        XL(1, "sc1 nt loads, sc1 nt stores");
        XL(2, "sc0 nt loads, sc1 nt stores");
        XL(3, "sc0 sc1 nt loads, sc1 nt stores");
        XL(4, "sc1 loads, sc1 nt stores");
    }
    // shifted out-of-place copy: src 269 MB + 16 B, 4 rotating destinations
    if (!quick) {
        u32x4 *src;
        CK(hipMalloc(&src, bytes + 64));
        CK(hipMemset(src, 7, bytes + 64));
        const double cb = 2.0 * bytes;
        for (int rep = 0; rep < 2; ++rep) {
            timeit("shift copy, 2 loads/chunk (cached)", [&](int i) {
                k_shift<0><<<(unsigned)((n16 / 256 + 1 + 3) / 4), 256>>>(src, bufs[i & 3], n16, 0x12345678u);
            }, cb);
            timeit("shift copy, 1 nt load + DPP shift", [&](int i) {
                k_shift<1><<<(unsigned)((n16 / 256 + 1 + 3) / 4), 256>>>(src, bufs[i & 3], n16, 0x12345678u);
            }, cb);
            timeit("shift copy, 1 cached load + DPP shift", [&](int i) {
                k_shift<2><<<(unsigned)((n16 / 256 + 1 + 3) / 4), 256>>>(src, bufs[i & 3], n16, 0x12345678u);
            }, cb);
        }
    }
    return 0;
}
