// tools/bw_probe2.hip -- second HBM ceiling probe (not part of the library):
// one 4 KiB unit per wave (C2's shape: grid = units / 4), in-place 16-B XOR over
// 4 rotating 269 MB buffers, across cache policy per direction, read-only and
// write-only ceilings, LDS-DMA loads, block size and an XCD-contiguous remap.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/bw_probe2 tools/bw_probe2.hip && /tmp/bw_probe2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

// LD/ST: 0 plain, 1 nontemporal. MODE: 0 xor in place, 1 read only, 2 write only.
// REMAP: 0 unit = wave id; 1 = waves of XCD x (block % 8) take the x-th eighth.
template <int BS, int LD, int ST, int MODE, int REMAP>
__global__ __launch_bounds__(BS) void k_unit(u32x4 *__restrict__ buf, uint64_t n16, uint32_t key,
                                             uint32_t *__restrict__ sink) {
    const uint32_t lane = threadIdx.x & 63;
    uint64_t b = blockIdx.x;
    if (REMAP) {
        const uint64_t per = (gridDim.x + 7) / 8;
        b = (b & 7) * per + (b >> 3);
    }
    const uint64_t wave = b * (BS / 64) + (threadIdx.x >> 6);
    const uint64_t base = wave * 256;
    g_u32x4 *p = (g_u32x4 *)buf;
    u32x4 v[4];
    if (MODE != 2) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + j * 64 + lane;
            const uint64_t ii = i < n16 ? i : 0;
            v[j] = LD ? __builtin_nontemporal_load(p + ii) : p[ii];
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = u32x4{key, key + 1, key + 2, (uint32_t)wave};
    }
    if (MODE == 1) {
        u32x4 s = v[0] ^ v[1] ^ v[2] ^ v[3];
        if ((s.x ^ s.y ^ s.z ^ s.w) == key) sink[0] = 1;
        return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = base + j * 64 + lane;
        if (i < n16) {
            const u32x4 w = v[j] ^ key;
            if (ST) __builtin_nontemporal_store(w, p + i); else p[i] = w;
        }
    }
}

// LDS-DMA loads: the wave's 4 KiB lands in LDS by 4 global_load_lds_dwordx4,
// then ds_read_b128, XOR, nontemporal global store.
template <int BS>
__global__ __launch_bounds__(BS) void k_unit_lds(u32x4 *__restrict__ buf, uint64_t n16, uint32_t key) {
    __shared__ u32x4 sm[BS / 64][256];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t wave = (uint64_t)blockIdx.x * (BS / 64) + w;
    const uint64_t base = wave * 256;
    g_u32x4 *p = (g_u32x4 *)buf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = base + j * 64 + lane;
        const uint64_t ii = i < n16 ? i : 0;
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)(p + ii),
                                         (void __attribute__((address_space(3))) *)&sm[w][j * 64], 16, 0, 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint64_t i = base + j * 64 + lane;
        const u32x4 x = sm[w][j * 64 + lane] ^ key;
        if (i < n16) __builtin_nontemporal_store(x, p + i);
    }
}

static hipEvent_t e0, e1;

template <typename F>
static void timeit(const char *name, F launch, double bytes_per_launch) {
    for (int i = 0; i < 4; ++i) launch(i);
    const int steps = 60;
    float best = 1e30f;
    for (int r = 0; r < 4; ++r) {
        hipEventRecord(e0);
        for (int i = 0; i < steps; ++i) launch(i & 3);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double us = best * 1e3 / steps;
    printf("%-34s %8.2f us  %7.1f GB/s\n", name, us, bytes_per_launch / us / 1e3);
    fflush(stdout);
}

int main() {
    const uint64_t bytes = 268959744ull;   // BASELINE C2 wire bytes
    const uint64_t n16 = bytes / 16;
    const uint64_t units = (n16 + 255) / 256;
    u32x4 *bufs[4];
    uint32_t *sink;
    for (int i = 0; i < 4; ++i) { hipMalloc(&bufs[i], bytes); hipMemset(bufs[i], i, bytes); }
    hipMalloc(&sink, 64);
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double rw = 2.0 * bytes, r1 = bytes;
#define U(BS, LD, ST, MODE, REMAP, NAME, BYTES)                                                                 \
    timeit(NAME, [&](int i) {                                                                                   \
        k_unit<BS, LD, ST, MODE, REMAP><<<(unsigned)((units + BS / 64 - 1) / (BS / 64)), BS>>>(bufs[i], n16,     \
                                                                                                0x12345678u, sink); \
    }, BYTES)
    U(256, 1, 1, 0, 0, "xor nt/nt bs256", rw);
    U(256, 0, 1, 0, 0, "xor ld/nt bs256", rw);
    U(256, 1, 0, 0, 0, "xor nt/st bs256", rw);
    U(256, 0, 0, 0, 0, "xor ld/st bs256", rw);
    U(256, 1, 1, 0, 1, "xor nt/nt bs256 xcd-remap", rw);
    U(512, 1, 1, 0, 0, "xor nt/nt bs512", rw);
    U(1024, 1, 1, 0, 0, "xor nt/nt bs1024", rw);
    U(64, 1, 1, 0, 0, "xor nt/nt bs64", rw);
    U(256, 1, 1, 1, 0, "read-only nt", r1);
    U(256, 0, 1, 1, 0, "read-only plain", r1);
    U(256, 1, 1, 2, 0, "write-only nt", r1);
    U(256, 1, 0, 2, 0, "write-only plain", r1);
    timeit("xor lds-dma(nt)/nt bs256", [&](int i) {
        k_unit_lds<256><<<(unsigned)((units + 3) / 4), 256>>>(bufs[i], n16, 0x12345678u);
    }, rw);
    timeit("xor lds-dma(nt)/nt bs512", [&](int i) {
        k_unit_lds<512><<<(unsigned)((units + 7) / 8), 512>>>(bufs[i], n16, 0x12345678u);
    }, rw);
    U(256, 1, 1, 0, 0, "xor nt/nt bs256 (again)", rw);
    return 0;
}
