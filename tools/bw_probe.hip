// tools/bw_probe.hip -- HBM streaming ceiling probe on MI355X (not part of the
// library). In-place 16-B XOR (the unmask's access pattern) and out-of-place
// copy over 4 rotating 269 MB buffers (C2's wire size), across unroll depth,
// workgroups and nontemporal policy. Prints GB/s of bytes read + written.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/bw_probe tools/bw_probe.hip && /tmp/bw_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

template <int U, bool NT, bool COPY>
__global__ __launch_bounds__(256) void k_stream(u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, uint64_t n16,
                                                uint32_t key) {
    const uint64_t lane = threadIdx.x & 63, wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
    const uint64_t nwaves = (gridDim.x * 256ull) >> 6;
    const g_u32x4 *s = (const g_u32x4 *)src;
    g_u32x4 *d = (g_u32x4 *)(COPY ? dst : (u32x4 *)src);
    for (uint64_t base = wave * 64 * U; base < n16; base += nwaves * 64 * U) {
        u32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t i = base + j * 64 + lane;
            if (i < n16) v[j] = NT ? __builtin_nontemporal_load(s + i) : s[i];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint64_t i = base + j * 64 + lane;
            if (i < n16) {
                u32x4 w = COPY ? v[j] : (v[j] ^ key);
                if (NT) __builtin_nontemporal_store(w, d + i); else d[i] = w;
            }
        }
    }
}

template <int U, bool NT, bool COPY>
static void run(const char *name, u32x4 **bufs, u32x4 *dst, uint64_t n16, int grid) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 4; ++i) k_stream<U, NT, COPY><<<grid, 256>>>(dst, bufs[i], n16, 0x12345678u);
    const int steps = 40;
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        hipEventRecord(e0);
        for (int i = 0; i < steps; ++i) k_stream<U, NT, COPY><<<grid, 256>>>(dst, bufs[i & 3], n16, 0x12345678u);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double us = best * 1e3 / steps;
    printf("%-10s U=%-2d NT=%d grid=%-6d  %8.2f us  %7.1f GB/s\n", name, U, (int)NT, grid, us, 2.0 * n16 * 16 / us / 1e3);
}

int main() {
    const uint64_t bytes = 268959744ull;   // BASELINE C2 wire bytes
    const uint64_t n16 = bytes / 16;
    u32x4 *bufs[4], *dst;
    for (int i = 0; i < 4; ++i) { hipMalloc(&bufs[i], bytes); hipMemset(bufs[i], i, bytes); }
    hipMalloc(&dst, bytes);
    const int grids[] = {2048, 4096, 8192, 16384, 65536};
    for (int g : grids) {
        run<4, false, false>("xor", bufs, dst, n16, g);
        run<4, true, false>("xor", bufs, dst, n16, g);
        run<8, true, false>("xor", bufs, dst, n16, g);
        run<16, true, false>("xor", bufs, dst, n16, g);
        run<4, false, true>("copy", bufs, dst, n16, g);
        run<4, true, true>("copy", bufs, dst, n16, g);
        run<8, true, true>("copy", bufs, dst, n16, g);
    }
    return 0;
}
