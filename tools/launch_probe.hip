// tools/launch_probe.hip -- device-time floor of small metadata kernels on
// MI355X (not part of the library): back-to-back launches of an empty kernel,
// a 64-block kernel that reads 24 B per thread of a 1.5 MB descriptor array,
// the same plus one device-scope atomic per block, and the same after a
// 269 MB streaming kernel (cold TLB / caches). HIP events over 200 launches.
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/launch_probe tools/launch_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void k_empty() {}

template <int MODE>   // 0 read, 1 read + atomic ticket, 2 read + 4 dependent rounds
__global__ __launch_bounds__(256) void k_meta(const uint64_t *__restrict__ d, uint64_t n, uint64_t *out,
                                              uint32_t *ticket) {
    uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x * 4;
    uint64_t s = 0;
    for (int k = 0; k < 4; ++k)
        if (i + k < n) s += d[3 * (i + k)];
    if (MODE == 1 && threadIdx.x == 0) s += atomicAdd(ticket, 1u);
    if (MODE == 2) {
        uint64_t j = s % n;
        for (int r = 0; r < 4; ++r) j = d[3 * (j % n)] % n;
        s += j;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream(u32x4 *p, uint64_t n16) {
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i < n16; i += (uint64_t)gridDim.x * 256) {
        u32x4 v = __builtin_nontemporal_load(p + i);
        v ^= 1u;
        __builtin_nontemporal_store(v, p + i);
    }
}

int main() {
    const uint64_t n = 65536;
    uint64_t *d, *out;
    uint32_t *ticket;
    u32x4 *big;
    const uint64_t big_bytes = 268959744ull;
    hipMalloc(&d, n * 24);
    hipMalloc(&out, 1 << 20);
    hipMalloc(&ticket, 64);
    hipMalloc(&big, big_bytes);
    hipMemset(d, 1, n * 24);
    hipMemset(big, 0, big_bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms;
    auto time = [&](const char *name, auto launch, int reps) {
        for (int i = 0; i < 5; ++i) launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-40s %8.2f us per launch\n", name, ms * 1e3 / reps);
        fflush(stdout);
    };
    time("empty 1 block", [&] { k_empty<<<1, 64>>>(); }, 200);
    time("empty 64 blocks", [&] { k_empty<<<64, 256>>>(); }, 200);
    time("meta read (64 blk)", [&] { k_meta<0><<<64, 256>>>(d, n, out, ticket); }, 200);
    time("meta read + atomic ticket", [&] { k_meta<1><<<64, 256>>>(d, n, out, ticket); }, 200);
    time("meta read + 4 dependent rounds", [&] { k_meta<2><<<64, 256>>>(d, n, out, ticket); }, 200);
    time("meta read x2 (two launches)", [&] {
        k_meta<0><<<64, 256>>>(d, n, out, ticket);
        k_meta<0><<<64, 256>>>(d, n, out, ticket);
    }, 100);
    time("stream 269MB", [&] { k_stream<<<16384, 256>>>(big, big_bytes / 16); }, 40);
    time("stream + meta read", [&] {
        k_stream<<<16384, 256>>>(big, big_bytes / 16);
        k_meta<0><<<64, 256>>>(d, n, out, ticket);
    }, 40);
    time("stream + meta 4 rounds", [&] {
        k_stream<<<16384, 256>>>(big, big_bytes / 16);
        k_meta<2><<<64, 256>>>(d, n, out, ticket);
    }, 40);
    time("stream + empty", [&] {
        k_stream<<<16384, 256>>>(big, big_bytes / 16);
        k_empty<<<64, 256>>>();
    }, 40);
    return 0;
}
