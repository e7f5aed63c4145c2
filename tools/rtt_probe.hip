// tools/rtt_probe.hip -- where the host read's round trip goes (VERDICT r03:
// the per-read drop-in adds ~24 us of RTT over the reference). Measures, with
// the median of many repetitions on one MI355X:
//   launch_sync      empty kernel + hipStreamSynchronize
//   launch_flag      empty kernel that stores a flag to pinned host memory; the
//                    host spins on the flag (no HIP sync call)
//   d2h64_sync       hipMemcpyAsync D2H of 64 B + hipStreamSynchronize
//   pinned_rw4k      kernel: 4 KiB read + XOR + write on pinned host memory (one
//                    wave per 1 KiB) + sync
//   session_feed     fws_rx_session_feed of one 4 KiB masked frame (the per-read
//                    drop-in path), host buffer in pageable memory
//   session_feed_reg the same on a hipHostRegister-ed buffer (fws_gpu_host_register)
//   mux_feed_N       fws_rx_mux_feed of N connections' 4 KiB reads (N = 1, 8, 64),
//                    in pageable memory (staged) and _reg: registered (in place)
// argv[1] = "spin" sets hipDeviceScheduleSpin before the context, "yield"
// hipDeviceScheduleYield, "block" hipDeviceScheduleBlockingSync, else the default.
// Build: hipcc --offload-arch=gfx950 -O2 -I../include rtt_probe.hip -L../flashws_amd/lib -lfws_gpu
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fws_gpu.h"

using Clock = std::chrono::steady_clock;

__global__ void k_empty() {}

__global__ void k_flag(volatile uint32_t *flag, uint32_t v) {
    if (threadIdx.x == 0) {
        __threadfence_system();
        *flag = v;
    }
}

__global__ void k_rw(uint4 *p, uint32_t key) {
    uint4 v = p[blockIdx.x * 64 + threadIdx.x];
    v.x ^= key; v.y ^= key; v.z ^= key; v.w ^= key;
    p[blockIdx.x * 64 + threadIdx.x] = v;
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}
static double pct(std::vector<double> v, double q) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[std::min(v.size() - 1, size_t(q * double(v.size() - 1)))];
}

template <class F>
static void run(const char *name, int reps, F &&f) {
    for (int i = 0; i < 50; ++i) f();
    std::vector<double> t;
    t.reserve(reps);
    for (int i = 0; i < reps; ++i) {
        const auto a = Clock::now();
        f();
        t.push_back(std::chrono::duration<double, std::micro>(Clock::now() - a).count());
    }
    std::printf("{\"probe\": \"%s\", \"p50_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, \"reps\": %d}\n", name,
                median(t), pct(t, 0.1), pct(t, 0.9), reps);
    std::fflush(stdout);
}

// one masked BIN frame with a 4 KiB payload (8-B header + key)
static void make_frame(std::vector<uint8_t> &w, uint32_t seed) {
    const uint32_t n = 4096;
    w.resize(8 + n);
    w[0] = 0x82;
    w[1] = 0xFE;
    w[2] = n >> 8;
    w[3] = n & 0xFF;
    uint32_t x = seed * 2654435761u + 1;
    for (uint32_t i = 4; i < w.size(); ++i) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; w[i] = uint8_t(x); }
}

int main(int argc, char **argv) {
    const std::string mode = argc > 1 ? argv[1] : "default";
    if (mode == "spin") (void)hipSetDeviceFlags(hipDeviceScheduleSpin);
    else if (mode == "yield") (void)hipSetDeviceFlags(hipDeviceScheduleYield);
    else if (mode == "block") (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
    std::printf("{\"mode\": \"%s\"}\n", mode.c_str());
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    const int reps = 3000;

    run("launch_sync", reps, [&] {
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
        (void)hipStreamSynchronize(st);
    });
    uint32_t *flag = nullptr;
    (void)hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent);
    uint32_t seq = 0;
    run("launch_flag", reps, [&] {
        ++seq;
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, flag, seq);
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) { }
    });
    (void)hipStreamSynchronize(st);
    void *d64 = nullptr, *h64 = nullptr;
    (void)hipMalloc(&d64, 64);
    (void)hipHostMalloc(&h64, 64);
    run("d2h64_sync", reps, [&] {
        (void)hipMemcpyAsync(h64, d64, 64, hipMemcpyDeviceToHost, st);
        (void)hipStreamSynchronize(st);
    });
    uint4 *pin = nullptr;
    (void)hipHostMalloc((void **)&pin, 4096);
    run("pinned_rw4k", reps, [&] {
        hipLaunchKernelGGL(k_rw, dim3(4), dim3(64), 0, st, pin, 0x5Au);
        (void)hipStreamSynchronize(st);
    });

    fws_gpu_ctx *ctx = nullptr;
    if (fws_gpu_ctx_create(0, &ctx) != 0) { std::printf("{\"error\": \"ctx\"}\n"); return 1; }
    std::vector<uint8_t> frame;
    make_frame(frame, 1);
    const size_t cap = 64 << 10;
    std::vector<fws_rx_event> ev(64);
    std::vector<uint8_t> ctl(256);
    {
        fws_rx_session *s = nullptr;
        fws_rx_session_create(ctx, 1, &s);
        std::vector<uint8_t> buf(cap);
        uint64_t ne = 0, cu = 0;
        run("session_feed", reps, [&] {
            std::memcpy(buf.data(), frame.data(), frame.size());
            const int r = fws_rx_session_feed(s, buf.data(), frame.size(), cap, ev.data(), ev.size(), &ne,
                                              ctl.data(), ctl.size(), &cu);
            if (r != 0 || ne != 1) std::abort();
        });
        uint8_t *reg = (uint8_t *)aligned_alloc(4096, cap);
        fws_gpu_host_register(reg, cap);
        run("session_feed_reg", reps, [&] {
            std::memcpy(reg, frame.data(), frame.size());
            const int r = fws_rx_session_feed(s, reg, frame.size(), cap, ev.data(), ev.size(), &ne, ctl.data(),
                                              ctl.size(), &cu);
            if (r != 0 || ne != 1) std::abort();
        });
        fws_gpu_host_unregister(reg);
        std::free(reg);
        fws_rx_session_destroy(s);
    }
    for (int reg = 0; reg < 2; ++reg) {
        for (uint32_t n : {1u, 8u, 64u}) {
            fws_rx_mux *m = nullptr;
            fws_rx_mux_create(ctx, n, &m);
            // the reads in pageable memory (staged) or in registered memory (in place)
            uint8_t *arena = (uint8_t *)aligned_alloc(4096, (size_t)n * cap);
            if (reg) fws_gpu_host_register(arena, (uint64_t)n * cap);
            std::vector<fws_rx_read> rd(n);
            std::vector<fws_rx_read_result> res(n);
            const std::string name = std::string("mux_feed_") + std::to_string(n) + (reg ? "_reg" : "");
            run(name.c_str(), reps / 4, [&] {
                for (uint32_t i = 0; i < n; ++i) {
                    uint8_t *b = arena + (size_t)i * cap;
                    std::memcpy(b, frame.data(), frame.size());
                    rd[i] = fws_rx_read{i, 0u, b, frame.size(), cap};
                }
                if (fws_rx_mux_feed(m, rd.data(), n, res.data()) != 0) std::abort();
                for (uint32_t i = 0; i < n; ++i)
                    if (res[i].ret != 0 || res[i].n_events != 1) std::abort();
            });
            if (reg) fws_gpu_host_unregister(arena);
            std::free(arena);
            fws_rx_mux_destroy(m);
        }
    }
    fws_gpu_ctx_destroy(ctx);
    return 0;
}
