// tools/vram_probe.hip -- can the host push a read into device memory faster
// than the device pulls it over PCIe? (the persistent receive decode's floor,
// DESIGN.md §4.5). A resident one-workgroup kernel answers requests; the host
// spins on the answer in coherent pinned memory. Request forms, p50 / p10 /
// p90 round trips over `reps` requests each:
//   pinned_flag    doorbell in coherent pinned host memory (the service's form)
//   pinned_4k      + the kernel reads 4 KiB from pinned host memory (a pull)
//   vram_flag      doorbell in fine-grained device memory, written by the CPU
//                  through its host mapping (hipExtMallocWithFlags fine-grained)
//   vram_4k        + the CPU first copies 4 KiB into device memory (a push)
//   *_writeback    + the kernel writes the 4 KiB back to pinned host memory
//                  before it answers (the in-place decode's store)
// A CPU store to device memory goes through write-combining buffers: the
// doorbell is followed by sfence, else it can wait there for milliseconds.
// Every answer carries a checksum of the 4 KiB the kernel read, checked.
// The kernel exits on a quit request or after 2 s without one.
//
// build: hipcc --offload-arch=gfx950 -O2 -o tools/bin/vram_probe tools/vram_probe.hip
#include <hip/hip_runtime.h>
#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

// door[0] = seq (0 = none), door[1] = quit, door[2] = bytes to read (0 or 4096),
// door[3] = 1: write the 4 KiB back (XOR 1) to `out` in pinned host memory first
__global__ void k_answer(const volatile uint32_t *door, const uint32_t *data, uint32_t *ack, uint64_t idle_ticks,
                         uint32_t *out) {
    __shared__ uint32_t s_cmd[4];
    __shared__ uint32_t s_sum[16];
    uint32_t last = 0;
    uint64_t t0 = wall_clock64();
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t seq, q, nb;
            for (;;) {
                seq = __hip_atomic_load((const uint32_t *)&door[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                q = __hip_atomic_load((const uint32_t *)&door[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (q || seq != last) break;
                if (wall_clock64() - t0 > idle_ticks) { q = 1; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            nb = __hip_atomic_load((const uint32_t *)&door[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const uint32_t wb = __hip_atomic_load((const uint32_t *)&door[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            s_cmd[0] = seq;
            s_cmd[1] = q;
            s_cmd[2] = nb;
            s_cmd[3] = wb;
        }
        __syncthreads();
        const uint32_t seq = s_cmd[0];
        if (s_cmd[1]) return;
        // the data: 4 KiB = 256 threads x 16 B, one load each, summed
        uint32_t v = 0;
        if (s_cmd[2] && threadIdx.x < 256) {         // (after thread 0's system-scope acquire)
            const uint4 x = reinterpret_cast<const uint4 *>(data)[threadIdx.x];
            v = x.x + x.y + x.z + x.w;
            if (s_cmd[3]) reinterpret_cast<uint4 *>(out)[threadIdx.x] = uint4{x.x ^ 1u, x.y ^ 1u, x.z ^ 1u, x.w ^ 1u};
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t sum = 0;
            for (uint32_t w = 0; w < blockDim.x / 64; ++w) sum += s_sum[w];
            __hip_atomic_store(&ack[1], sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __hip_atomic_store(&ack[0], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        last = seq;
        t0 = wall_clock64();
        __syncthreads();
    }
}

static sigjmp_buf g_jb;
static void on_fault(int) { siglongjmp(g_jb, 1); }

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5000;
    int khz = 0;
    CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
    const uint64_t idle = (uint64_t)khz * 2000u;            // 2 s
    uint32_t *ack = nullptr, *hdoor = nullptr, *hdata = nullptr, *hout = nullptr;
    CK(hipHostMalloc((void **)&hout, 4096, hipHostMallocCoherent));
    CK(hipHostMalloc((void **)&ack, 64, hipHostMallocCoherent));
    CK(hipHostMalloc((void **)&hdoor, 64, hipHostMallocCoherent));
    CK(hipHostMalloc((void **)&hdata, 4096, hipHostMallocCoherent));
    uint32_t *vdoor = nullptr, *vdata = nullptr;
    CK(hipExtMallocWithFlags((void **)&vdoor, 4096, hipDeviceMallocFinegrained));
    CK(hipExtMallocWithFlags((void **)&vdata, 4096, hipDeviceMallocFinegrained));
    hipPointerAttribute_t at{};
    CK(hipPointerGetAttributes(&at, vdoor));
    printf("{\"vram_attr\": {\"type\": %d, \"device\": %d, \"hostPointer\": \"%p\", \"devicePointer\": \"%p\"}}\n",
           (int)at.type, at.device, at.hostPointer, at.devicePointer);
    // can the CPU write it through the same pointer?
    struct sigaction sa{}, o1{}, o2{};
    sa.sa_handler = on_fault;
    sigaction(SIGSEGV, &sa, &o1);
    sigaction(SIGBUS, &sa, &o2);
    bool cpu_ok = false;
    if (!sigsetjmp(g_jb, 1)) {
        volatile uint32_t *p = vdoor;
        p[3] = 0x1234u;
        cpu_ok = p[3] == 0x1234u;
    }
    sigaction(SIGSEGV, &o1, nullptr);
    sigaction(SIGBUS, &o2, nullptr);
    printf("{\"cpu_write_vram\": %s}\n", cpu_ok ? "true" : "false");
    fflush(stdout);
    std::vector<uint32_t> payload(1024);
    uint32_t want = 0;
    for (int i = 0; i < 1024; ++i) {
        payload[i] = (uint32_t)(i * 2654435761u);
        want += payload[i];
    }
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    struct Mode { const char *name; bool vram; uint32_t nb, wb; };
    std::vector<Mode> modes = {{"pinned_flag", false, 0, 0}, {"pinned_4k", false, 4096, 0},
                               {"pinned_4k_writeback", false, 4096, 1}};
    if (cpu_ok) {
        modes.push_back({"vram_flag", true, 0, 0});
        modes.push_back({"vram_4k", true, 4096, 0});
        modes.push_back({"vram_4k_writeback", true, 4096, 1});
    }
    for (const Mode &m : modes) {
        volatile uint32_t *door = m.vram ? vdoor : hdoor;
        uint32_t *data = m.vram ? vdata : hdata;
        door[0] = 0;
        door[1] = 0;
        door[2] = m.nb;
        door[3] = m.wb;
        __builtin_ia32_sfence();
        ack[0] = 0;
        ack[1] = 0;
        memcpy(hdata, payload.data(), 4096);
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_answer, dim3(1), dim3(1024), 0, st, (const volatile uint32_t *)door, (const uint32_t *)data,
                           ack, idle, hout);
        CK(hipGetLastError());
        std::vector<double> us;
        bool bad = false;
        for (int i = 1; i <= reps + 200 && !bad; ++i) {
            want += (uint32_t)i - payload[0];               // a new first word per request: stale data fails
            payload[0] = (uint32_t)i;
            const auto t0 = std::chrono::steady_clock::now();
            if (m.nb) {
                if (m.vram) memcpy(vdata, payload.data(), 4096);   // the push (write-combined stores)
                else memcpy(hdata, payload.data(), 4096);
            }
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            __atomic_store_n((uint32_t *)&door[0], (uint32_t)i, __ATOMIC_RELEASE);
            if (m.vram) __builtin_ia32_sfence();            // out of the write-combining buffers now
            const auto tw = std::chrono::steady_clock::now();
            while (__atomic_load_n(&ack[0], __ATOMIC_ACQUIRE) != (uint32_t)i) {
                if (std::chrono::steady_clock::now() - tw > std::chrono::seconds(1)) { bad = true; break; }
            }
            const auto t1 = std::chrono::steady_clock::now();
            if (!bad && m.nb && __atomic_load_n(&ack[1], __ATOMIC_ACQUIRE) != want) {
                fprintf(stderr, "%s: checksum %u != %u at %d\n", m.name, ack[1], want, i);
                bad = true;
            }
            if (i > 200) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        __atomic_store_n((uint32_t *)&door[1], 1u, __ATOMIC_RELEASE);
        __builtin_ia32_sfence();
        CK(hipStreamSynchronize(st));
        if (bad || us.empty()) {
            printf("{\"mode\": \"%s\", \"error\": \"no answer or bad checksum\"}\n", m.name);
            continue;
        }
        std::sort(us.begin(), us.end());
        printf("{\"mode\": \"%s\", \"p10_us\": %.2f, \"p50_us\": %.2f, \"p90_us\": %.2f, \"p99_us\": %.2f, \"reps\": %zu}\n",
               m.name, us[us.size() / 10], us[us.size() / 2], us[us.size() * 9 / 10], us[us.size() * 99 / 100],
               us.size());
        fflush(stdout);
    }
    return 0;
}
