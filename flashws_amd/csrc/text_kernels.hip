// text_kernels.hip -- per-frame UTF-8 validation (BASELINE config 5) and
// out-of-place unmask + reassembly of a fragmented message (config 4).
//
// UTF-8 (Unicode Table 3-7 / RFC 3629; the reference defines close code 1007
// at net/w_socket.h:41 but never validates): a byte string is well formed iff
// at every offset j the number of lead bytes in j-1..j-3 that still expect a
// continuation at j is exactly [byte j is a continuation], no byte is C0, C1 or
// F5..FF, the second byte after E0/ED/F0/F4 lies in its narrowed range, and
// no lead runs past the end. That test needs only the 3 preceding bytes, so a
// 16-B window is checked independently given its 3-byte left context: one
// wave per frame, 1 KiB per wave step, a wave-wide AND per frame.
#include "fws_device.h"
#include "fws_internal.h"

namespace fwsk {

__device__ __forceinline__ uint32_t utf8_need(uint32_t c) {
    return (c >= 0xC2u && c <= 0xDFu) ? 1u : (c >= 0xE0u && c <= 0xEFu) ? 2u : (c >= 0xF0u && c <= 0xF4u) ? 3u : 0u;
}

// Validate bytes [w, w+16) intersected with [lo, hi); ctx = the up-to-3
// bytes before w that lie in the region (need() of bytes outside is 0).
__device__ __forceinline__ bool utf8_window(const uint8_t *__restrict__ p, uintptr_t w, uintptr_t lo, uintptr_t hi) {
    uint32_t n1 = 0, n2 = 0, n3 = 0;       // need of bytes j-1, j-2, j-3
    uint32_t prev = 0;                     // byte j-1
    for (int b = -3; b < 0; ++b) {
        const uintptr_t a = w + b;
        uint32_t c = 0, nd = 0;
        if (a >= lo && a < hi) { c = p[a - lo]; nd = utf8_need(c); }
        n3 = n2; n2 = n1; n1 = nd; prev = c;
    }
    bool ok = true;
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        const uintptr_t a = w + b;
        if (a < lo || a >= hi) {           // outside: shift an empty byte through
            n3 = n2; n2 = n1; n1 = 0; prev = 0;
            continue;
        }
        const uint32_t c = p[a - lo];
        const uint32_t req = (n1 >= 1u) + (n2 >= 2u) + (n3 >= 3u);
        const bool cont = (c & 0xC0u) == 0x80u;
        ok &= req <= 1u;
        ok &= cont == (req == 1u);
        ok &= !(c == 0xC0u || c == 0xC1u || c >= 0xF5u);
        if (n1 >= 1u) {                    // c is the second byte of prev's sequence
            ok &= !(prev == 0xE0u && c < 0xA0u);
            ok &= !(prev == 0xEDu && c > 0x9Fu);
            ok &= !(prev == 0xF0u && c < 0x90u);
            ok &= !(prev == 0xF4u && c > 0x8Fu);
        }
        const uint32_t nd = utf8_need(c);
        ok &= (uint64_t)nd < (uint64_t)(hi - a);   // the sequence must end inside the region
        n3 = n2; n2 = n1; n1 = nd; prev = c;
    }
    return ok;
}

// One wave per region. kFrames: regions come from fws_frame_info (payload
// after the header; result 0 unless TEXT, FIN and complete).
template <bool kFrames>
__global__ __launch_bounds__(kBlock) void k_utf8(const uint8_t *__restrict__ base, uint64_t N,
                                                 const fws_frame_desc *__restrict__ descs,
                                                 const fws_frame_info *__restrict__ frames, uint32_t n,
                                                 const uint32_t *__restrict__ n_dev, uint8_t *__restrict__ ok_out) {
    if (n_dev && *n_dev < n) n = *n_dev;
    const int lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (kBlock / 64);
    for (uint32_t f = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); f < n; f += nw) {
        uint64_t off, len;
        bool eligible = true;
        if (kFrames) {
            const fws_frame_info fi = frames[f];
            off = fi.hdr_off + fi.hdr_len;
            len = fi.payload_len;
            eligible = fi.opcode == 1u && fi.fin && !(fi.flags & FWS_FRAME_TRUNCATED) && off + len <= N;
        } else {
            off = descs[f].payload_off;
            len = descs[f].payload_len;
        }
        bool ok = eligible;
        if (eligible) {
            const uint8_t *p = base + off;
            const uintptr_t lo = (uintptr_t)p, hi = lo + len;
            for (uintptr_t w = (lo & ~uintptr_t(15)) + uintptr_t(lane) * 16u; w < hi; w += 1024u)
                ok &= utf8_window(p, w, lo, hi);
            ok = __all(ok);
        }
        if (lane == 0) ok_out[f] = ok ? 1 : 0;
    }
}

// ------------------------------------------------------------------ gather
// dst byte space = concatenation of the payload regions (dst_off = exclusive
// prefix of payload_len, built by k_gather_plan*). One wave per 4 KiB unit of
// dst; a full 16-B dst chunk inside one region is two aligned 16-B source
// loads + v_alignbyte + XOR + one 16-B store.
constexpr uint64_t kGatherUnit = 4096;

__global__ __launch_bounds__(kBlock) void k_gather_count(const fws_frame_desc *__restrict__ d, uint32_t n,
                                                         uint64_t *__restrict__ block_sums) {
    __shared__ uint64_t ws[kBlock / 64];
    uint64_t s = 0;
    for (uint32_t i = 0; i < 4; ++i) {
        const uint64_t f = (uint64_t)blockIdx.x * 1024u + threadIdx.x * 4u + i;
        if (f < n) s += d[f].payload_len;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) block_sums[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(kBlock) void k_gather_scan(const fws_frame_desc *__restrict__ d, uint32_t n,
                                                        const uint64_t *__restrict__ block_sums,
                                                        uint64_t *__restrict__ dbase, uint32_t *__restrict__ unit_first,
                                                        uint64_t unit_cap, uint64_t *__restrict__ total_out) {
    __shared__ uint64_t wsum[kBlock / 64];
    __shared__ uint64_t sprefix;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t p = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += kBlock) p += block_sums[b];
    for (int o = 32; o > 0; o >>= 1) p += __shfl_down(p, o, 64);
    if (lane == 0) wsum[w] = p;
    __syncthreads();
    if (threadIdx.x == 0) sprefix = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    const uint64_t f0 = (uint64_t)blockIdx.x * 1024u + threadIdx.x * 4u;
    uint64_t c[4], s = 0;
    for (int i = 0; i < 4; ++i) { c[i] = (f0 + i < n) ? d[f0 + i].payload_len : 0; s += c[i]; }
    uint64_t inc = s;
    for (int o = 1; o < 64; o <<= 1) { const uint64_t x = __shfl_up(inc, o, 64); if (lane >= o) inc += x; }
    __syncthreads();
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t off = sprefix;
    for (int i = 0; i < w; ++i) off += wsum[i];
    uint64_t run = off + inc - s;
    for (int i = 0; i < 4; ++i) {
        const uint64_t f = f0 + i;
        if (f >= n) break;
        dbase[f] = run;
        if (c[i]) {
            uint64_t u = (run + kGatherUnit - 1) / kGatherUnit, ue = (run + c[i] + kGatherUnit - 1) / kGatherUnit;
            if (ue > unit_cap) ue = unit_cap;
            for (; u < ue; ++u) unit_first[u] = (uint32_t)f;
        }
        run += c[i];
        if (f == n - 1) { dbase[n] = run; *total_out = run; }
    }
}

__device__ __forceinline__ u32x4 load16_unaligned(const uint8_t *src) {
    const uintptr_t a = (uintptr_t)src;
    const uintptr_t base = a & ~uintptr_t(15);
    const uint32_t sh = (uint32_t)(a & 15u);
    const u32x4 v0 = *reinterpret_cast<const u32x4 *>(base);
    if (sh == 0) return v0;
    const u32x4 v1 = *reinterpret_cast<const u32x4 *>(base + 16);
    const uint32_t d[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const uint32_t bs = 8u * (sh & 3u);
    u32x4 r;
    switch (sh >> 2) {
#define FWS_AL(i, q) (uint32_t)((((uint64_t)d[(i) + (q) + 1] << 32) | d[(i) + (q)]) >> bs)
    case 0: r = u32x4{FWS_AL(0, 0), FWS_AL(1, 0), FWS_AL(2, 0), FWS_AL(3, 0)}; break;
    case 1: r = u32x4{FWS_AL(0, 1), FWS_AL(1, 1), FWS_AL(2, 1), FWS_AL(3, 1)}; break;
    case 2: r = u32x4{FWS_AL(0, 2), FWS_AL(1, 2), FWS_AL(2, 2), FWS_AL(3, 2)}; break;
    default: r = u32x4{FWS_AL(0, 3), FWS_AL(1, 3), FWS_AL(2, 3), FWS_AL(3, 3)}; break;
#undef FWS_AL
    }
    return r;
}

// Requires dst 16-B aligned. Partial chunks and region seams go byte by byte.
__global__ __launch_bounds__(kBlock) void k_gather(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                                   const fws_frame_desc *__restrict__ d, uint32_t n,
                                                   const uint64_t *__restrict__ dbase,
                                                   const uint32_t *__restrict__ unit_first, uint64_t unit_cap,
                                                   const uint64_t *__restrict__ total_ptr) {
    const uint64_t total = *total_ptr;
    uint64_t n_units = (total + kGatherUnit - 1) / kGatherUnit;
    if (n_units > unit_cap) n_units = unit_cap;
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (kBlock / 64);
    for (uint64_t u = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); u < n_units; u += nw) {
        const uint32_t flo = unit_first[u];
        const uint32_t fhi = (u + 1 < n_units) ? unit_first[u + 1] : n - 1;
        for (int j = 0; j < 4; ++j) {
            const uint64_t a = u * kGatherUnit + (uint64_t)j * 1024u + (uint64_t)lane * 16u;
            if (a >= total) break;
            uint32_t f = find_frame(dbase, flo, fhi, a);
            const uint64_t fb = dbase[f], fe = dbase[f + 1];
            if (a + 16 <= fe && a + 16 <= total) {
                const fws_frame_desc fd = d[f];
                const uint8_t *s = src + fd.payload_off + (a - fb);
                // key byte of dst byte a+i: (a + i - fb + phase) & 3
                const uint32_t rk = rotr32(fd.key, 8u * ((uint32_t)(a - fb + fd.phase) & 3u));
                *reinterpret_cast<u32x4 *>(dst + a) = load16_unaligned(s) ^ rk;
            } else {
                for (uint64_t b = a; b < a + 16 && b < total; ++b) {
                    while (b >= dbase[f + 1]) ++f;
                    const fws_frame_desc fd = d[f];
                    const uint64_t k = b - dbase[f];
                    const uint32_t kb = (fd.key >> (8u * ((uint32_t)(k + fd.phase) & 3u))) & 0xFFu;
                    dst[b] = (uint8_t)(src[fd.payload_off + k] ^ kb);
                }
            }
        }
    }
}

}  // namespace fwsk

using namespace fwsk;

int fws_launch_utf8_frames(const uint8_t *base, uint64_t N, const fws_frame_info *frames, uint32_t n,
                           const uint32_t *n_dev, uint8_t *ok, hipStream_t s) {
    if (n == 0) return 0;
    uint32_t blocks = (n + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_utf8<true>, dim3(blocks), dim3(kBlock), 0, s, base, N, nullptr, frames, n, n_dev, ok);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_utf8_descs(const uint8_t *base, const fws_frame_desc *descs, uint32_t n, uint8_t *ok,
                          hipStream_t s) {
    if (n == 0) return 0;
    uint32_t blocks = (n + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_utf8<false>, dim3(blocks), dim3(kBlock), 0, s, base, ~0ull, descs, nullptr, n, nullptr, ok);
    return fws_hip_status(hipGetLastError());
}

int fws_launch_gather(uint8_t *dst, const uint8_t *src, const fws_frame_desc *d, uint32_t n, fws_plan_ws &ws,
                      uint64_t max_bytes, hipStream_t s) {
    if (n == 0) return 0;
    const uint32_t nb = (n + 1023) / 1024;
    hipLaunchKernelGGL(k_gather_count, dim3(nb), dim3(kBlock), 0, s, d, n, ws.block_sums);
    hipLaunchKernelGGL(k_gather_scan, dim3(nb), dim3(kBlock), 0, s, d, n, ws.block_sums, ws.cbase, ws.unit_first,
                       ws.unit_cap, ws.total);
    uint64_t units = max_bytes / kGatherUnit + 1;
    uint64_t blocks = (units + 3) / 4;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_gather, dim3((unsigned)blocks), dim3(kBlock), 0, s, dst, src, d, n, ws.cbase, ws.unit_first,
                       ws.unit_cap, ws.total);
    return fws_hip_status(hipGetLastError());
}
