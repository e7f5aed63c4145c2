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
// wave per frame, 1 KiB per wave step, bytewise in 32-bit SWAR, a wave-wide
// OR of the error flags per frame.
#include "fws_device.h"
#include "fws_internal.h"
#include "plan_common.h"

namespace fwsk {

// One wave per region, 1 KiB per step (lane L: the 16-B chunk at 16 L); the
// 3-byte left context of a chunk is the previous lane's last dword (lane 0:
// lane 63's of the previous step; none before the region). Chunks run to
// hi + 3 so an unfinished sequence at the end meets zero bytes.
// kFrames: regions come from fws_frame_info (payload after the header; result
// 0 unless TEXT, FIN and complete).
template <bool kFrames>
__global__ __launch_bounds__(kBlock) void k_utf8(const uint8_t *__restrict__ base, uint64_t N,
                                                 const fws_frame_desc *__restrict__ descs,
                                                 const fws_frame_info *__restrict__ frames, uint32_t n,
                                                 const uint32_t *__restrict__ n_dev, uint8_t *__restrict__ ok_out) {
    if (n_dev && *n_dev < n) n = *n_dev;
    const int lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (kBlock / 64);
    for (uint32_t f = blockIdx.x * (kBlock / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); f < n; f += nw) {
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
        uint32_t bad = 0;
        if (eligible) {
            const uintptr_t lo = (uintptr_t)(base + off), hi = lo + len;
            uint32_t carry = 0;                      // lane 63's last dword of the previous step
            for (uintptr_t w0 = lo & ~uintptr_t(15); w0 < hi + 3u; w0 += 1024u) {
                const uintptr_t w = w0 + uintptr_t(lane) * 16u;
                u32x4 v{0u, 0u, 0u, 0u};
                if (w < hi) v = gload16(w);
                v.x &= sel_bytes(w, lo, hi);
                v.y &= sel_bytes(w + 4u, lo, hi);
                v.z &= sel_bytes(w + 8u, lo, hi);
                v.w &= sel_bytes(w + 12u, lo, hi);
                uint32_t prev = __shfl_up(v.w, 1, 64);
                if (lane == 0) prev = carry;
                carry = __shfl(v.w, 63, 64);
                if (w < hi + 3u && ((v.x | v.y | v.z | v.w | prev) & 0x80808080u))
                    bad |= utf8_err(v.x, prev) | utf8_err(v.y, v.x) | utf8_err(v.z, v.y) | utf8_err(v.w, v.z);
            }
        }
        const bool ok = eligible && !__any(bad != 0);
        if (lane == 0) ok_out[f] = ok ? 1 : 0;
    }
}

// ------------------------------------------------------------------ gather
// Out-of-place reassembly of a fragmented message (C4): dst byte space = the
// payload regions concatenated (dbase = exclusive prefix of payload_len), each
// byte XORed with its region's key at its region-relative phase. That is the
// concatenation of the on_read() parts (w_socket.h:713-747), the user-level copy
// of tests/new-ws-echo/test_ws_server.cpp:205-206.
//
// Plan: k_out_plan (outplan_kernels.hip: dbase, the unit map unit_first[u] = the
// region holding byte u * 4 KiB, and the total, in one launch).
// k_gather_fast: one wave per 4 KiB dst unit (4 steps of 64 lanes x 16 B).
// When the unit meets at most 2 regions (regions >= 4 KiB, as C4's 4 KiB..1 MiB
// fragments) their metadata is wave-uniform (scalar loads); a dst chunk inside
// one region is two aligned 16-B source loads shifted by the region's source
// misalignment, XORed and stored; all 8 loads of a lane are issued before the
// first use. A chunk on a region seam (<= 1 per region) goes byte by byte;
// units with more regions take the per-chunk search path.
constexpr uint64_t kGatherUnit = 4096;

// 16 bytes starting sh (0..15) bytes into the 32-byte window v0:v1
__device__ __forceinline__ u32x4 shr_bytes(const u32x4 &v0, const u32x4 &v1, uint32_t sh) {
    const bool s8 = (sh & 8u) != 0, s4 = (sh & 4u) != 0;
    const uint32_t a0 = s8 ? v0.z : v0.x, a1 = s8 ? v0.w : v0.y, a2 = s8 ? v1.x : v0.z;
    const uint32_t a3 = s8 ? v1.y : v0.w, a4 = s8 ? v1.z : v1.x;
    const uint32_t c0 = s4 ? a1 : a0, c1 = s4 ? a2 : a1, c2 = s4 ? a3 : a2, c3 = s4 ? a4 : a3;
    const uint32_t c4 = s4 ? (s8 ? v1.w : v1.y) : a4;
    const uint32_t b = sh & 3u;
    return u32x4{__builtin_amdgcn_alignbyte(c1, c0, b), __builtin_amdgcn_alignbyte(c2, c1, b),
                 __builtin_amdgcn_alignbyte(c3, c2, b), __builtin_amdgcn_alignbyte(c4, c3, b)};
}

// dst bytes [a, min(a + 16, total)) one by one (region seams, the tail)
__device__ __forceinline__ void gather_bytes(uint8_t *dst, const uint8_t *src, const fws_frame_desc *__restrict__ d,
                                             const uint64_t *__restrict__ dbase, uint32_t f, uint64_t a,
                                             uint64_t total) {
    for (uint64_t b = a; b < a + 16 && b < total; ++b) {
        while (b >= dbase[f + 1]) ++f;
        const fws_frame_desc fd = d[f];
        const uint64_t k = b - dbase[f];
        const uint32_t kb = (fd.key >> (8u * ((uint32_t)(k + fd.phase) & 3u))) & 0xFFu;
        dst[b] = (uint8_t)(src[fd.payload_off + k] ^ kb);
    }
}

// Byte-select mask of the chunk's bytes [lo, hi) (offsets 0..16) for dword i
__device__ __forceinline__ uint32_t chunk_sel(uint32_t lo, uint32_t hi, int i) {
    const uint32_t o = 4u * (uint32_t)i;
    if (hi <= o || lo >= o + 4u) return 0u;
    const uint32_t s = lo > o ? lo - o : 0u, e = hi < o + 4u ? o + 4u - hi : 0u;
    return (0xFFFFFFFFu << (8u * s)) & (0xFFFFFFFFu >> (8u * e));
}
__device__ __forceinline__ uint32_t chunk_rel(uint64_t x, uint64_t a) {   // x clipped to [a, a + 16), from a
    return x <= a ? 0u : (x >= a + 16u ? 16u : (uint32_t)(x - a));
}

// dst chunk [a, min(a + 16, total)) of a unit whose regions flo (dst [B0, B1)) and
// fhi (from B1 to B2; two = fhi > flo) cover it, in registers (r06): each
// region's keyed 16-B source window (two aligned loads, a block outside the
// region's source bytes replaced by the region's first block), bytes selected
// per region. The chunks at region seams and the output's end took a
// per-byte loop with three dependent loads per byte (gather_bytes: ~48 round
// trips on the one lane of the wave that had one). Returns false (nothing
// written) when a third region meets the chunk.
__device__ __forceinline__ bool gather_seam(uint8_t *dst, const uint8_t *src, uint64_t a, uint64_t total,
                                            const fws_frame_desc &d0, const fws_frame_desc &d1, uint64_t B0,
                                            uint64_t B1, uint64_t B2, bool two) {
    const uint64_t end = two ? B2 : B1;
    if ((a + 16u < total ? a + 16u : total) > end) return false;
    u32x4 w[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const fws_frame_desc &fd = r ? d1 : d0;
        const uint64_t Br = r ? B1 : B0;
        const uintptr_t s0 = (uintptr_t)(src + fd.payload_off);
        const uintptr_t sa = s0 + (uintptr_t)(a - Br);   // (a < Br: wraps like the offsets it mirrors)
        const uintptr_t safe = s0 & ~uintptr_t(15);
        uintptr_t b0 = sa & ~uintptr_t(15), b1 = b0 + 16u;
        const bool use = fd.payload_len != 0 && (r == 0 || two);
        if (!use || b0 + 16u <= s0 || b0 >= s0 + fd.payload_len) b0 = safe;
        if (!use || b1 + 16u <= s0 || b1 >= s0 + fd.payload_len) b1 = safe;
        u32x4 v0{0u, 0u, 0u, 0u}, v1{0u, 0u, 0u, 0u};
        if (use) {
            v0 = gload16<true>(b0);
            v1 = gload16<true>(b1);
        }
        const uint32_t rk = rotr32(fd.key, 8u * ((uint32_t)(a - Br + fd.phase) & 3u));
        w[r] = shr_bytes(v0, v1, (uint32_t)(sa & 15u)) ^ rk;
    }
    const uint32_t t = chunk_rel(total, a), e0 = chunk_rel(B1, a), e1 = chunk_rel(end, a);
    const uint32_t wa[4] = {w[0].x, w[0].y, w[0].z, w[0].w}, wb[4] = {w[1].x, w[1].y, w[1].z, w[1].w};
    uint32_t x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        x[i] = chunk_sel(0u, t, i) & ((wa[i] & chunk_sel(0u, e0, i)) | (two ? wb[i] & chunk_sel(e0, e1, i) : 0u));
    if (a + 16u <= total) {
        gstore16<true>((uintptr_t)(dst + a), u32x4{x[0], x[1], x[2], x[3]});
    } else {
        for (uint64_t b = a; b < total; ++b) dst[b] = (uint8_t)(x[(b - a) >> 2] >> (8u * ((b - a) & 3u)));
    }
    return true;
}

// kFlat (r06): the metadata in two scalar rounds (the total with the unit map,
// then both regions' offsets and descriptors together -- the compiler had given
// each its own dependent round, five per unit) and one nontemporal load per
// chunk with the neighbour lane's block by DPP (the second block of a shifted
// window re-read through the cache costs a second L2 request per line when the
// source comes from HBM); region seams and the tail bytewise after the unit's
// full chunks. tools/bw_probe3 (4 rotating sources, past the 256 MB MALL): the
// DPP form of a shifted copy 84.0-84.6 us against 89.6-90.3 us for two loads.
__device__ __forceinline__ fws_frame_desc frame_desc_of(const uint32_t (&w)[6]) {
    fws_frame_desc x;
    x.payload_off = w[0] | ((uint64_t)w[1] << 32);
    x.payload_len = w[2] | ((uint64_t)w[3] << 32);
    x.key = w[4];
    x.phase = w[5];
    return x;
}

// Requires dst 16-B aligned.
template <bool kFlat>
__global__ __launch_bounds__(kBlock) void k_gather_fast(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                                        const fws_frame_desc *__restrict__ d, uint32_t n,
                                                        const uint64_t *__restrict__ dbase,
                                                        const uint32_t *__restrict__ unit_first, uint64_t unit_cap,
                                                        const uint64_t *__restrict__ total_ptr) {
    static_assert(sizeof(fws_frame_desc) == 24, "6 words");
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (kBlock / 64);
    const uint64_t ufirst = (uint64_t)blockIdx.x * (kBlock / 64) + wave;
    // one scalar round: the total and this wave's first unit map entries (clamped in bounds)
    const uint64_t uc = ufirst + 1 < unit_cap ? ufirst : (unit_cap >= 2 ? unit_cap - 2 : 0);
    uint32_t uf0 = unit_first[uc], uf1 = unit_first[uc + 1];
    const uint64_t total = *total_ptr;
    if (kFlat) asm volatile("" ::"s"(uf0), "s"(uf1), "s"((uint32_t)total));
    const uint64_t n_units = (total + kGatherUnit - 1) / kGatherUnit;
    for (uint64_t u = ufirst; u < n_units; u += nw) {
        if (u != ufirst || u + 1 >= unit_cap) {       // past the map's capacity: searched (dbase)
            uf0 = unit_owner(unit_first, unit_cap, dbase, n, u, u * kGatherUnit);
            uf1 = u + 1 < n_units ? unit_owner(unit_first, unit_cap, dbase, n, u + 1, (u + 1) * kGatherUnit) : 0u;
        }
        const uint32_t flo = uf0;
        const uint32_t fhi = (u + 1 < n_units) ? uf1 : n - 1;
        const uint64_t a0 = u * kGatherUnit + (uint64_t)lane * 16u;
        if (fhi - flo >= 2u) {                         // many small regions: per-chunk search
            for (int j = 0; j < 4; ++j) {
                const uint64_t a = a0 + (uint64_t)j * 1024u;
                if (a >= total) break;
                const uint32_t f = find_frame(dbase, flo, fhi, a);
                const uint64_t fb = dbase[f], fe = dbase[f + 1];
                if (a + 16 <= fe) {
                    const fws_frame_desc fd = d[f];
                    const uintptr_t sa = (uintptr_t)(src + fd.payload_off + (a - fb));
                    const uintptr_t sb = sa & ~uintptr_t(15);
                    const uint32_t sh = (uint32_t)(sa & 15u);
                    const u32x4 v0 = gload16(sb), v1 = gload16(sh ? sb + 16u : sb);
                    const uint32_t rk = rotr32(fd.key, 8u * ((uint32_t)(a - fb + fd.phase) & 3u));
                    gstore16<true>((uintptr_t)(dst + a), shr_bytes(v0, v1, sh) ^ rk);
                } else {
                    gather_bytes(dst, src, d, dbase, f, a, total);
                }
            }
            continue;
        }
        // at most two regions: uniform metadata
        uint64_t B0, B1, B2;
        fws_frame_desc d0, d1;
        if constexpr (kFlat) {
            const uint32_t *w0 = reinterpret_cast<const uint32_t *>(d + flo);
            const uint32_t *w1 = reinterpret_cast<const uint32_t *>(d + fhi);
            uint32_t r0[6], r1[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                r0[i] = w0[i];
                r1[i] = w1[i];
            }
            B0 = dbase[flo];
            B1 = dbase[flo + 1];
            const uint64_t b2 = dbase[fhi > flo ? flo + 2 : flo + 1];   // (dbase has n + 1 entries)
            asm volatile("" ::"s"(r0[0]), "s"(r0[5]), "s"(r1[0]), "s"(r1[5]), "s"((uint32_t)B0), "s"((uint32_t)B1),
                         "s"((uint32_t)b2));
            B2 = b2;
            d0 = frame_desc_of(r0);
            d1 = frame_desc_of(r1);
        } else {
            B0 = dbase[flo];
            B1 = dbase[flo + 1];
            B2 = fhi > flo ? dbase[flo + 2] : B1;
            d0 = d[flo];
            d1 = d[fhi];
        }
        const uintptr_t S0 = (uintptr_t)(src + d0.payload_off) - (uintptr_t)B0;   // src of dst byte a: S + a
        const uintptr_t S1 = (uintptr_t)(src + d1.payload_off) - (uintptr_t)B1;
        uintptr_t sb[4];
        uint32_t sh[4], rk[4];
        bool full[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t a = a0 + (uint64_t)j * 1024u;
            const bool in0 = a >= B0 && a + 16 <= B1;
            const bool in1 = fhi > flo && a >= B1 && a + 16 <= B2;
            full[j] = (in0 || in1) && a + 16 <= total;
            const uintptr_t sa = (in1 ? S1 : S0) + (uintptr_t)a;
            sb[j] = full[j] ? (sa & ~uintptr_t(15)) : ((uintptr_t)(src + d0.payload_off) & ~uintptr_t(15));
            sh[j] = (uint32_t)(sa & 15u);
            const uint32_t ph = in1 ? (uint32_t)(a - B1) + d1.phase : (uint32_t)(a - B0) + d0.phase;
            rk[j] = rotr32(in1 ? d1.key : d0.key, 8u * (ph & 3u));
        }
        if constexpr (kFlat) {
            // one nontemporal load per chunk; the window's second block is lane L + 1's
            // first when that is the next block (lane 63: lane 0's of the next chunk,
            // or for the last chunk a load of its own); a full chunk without it, a
            // region seam and the tail go bytewise after the full chunks
            u32x4 w0[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) w0[j] = gload16<true>(sb[j]);
            u32x4 last = u32x4{0u, 0u, 0u, 0u};
            if (lane == 63) last = gload16<true>(full[3] && sh[3] ? sb[3] + 16u : sb[3]);
            uint32_t pend = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t a = a0 + (uint64_t)j * 1024u;
                uint64_t nsb = wave_shl1_64(sb[j]);
                u32x4 w1 = wave_shl1(w0[j]);
                if (j < 3) {
                    const uint64_t nsb0 = lane0_of64(sb[j < 3 ? j + 1 : 0]);
                    const u32x4 nv0 = lane0_of(w0[j < 3 ? j + 1 : 0]);
                    if (lane == 63) {
                        nsb = nsb0;
                        w1 = nv0;
                    }
                } else if (lane == 63) {
                    nsb = sb[3] + 16u;
                    w1 = last;
                }
                const bool ok = sh[j] == 0u || nsb == sb[j] + 16u;
                if (full[j] && ok) gstore16<true>((uintptr_t)(dst + a), shr_bytes(w0[j], w1, sh[j]) ^ rk[j]);
                else if (a < total) pend |= 1u << j;
            }
            for (; pend; pend &= pend - 1u) {
                const uint64_t a = a0 + (uint64_t)__builtin_ctz(pend) * 1024u;
                if (!gather_seam(dst, src, a, total, d0, d1, B0, B1, B2, fhi > flo))
                    gather_bytes(dst, src, d, dbase, flo, a, total);
            }
            continue;
        }
        u32x4 v0[4], v1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {                 // default policy: lane L's second block is
            uintptr_t s1 = full[j] && sh[j] ? sb[j] + 16u : sb[j];   // lane L + 1's first (nontemporal
            asm volatile("" : "+v"(s1));                // pairs fetched it twice); opaque: no
            v0[j] = gload16(sb[j]);                     // "same address" copy of v0 (a copy
            v1[j] = gload16(s1);                        // would wait for the load)
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t a = a0 + (uint64_t)j * 1024u;
            if (full[j]) gstore16<true>((uintptr_t)(dst + a), shr_bytes(v0[j], v1[j], sh[j]) ^ rk[j]);
            else if (a < total) gather_bytes(dst, src, d, dbase, flo, a, total);
        }
    }
}

// ------------------------------------------------------------- one launch
// k_gather_one: the same gather with no plan launch, for batches of at most
// kGatherLdsMax regions (C4: 1427 fragments). Every workgroup of a grid-stride
// grid builds the whole dst prefix (dbase) in LDS from the descriptors -- one
// round of coalesced loads (L2-resident after the first workgroups) and a
// block scan, about the latency of one dependent round trip -- and then walks
// its units as k_gather_fast does. The regions of a wave's first 64 units are
// found up front, one unit per lane (a binary search of that LDS prefix), and
// read back per unit with readlane; later units use two rounds of 64 lane
// probes. The plan launch (k_out_plan, 6.9 us on C4) and its launch boundary
// are gone.
constexpr uint32_t kGatherLdsMax = 2048;

// The last f < n with base[f] <= pos (base[0] = 0 <= pos; base in LDS): lane
// probes at a stride, then inside the bracketed stride. Wave-uniform result.
__device__ __forceinline__ uint32_t lds_owner(const uint64_t *base, uint32_t n, uint64_t pos, int lane) {
    const uint32_t stride = (n + 63u) / 64u;                // <= kGatherLdsMax / 64
    const uint32_t i1 = (uint32_t)lane * stride;
    const uint64_t m1 = __ballot(i1 < n && base[i1] <= pos);
    const uint32_t j = 63u - (uint32_t)__builtin_clzll(m1);
    const uint32_t i2 = j * stride + (uint32_t)lane;
    const uint64_t m2 = __ballot((uint32_t)lane < stride && i2 < n && base[i2] <= pos);
    return __builtin_amdgcn_readfirstlane(j * stride + (63u - (uint32_t)__builtin_clzll(m2)));
}

// The same search by one lane: binary search over base[0, n) (per-lane result).
__device__ __forceinline__ uint32_t lds_search(const uint64_t *base, uint32_t n, uint64_t pos) {
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1u) >> 1;
        if (base[mid] <= pos) lo = mid;
        else hi = mid - 1u;
    }
    return lo;
}

// Requires dst 16-B aligned and 1 <= n <= kGatherLdsMax. 74 VGPRs, 6 waves per
// SIMD; forced to 7 (72 VGPRs, 2 spilled on the probe path only) it measured
// 0.096-0.101 against 0.085-0.089 ms on C4 (profiles/r04/ab_gather_shapes.jsonl).
template <uint32_t kT, bool kDpp, bool kLate>
__device__ __forceinline__ void gather_one_body(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                                const fws_frame_desc *__restrict__ d, uint32_t n) {
    constexpr uint32_t kGatherPer = kGatherLdsMax / kT;   // regions per thread in the block scan
    __shared__ uint64_t s_base[kGatherLdsMax + 1];
    __shared__ uint64_t s_wsum[kT / 64];
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // dbase in LDS: lengths (all loads in flight together), then each thread's
    // contiguous run of kGatherPer regions, a block scan of the run sums
    {
        uint64_t l[kGatherPer];
#pragma unroll
        for (uint32_t i = 0; i < kGatherPer; ++i) {
            const uint32_t f = threadIdx.x + i * kT;
            l[i] = f < n ? d[f].payload_len : 0;
        }
#pragma unroll
        for (uint32_t i = 0; i < kGatherPer; ++i) {
            const uint32_t f = threadIdx.x + i * kT;
            if (f < n) s_base[f] = l[i];
        }
        __syncthreads();
        const uint32_t f0 = threadIdx.x * kGatherPer;
        uint64_t sum = 0;
#pragma unroll
        for (uint32_t i = 0; i < kGatherPer; ++i) {
            l[i] = f0 + i < n ? s_base[f0 + i] : 0;
            sum += l[i];
        }
        const uint64_t inc = wave_incl_scan64(sum, lane);
        if (lane == 63) s_wsum[wave] = inc;
        __syncthreads();                              // every run read before it is overwritten
        uint64_t run = inc - sum;
        for (uint32_t i = 0; i < wave; ++i) run += s_wsum[i];
#pragma unroll
        for (uint32_t i = 0; i < kGatherPer; ++i) {
            if (f0 + i < n) s_base[f0 + i] = run;
            run += l[i];
        }
        if (f0 < n && f0 + kGatherPer >= n) s_base[n] = run;
        __syncthreads();
    }
    const uint64_t total = s_base[n];
    const uint64_t n_units = (total + kGatherUnit - 1) / kGatherUnit;
    const uint64_t nw = (uint64_t)gridDim.x * (kT / 64);
    const uint64_t ufirst = (uint64_t)blockIdx.x * (kT / 64) + wave;
    // the regions of the wave's first 64 units, one unit per lane, all lanes
    // searching at once (one chain of LDS round trips per wave, not two per unit)
    // (both region indices < kGatherLdsMax: packed in one register, lo | hi << 16)
    uint32_t my_lh = (n - 1u) << 16;
    {
        const uint64_t u = ufirst + (uint64_t)lane * nw;
        if (u < n_units) {
            const uint32_t lo = lds_search(s_base, n, u * kGatherUnit);
            const uint32_t hi = u + 1 < n_units ? lds_search(s_base, n, (u + 1) * kGatherUnit) : n - 1u;
            my_lh = lo | (hi << 16);
        }
    }
    uint32_t k = 0;
    for (uint64_t u = ufirst; u < n_units; u += nw, ++k) {
        uint32_t flo, fhi;
        if (k < 64u) {
            const uint32_t lh = __builtin_amdgcn_readlane(my_lh, k);
            flo = lh & 0xFFFFu;
            fhi = lh >> 16;
        } else {
            flo = lds_owner(s_base, n, u * kGatherUnit, lane);
            fhi = u + 1 < n_units ? lds_owner(s_base, n, (u + 1) * kGatherUnit, lane) : n - 1;
        }
        const uint64_t a0 = u * kGatherUnit + (uint64_t)lane * 16u;
        if (fhi - flo >= 2u) {                         // many small regions: per-chunk search
            for (int j = 0; j < 4; ++j) {
                const uint64_t a = a0 + (uint64_t)j * 1024u;
                if (a >= total) break;
                const uint32_t f = find_frame(s_base, flo, fhi, a);
                const uint64_t fb = s_base[f], fe = s_base[f + 1];
                if (a + 16 <= fe) {
                    const fws_frame_desc fd = d[f];
                    const uintptr_t sa = (uintptr_t)(src + fd.payload_off + (a - fb));
                    const uintptr_t sb = sa & ~uintptr_t(15);
                    const uint32_t sh = (uint32_t)(sa & 15u);
                    const u32x4 v0 = gload16(sb), v1 = gload16(sh ? sb + 16u : sb);
                    const uint32_t rk = rotr32(fd.key, 8u * ((uint32_t)(a - fb + fd.phase) & 3u));
                    gstore16<true>((uintptr_t)(dst + a), shr_bytes(v0, v1, sh) ^ rk);
                } else {
                    gather_bytes(dst, src, d, s_base, f, a, total);
                }
            }
            continue;
        }
        // at most two regions: uniform metadata (k_gather_fast's body)
        const uint64_t B0 = s_base[flo], B1 = s_base[flo + 1];
        const uint64_t B2 = fhi > flo ? s_base[flo + 2] : B1;
        const fws_frame_desc d0 = d[flo], d1 = d[fhi];
        const uintptr_t S0 = (uintptr_t)(src + d0.payload_off) - (uintptr_t)B0;
        const uintptr_t S1 = (uintptr_t)(src + d1.payload_off) - (uintptr_t)B1;
        uintptr_t sb[4];
        uint32_t sh[4], rk[4];
        bool full[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t a = a0 + (uint64_t)j * 1024u;
            const bool in0 = a >= B0 && a + 16 <= B1;
            const bool in1 = fhi > flo && a >= B1 && a + 16 <= B2;
            full[j] = (in0 || in1) && a + 16 <= total;
            const uintptr_t sa = (in1 ? S1 : S0) + (uintptr_t)a;
            sb[j] = full[j] ? (sa & ~uintptr_t(15)) : ((uintptr_t)(src + d0.payload_off) & ~uintptr_t(15));
            sh[j] = (uint32_t)(sa & 15u);
            const uint32_t ph = in1 ? (uint32_t)(a - B1) + d1.phase : (uint32_t)(a - B0) + d0.phase;
            rk[j] = rotr32(in1 ? d1.key : d0.key, 8u * (ph & 3u));
        }
        if constexpr (kDpp) {
            // one nontemporal load per chunk: a lane's second block is lane L + 1's
            // first when that lane's block is the next one (same region and shift);
            // lane 63's is lane 0's of the next chunk, or for the last chunk a load
            // of its own. A full chunk whose neighbour block is another (a region
            // seam) goes bytewise with the seam / tail chunks.
            u32x4 v0[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v0[j] = gload16<true>(sb[j]);
            u32x4 last = u32x4{0u, 0u, 0u, 0u};
            if (lane == 63) last = gload16<true>(full[3] && sh[3] ? sb[3] + 16u : sb[3]);
            uint32_t pend = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t a = a0 + (uint64_t)j * 1024u;
                uint64_t nsb = wave_shl1_64(sb[j]);
                u32x4 v1 = wave_shl1(v0[j]);
                if (j < 3) {
                    const uint64_t nsb0 = lane0_of64(sb[j < 3 ? j + 1 : 0]);
                    const u32x4 nv0 = lane0_of(v0[j < 3 ? j + 1 : 0]);
                    if (lane == 63) {
                        nsb = nsb0;
                        v1 = nv0;
                    }
                } else if (lane == 63) {
                    nsb = sb[3] + 16u;
                    v1 = last;
                }
                const bool ok = sh[j] == 0u || nsb == sb[j] + 16u;
                if (full[j] && ok) gstore16<true>((uintptr_t)(dst + a), shr_bytes(v0[j], v1, sh[j]) ^ rk[j]);
                else if (a < total) pend |= 1u << j;
            }
            for (; pend; pend &= pend - 1u)
                gather_bytes(dst, src, d, s_base, flo, a0 + (uint64_t)__builtin_ctz(pend) * 1024u, total);
            continue;
        }
        u32x4 v0[4], v1[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uintptr_t s1 = full[j] && sh[j] ? sb[j] + 16u : sb[j];
            asm volatile("" : "+v"(s1));
            v0[j] = gload16(sb[j]);
            v1[j] = gload16(s1);
        }
        // the full chunks first; the seam / tail chunks bytewise after them, when
        // the data registers are dead (inline with them, the byte loop's registers
        // held the kernel at 73 VGPRs, 6 waves per SIMD)
        uint32_t pend = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t a = a0 + (uint64_t)j * 1024u;
            if (full[j]) gstore16<true>((uintptr_t)(dst + a), shr_bytes(v0[j], v1[j], sh[j]) ^ rk[j]);
            else if (a < total) pend |= 1u << j;
        }
        if (kLate) {
            for (; pend; pend &= pend - 1u)
                gather_bytes(dst, src, d, s_base, flo, a0 + (uint64_t)__builtin_ctz(pend) * 1024u, total);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((pend >> j) & 1u) gather_bytes(dst, src, d, s_base, flo, a0 + (uint64_t)j * 1024u, total);
        }
    }
}

template <uint32_t kT, bool kDpp = false>
__global__ __launch_bounds__(kT) void k_gather_one(uint8_t *__restrict__ dst, const uint8_t *__restrict__ src,
                                                   const fws_frame_desc *__restrict__ d, uint32_t n) {
    gather_one_body<kT, kDpp, false>(dst, src, d, n);
}

// The same at 8 waves per SIMD (62 VGPRs, no spill): the seam / tail chunks'
// byte loop runs after the unit's full chunks (kLate), not inline with them.
template <uint32_t kT, bool kDpp = false>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(8))) void k_gather_one_w8(
    uint8_t *__restrict__ dst, const uint8_t *__restrict__ src, const fws_frame_desc *__restrict__ d, uint32_t n) {
    gather_one_body<kT, kDpp, true>(dst, src, d, n);
}

}  // namespace fwsk

using namespace fwsk;

// tuning / test hook: 1 = k_gather_one for batches of <= kGatherLdsMax regions,
// 0 = always the plan launch + k_gather_fast (the default since r06: with the
// source past the 256 MB MALL, plan + k_gather_fast<kFlat> 93.4-93.6 us on C4
// against 99.7-99.9 us for k_gather_one_w8, whose grid-stride loop waits for a
// unit's stores before the next unit's loads -- the compiler's vmcnt(0) at the
// loop head -- profiles/r06/ab_c4_flat_seam.jsonl; r04-r05 measured the
// opposite order with one source re-read every step, partly from the MALL)
static int g_gather_one = 0;
// tuning hook: the plan path's kernel, k_gather_fast<true> (r06 kFlat, the
// default) or <false> (two loads per chunk, r05)
static int g_gather_flat = 1;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_gather_flat(int on) {
    const int old = g_gather_flat;
    g_gather_flat = on != 0;
    return old;
}
static int g_gather_blocks = 0;        // tuning: k_gather_one grid cap (0 = 4 x resident workgroups)
extern "C" __attribute__((visibility("default"))) int fws_internal_set_gather_blocks(int blocks) {
    const int old = g_gather_blocks;
    g_gather_blocks = blocks > 0 ? blocks : 0;
    return old;
}
extern "C" __attribute__((visibility("default"))) int fws_internal_set_gather_one(int on) {
    const int old = g_gather_one;
    g_gather_one = on != 0;
    return old;
}

int fws_launch_utf8_descs(const uint8_t *base, const fws_frame_desc *descs, uint32_t n, uint8_t *ok,
                          hipStream_t s) {
    if (n == 0) return 0;
    uint32_t blocks = (n + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_utf8<false>, dim3(blocks), dim3(kBlock), 0, s, base, ~0ull, descs, nullptr, n, nullptr, ok);
    return fws_hip_status(hipGetLastError());
}

// k_gather_one's grid: 4 x the resident workgroups (each builds the prefix
// once; a grid-stride loop over units, 2-3 per wave on C4): fewer workgroups
// leave a static tail (1 x resident: 0.095 ms on C4), more repeat the prefix
// build (one unit per wave: 0.098 ms); 4 x: 0.0865 ms
// (profiles/r04/ab_gather.jsonl). Fewer for a small reservation.
// k_gather_one's shape: 512 threads (one prefix build per 8 waves) and 4 x the
// resident workgroups; on C4 0.0850-0.0852 ms against 0.0864-0.0892 ms for
// 256 threads x 4 and 0.0888-0.0897 for plan + k_gather_fast, in one process
// (profiles/r04/ab_gather_shapes.jsonl; on a 64 MiB message 256 threads is
// ~1 us faster). Tuning hook below.
static int g_gather_threads = 512, g_gather_mult = 4;
// tuning hook: 0 = k_gather_one (r05); 1 = k_gather_one<.., true> (one
// nontemporal load per chunk + the neighbour's block by DPP); 2 =
// k_gather_one_w8 (8 waves per SIMD), the default; 3 = k_gather_one_w8<.., true>
static int g_gather_dpp = 2;
extern "C" __attribute__((visibility("default"))) int fws_internal_set_gather_dpp(int on) {
    const int old = g_gather_dpp;
    g_gather_dpp = on >= 0 && on <= 3 ? on : 0;
    return old;
}
// threads 256 or 512 (0: the default), mult > 0 (0: the default)
extern "C" __attribute__((visibility("default"))) int fws_internal_set_gather_shape(int threads, int mult) {
    if (threads != 0 && threads != 256 && threads != 512) return FWS_ERR_INVALID;
    g_gather_threads = threads ? threads : 512;
    g_gather_mult = mult > 0 ? mult : 4;
    return 0;
}

// the k_gather_one form of the hooks: (k_gather_dpp, 512 threads) -> kernel
static const void *gather_one_kernel(int mode, bool t512) {
    switch (mode * 2 + (t512 ? 1 : 0)) {
    case 0: return (const void *)k_gather_one<256>;
    case 1: return (const void *)k_gather_one<512>;
    case 2: return (const void *)k_gather_one<256, true>;
    case 3: return (const void *)k_gather_one<512, true>;
    case 4: return (const void *)k_gather_one_w8<256>;
    case 5: return (const void *)k_gather_one_w8<512>;
    case 6: return (const void *)k_gather_one_w8<256, true>;
    default: return (const void *)k_gather_one_w8<512, true>;
    }
}

static int gather_one_grid(uint64_t max_bytes, uint64_t *out) {
    static int resident[8][64] = {};               // [mode * 2 + (512 threads)][device]
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return FWS_ERR_INVALID;
    const int v = g_gather_dpp * 2 + (g_gather_threads == 512 ? 1 : 0);
    if (!resident[v][dev]) {
        int cus = 0, per = 0;
        hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, gather_one_kernel(g_gather_dpp, v & 1),
                                                             g_gather_threads, 0);
        if (e != hipSuccess) return FWS_ERR_NO_DEVICE;
        resident[v][dev] = cus * (per > 0 ? per : 1);
    }
    const uint64_t wpb = (uint64_t)g_gather_threads / 64u;
    uint64_t blocks = (max_bytes / kGatherUnit + wpb) / wpb;
    const uint64_t cap = g_gather_blocks ? (uint64_t)g_gather_blocks
                                         : (uint64_t)g_gather_mult * (uint64_t)resident[v][dev];
    if (blocks > cap) blocks = cap;
    *out = blocks < 1 ? 1 : blocks;
    return 0;
}

// tuning hook: the grid k_gather_one gets for a context of max_bytes (0 on error)
extern "C" __attribute__((visibility("default"))) uint64_t fws_internal_gather_one_grid(uint64_t max_bytes) {
    uint64_t b = 0;
    return gather_one_grid(max_bytes, &b) == 0 ? b : 0;
}

int fws_launch_gather(uint8_t *dst, const uint8_t *src, const fws_frame_desc *d, uint32_t n, fws_plan_ws &ws,
                      uint64_t max_bytes, hipStream_t s) {
    if (n == 0) return 0;
    if (g_gather_one && n <= kGatherLdsMax) {
        uint64_t blocks = 0;
        const int r = gather_one_grid(max_bytes, &blocks);
        if (r != 0) return r;
        const void *k = gather_one_kernel(g_gather_dpp, g_gather_threads == 512);
        void *args[] = {&dst, &src, &d, &n};
        const hipError_t e = hipLaunchKernel(k, dim3((unsigned)blocks), dim3((unsigned)g_gather_threads), args, 0, s);
        if (e != hipSuccess) return fws_hip_status(e);
        return fws_hip_status(hipGetLastError());
    }
    int r = fws_launch_gather_plan(d, n, ws, s);
    if (r) return r;
    uint64_t units = max_bytes / kGatherUnit + 1;
    if (units > ws.unit_cap) units = ws.unit_cap;
    uint64_t blocks = (units + 3) / 4;
    // one wave per unit in one pass (a cap at 16 384 workgroups left a C2-shaped
    // TX batch's last 129 units to a second round of a few waves)
    if (blocks > (1u << 30)) blocks = 1u << 30;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(g_gather_flat ? k_gather_fast<true> : k_gather_fast<false>, dim3((unsigned)blocks),
                       dim3(kBlock), 0, s, dst, src, d, n, ws.cbase,
                       ws.unit_first, ws.unit_cap, ws.total);
    return fws_hip_status(hipGetLastError());
}
