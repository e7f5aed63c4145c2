// fws_device.h -- device-side helpers shared by the flashws_amd HIP kernels
// (gfx950 only). Integer/byte work: no MFMA anywhere on this path.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fws_gpu.h"

namespace fwsk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;           // CDNA wavefront width
constexpr int kBlock = 256;         // 4 waves per workgroup
constexpr int kUnmaskU = 4;         // 16-B chunks per lane per work unit
constexpr uint64_t kUnitChunks = uint64_t(kWave) * kUnmaskU;   // 256 chunks = 4 KiB per wave unit

// 16-B accesses through the global address space. Addresses are computed as
// integers (chunk arithmetic), which would otherwise make hipcc emit flat_*
// loads (counted on both vmcnt and lgkmcnt) and serialise them.
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

template <bool kNT = false>
__device__ __forceinline__ u32x4 gload16(uintptr_t a) {
    const g_u32x4 *p = (const g_u32x4 *)a;
    if constexpr (kNT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <bool kNT = false>
__device__ __forceinline__ void gstore16(uintptr_t a, u32x4 v) {
    g_u32x4 *p = (g_u32x4 *)a;
    if constexpr (kNT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// A 16-B store with cache policy `sc1 nt`: write-through, the line not kept in
// the XCD's L2. On the in-place XOR stream it beats the plain nontemporal
// store (tools/bw_probe3.hip, profiles/r06/bw_probe3.txt: 82.35 against
// 83.0-83.1 us per 269 MB; `sc1` alone or `sc0 sc1`: 84.2), and the C2 headline
// went 85.1 -> 83.0-83.4 us with it; on the out-of-place kernels (C4 gather,
// TX encode) it measured slower, so they keep gstore16<true>
// (profiles/r06/ab_wt_stores.jsonl). hipcc has no builtin for the policy: one
// asm store, whose trailing s_nop covers the store-data hazard (the compiler
// pads nothing inside asm). Its completion is outside the compiler's vmcnt
// bookkeeping; that stays correct because vector memory operations complete
// in issue order (a later compiler wait can only wait longer).
__device__ __forceinline__ void gstore16_wt(uintptr_t a, u32x4 v) {
    g_u32x4 *p = (g_u32x4 *)a;
    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt\n\ts_nop 1" : : "v"(p), "v"(v) : "memory");
}

// Lane L gets lane L + 1's value (DPP wave_shl:1; lane 63 gets 0), and lane
// 0's value in every lane: the 16-B window of a lane whose aligned source
// block is its neighbour's minus 16 is its own block and the neighbour's,
// so one load per chunk serves two windows (tools/bw_probe3.hip, shifted
// copy: 78.2 us with one default-policy load + the shift against 79.1 us with
// two loads per chunk).
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, false);
}
__device__ __forceinline__ u32x4 wave_shl1(const u32x4 &v) {
    return u32x4{wave_shl1(v.x), wave_shl1(v.y), wave_shl1(v.z), wave_shl1(v.w)};
}
__device__ __forceinline__ uint64_t wave_shl1_64(uint64_t v) {
    return (uint64_t)wave_shl1((uint32_t)v) | ((uint64_t)wave_shl1((uint32_t)(v >> 32)) << 32);
}
__device__ __forceinline__ u32x4 lane0_of(const u32x4 &v) {
    return u32x4{(uint32_t)__builtin_amdgcn_readlane((int)v.x, 0), (uint32_t)__builtin_amdgcn_readlane((int)v.y, 0),
                 (uint32_t)__builtin_amdgcn_readlane((int)v.z, 0), (uint32_t)__builtin_amdgcn_readlane((int)v.w, 0)};
}
__device__ __forceinline__ uint64_t lane0_of64(uint64_t v) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 0) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 0) << 32);
}

// A store through a global-address-space pointer: global_store (vmcnt only),
// where a generic pointer gives flat_store, which also counts in lgkmcnt --
// so the next workgroup barrier's lgkmcnt(0) would wait for the store's
// acknowledgment (a PCIe round trip when it lands in host memory).
// (A record goes out as dwords: its type's copy assignment cannot bind to an
// address-space-qualified object.)
template <typename T>
__device__ __forceinline__ void gput(T *p, const T &v) {
    if constexpr (sizeof(T) % 4 == 0 && alignof(T) >= 4) {
        typedef __attribute__((address_space(1))) uint32_t g_u32;
        uint32_t w[sizeof(T) / 4];
        __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
        for (uint32_t i = 0; i < sizeof(T) / 4; ++i) ((g_u32 *)(uintptr_t)p)[i] = w[i];
    } else {
        static_assert(sizeof(T) == 1, "gput: bytes or dword-aligned records");
        *(__attribute__((address_space(1))) T *)(uintptr_t)p = v;
    }
}
__device__ __forceinline__ uint8_t gget(const uint8_t *p) {
    return *(const __attribute__((address_space(1))) uint8_t *)(uintptr_t)p;
}

// base/constexpr_math.h:67-82 RotateR, 32-bit.
__device__ __forceinline__ uint32_t rotr32(uint32_t v, uint32_t b) {
    b &= 31u;
    return (v >> b) | (v << ((32u - b) & 31u));
}

// Rotated key for any 4-aligned address inside the region starting at
// `region_addr` with key phase `phase`: byte at address x uses key byte
// (x - region_addr + phase) & 3 (ws_mask.h:20,27 + w_socket.h:758).
__device__ __forceinline__ uint32_t aligned_key(uint32_t key, uint32_t phase, uintptr_t region_addr) {
    return rotr32(key, 8u * ((phase - (uint32_t)region_addr) & 3u));
}

// Number of 16-B aligned chunks touched by [addr, addr + len).
__device__ __forceinline__ uint64_t chunks_of(uintptr_t addr, uint64_t len) {
    if (len == 0) return 0;
    return ((addr + len + 15u) >> 4) - (addr >> 4);
}

// XOR only the bytes of chunk [ca, ca+16) that lie inside [lo, hi); rk is the
// key rotated for 4-aligned addresses. Never touches bytes outside [lo, hi).
__device__ __forceinline__ void xor_partial_chunk(uintptr_t ca, uintptr_t lo, uintptr_t hi, uint32_t rk) {
    uintptr_t b = ca > lo ? ca : lo;
    uintptr_t e = (ca + 16u) < hi ? (ca + 16u) : hi;
    while (b < e) {
        if ((b & 3u) == 0 && b + 4u <= e) {
            uint32_t *w = reinterpret_cast<uint32_t *>(b);
            *w = *w ^ rk;
            b += 4u;
        } else {
            uint8_t *p = reinterpret_cast<uint8_t *>(b);
            *p = (uint8_t)(*p ^ (uint8_t)(rk >> (8u * (b & 3u))));
            b += 1u;
        }
    }
}

// Largest f in [lo, hi] with cbase[f] <= g (cbase non-decreasing).
__device__ __forceinline__ uint32_t find_frame(const uint64_t *__restrict__ cbase, uint32_t lo,
                                               uint32_t hi, uint64_t g) {
    while (lo < hi) {
        uint32_t mid = lo + ((hi - lo + 1u) >> 1);
        if (cbase[mid] <= g) lo = mid; else hi = mid - 1u;
    }
    return lo;
}

// RFC 6455 §5.2 header parse with the reference's exact semantics
// (w_socket.h:435-524), for `avail` readable bytes at p (avail may exceed 14).
// Returns header length (>0), 0 = incomplete, or a negative FWS_ERR_* code.
struct Hdr {
    uint64_t plen;
    uint32_t key;
    uint32_t opcode;
    uint32_t fin;
};

__device__ __forceinline__ bool valid_opcode(uint32_t op) {   // w_socket.h:526-528
    return (op <= 2u) | ((op >= 8u) & (op <= 10u));
}

template <typename ByteAt>
__device__ __forceinline__ int parse_hdr(ByteAt at, uint64_t avail, bool is_server, Hdr &h) {
    if (avail < 2) return 0;                                   // :443-445
    uint32_t b0 = at(0);
    h.opcode = b0 & 15u;                                       // :448
    if (!valid_opcode(h.opcode)) return FWS_ERR_OPCODE;        // :451-454
    h.fin = b0 >> 7;                                           // :465
    if (b0 & 112u) return FWS_ERR_RSV;                         // :466-470
    uint32_t b1 = at(1);
    uint32_t masked = b1 >> 7;                                 // :472
    uint64_t plen = b1 & 127u;                                 // :473
    int n = 2;
    if (plen == 126u) {                                        // :476-482
        if (avail < 4) return 0;
        plen = (uint64_t(at(2)) << 8) | at(3);
        n = 4;
    } else if (plen == 127u) {                                 // :483-492
        if (avail < 10) return 0;
        uint64_t v = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) v = (v << 8) | at(2 + i);
        plen = v;
        n = 10;
    }
    if (plen > (1ull << 32)) return FWS_ERR_TOO_LARGE;         // :493-498
    h.plen = plen;
    if (is_server) {                                           // :502-516
        if (!masked) return FWS_ERR_NOT_MASKED;
        if (avail < (uint64_t)n + 4u) return 0;
        h.key = uint32_t(at(n)) | (uint32_t(at(n + 1)) << 8) | (uint32_t(at(n + 2)) << 16) |
                (uint32_t(at(n + 3)) << 24);
        n += 4;
    } else {
        if (masked) return FWS_ERR_MASKED;                     // :518-521
        h.key = 0;
    }
    return n;
}

// ---- UTF-8 (Unicode Table 3-7 / RFC 3629), bytewise in 32-bit SWAR --------
// Byte-select mask of the dword at address w: bytes inside [lo, hi).
__device__ __forceinline__ uint32_t sel_bytes(uintptr_t w, uintptr_t lo, uintptr_t hi) {
    if (w + 4u <= lo || w >= hi) return 0u;
    const uint32_t s = lo > w ? (uint32_t)(lo - w) : 0u;
    const uint32_t e = hi < w + 4u ? (uint32_t)(w + 4u - hi) : 0u;
    return (0xFFFFFFFFu << (8u * s)) & (0xFFFFFFFFu >> (8u * e));
}

// UTF-8 error flags of the 4 bytes of x, p = the dword before x: byte k of the
// result is nonzero iff byte k of x is in error. Bytes outside the region are
// zero, so a sequence cut by the region end fails rule (A) at the first zero
// byte after it. Unicode Table 3-7 / RFC 3629 as two rules:
//  (A) x is a continuation (10xxxxxx) <=> prev1 >= C0 or prev2 >= E0 or
//      prev3 >= F0 (bit 7 of each byte);
//  (B) prev1 in {C0, C1, F5..FF} and x a continuation; E0 and x < A0; ED and
//      x > 9F; F0 and x < 90; F4 and x > 8F (bits 0..6).
// (B) is three v_perm_b32 lookups on prev1 -- bits 7:5, 4:2 and 2:0, 8-entry
// tables whose AND is exact on every byte, one flag per rule -- against one on
// x's bits 6:4 (exact on continuation bytes; when a non-continuation follows a
// flagged prev1, (A) fails anyway). The lead flags of (A) come from the same
// tables (bit 7: bits 7:5 == 111 is >= E0, and with bit 4 it is >= F0), so
// only >= C0 is computed by shifts. An invalid byte (C0, C1, F5..FF) is flagged
// at the byte after it (by (A) or (B)); the walks run 3 zero bytes past every
// region, so a frame's verdict is the per-rule form's (r02-r04 SWAR, ~36 VALU
// per dword; this form ~22 with the x-side values shared by the chain's next
// call). tools/utf8_lookup_check.c proves the per-byte equivalence on every
// (prev3, prev2) of 48 boundary bytes x every (prev1, x) at each position, and
// on 4e8 random dword pairs.
__device__ __forceinline__ uint32_t utf8_lead_tables(uint32_t x, uint32_t &ta) {
    const uint32_t m = 0x07070707u;
    ta = __builtin_amdgcn_perm(0xFE010000u, 0x00000000u, (x >> 5) & m);     // bits 7:5
    const uint32_t tb = __builtin_amdgcn_perm(0x8282C4A0u, 0x10000009u, (x >> 2) & m);   // bits 4:2
    const uint32_t tc = __builtin_amdgcn_perm(0x868696C2u, 0x828283ABu, x & m);          // bits 2:0
    return ta & tb & tc;
}
__device__ __forceinline__ uint32_t utf8_err_lookup(uint32_t x, uint32_t p) {
    uint32_t tax, tap;
    const uint32_t b1x = utf8_lead_tables(x, tax), b1p = utf8_lead_tables(p, tap);
    const uint32_t x1 = x << 1, tx = x & x1, tp = p & (p << 1);
    const uint32_t req = __builtin_amdgcn_alignbyte(tx, tp, 3u) | __builtin_amdgcn_alignbyte(tax, tap, 2u) |
                         __builtin_amdgcn_alignbyte(b1x, b1p, 1u);
    const uint32_t ea = (x & ~x1) ^ req;
    const uint32_t b2 = __builtin_amdgcn_perm(0u, 0x57574F2Fu, (x >> 4) & 0x07070707u);
    return (ea & 0x80808080u) | (__builtin_amdgcn_alignbyte(b1x, b1p, 3u) & b2);
}

// r02-r04 form (bit 7 of each byte = error; invalid bytes flagged at their own
// position), kept for the A/B build FWS_UTF8_SWAR
__device__ __forceinline__ uint32_t utf8_err_swar(uint32_t x, uint32_t p) {
    const uint32_t H = 0x80808080u;
    const uint32_t x1 = x << 1, x2 = x << 2, x3 = x << 3;
    const uint32_t tx = x & x1, ux = tx & x2, wx = ux & x3;
    const uint32_t tp = p & (p << 1), up = tp & (p << 2), wp = up & (p << 3);
    const uint32_t req = __builtin_amdgcn_alignbyte(tx, tp, 3u) | __builtin_amdgcn_alignbyte(ux, up, 2u) |
                         __builtin_amdgcn_alignbyte(wx, wp, 1u);
    uint32_t err = (x & ~x1) ^ req;
    err |= tx & ~((x & 0x3E3E3E3Eu) + 0x7E7E7E7Eu);             // C0, C1: >= C0, bits 5..1 zero
    err |= ((x & 0x7F7F7F7Fu) + 0x0B0B0B0Bu) & x;               // F5..FF
    const uint32_t e1 = __builtin_amdgcn_alignbyte(ux, up, 3u);  // prev1 >= E0
    const uint32_t q = __builtin_amdgcn_alignbyte(x, p, 3u) & 0x1F1F1F1Fu;
    const uint32_t nzE0 = q + 0x7F7F7F7Fu, nzED = (q ^ 0x0D0D0D0Du) + 0x7F7F7F7Fu;   // bit 7: q != lead & 1F
    const uint32_t nzF0 = (q ^ 0x10101010u) + 0x7F7F7F7Fu, nzF4 = (q ^ 0x14141414u) + 0x7F7F7F7Fu;
    const uint32_t s5 = x2, s54 = x2 | x3;                       // bit 5 / bits 5|4 of each byte at bit 7
    const uint32_t bE = (s5 & nzED) | (~s5 & nzE0);
    const uint32_t bF = (s54 & nzF4) | (~s54 & nzF0);
    err |= e1 & ~(bE & bF);
    return err & H;
}

#ifndef FWS_UTF8_SWAR
#define FWS_UTF8_SWAR 0
#endif
// callers test byte k != 0 (masks 0xFF000000 / 0x00FFFFFF select bytes), which
// both forms satisfy
__device__ __forceinline__ uint32_t utf8_err(uint32_t x, uint32_t p) {
    if constexpr (FWS_UTF8_SWAR != 0) return utf8_err_swar(x, p);
    else return utf8_err_lookup(x, p);
}

}  // namespace fwsk
