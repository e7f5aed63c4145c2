// scan_common.h -- the header scan's per-wavefront building blocks, shared by
// k_scan (decode_kernels.hip) and the dense-tile path of k_merge
// (merge_kernels.hip): the two-byte candidate test, header windows and parses
// with ParseFrameHdr's semantics (net/w_socket.h:435-524), wavefront scans, and
// dense_tile() for the tiles k_scan leaves.
#pragma once

#include "decode_common.h"

namespace fwsk {


// ------------------------------------------------------------------ k_scan
// Offsets whose first two bytes cannot start a server-side header (RSV set,
// reserved opcode, MASK clear: w_socket.h:451-515) are dead on sight; only the
// rest ("candidates", ~2% of random payload bytes) are parsed in full and
// pointer-jumped. Candidate k is the k-th candidate offset of the tile (node).
//
// One wavefront owns one 2 KiB tile at a time (lane L: bytes 32L..32L+31), so
// every step is wave-synchronous: ballots, shuffles and the wave's private LDS
// area, no workgroup barrier anywhere in the scan.
constexpr int kScanWaves = 4;                          // wavefronts per workgroup
constexpr int kScanThreads = kScanWaves * 64;
constexpr uint32_t kWCap = 1024;                       // node list capacity of a sparse tile
constexpr uint32_t kCandCap = 256;           // k_scan: candidates per tile (else dense)
constexpr uint32_t kLiveCap = 64;            // live nodes per tile, one per lane
constexpr uint32_t kDeadLane = 0xFFu;        // pointer jumping in registers: the chain dies
// the scan's halo: the next tile's first bytes, enough for the two-byte test at
// any exit a 7-bit length form can reach from inside the tile (2047 + 6 + 125,
// + 1) -- a chain whose exit there fails it is dead, not a survivor
constexpr uint32_t kHaloX = 144;
static_assert(kHaloX >= 2047u + 6u + 125u + 2u - kTile && kHaloX % 16u == 0 && kHaloX / 16u <= 64u, "halo");


// Bit i set <=> offset i of the chunk passes the two-byte header test
// (RSV clear, opcode in {0,1,2,8,9,10}, MASK set), four offsets per dword.
// RSV clear and (b0 & 7) <= 2 <=> (b0 & 0x77) <= 2 <=> bit 7 of
// (b0 & 0x77) + 0x7D is clear (no carry leaves the byte: 0x77 + 0x7D < 0x100);
// MASK is bit 7 of b1 (= byte i+1, v_alignbyte by one).
__device__ __forceinline__ uint32_t cand_bits16(const u32x4 &lo, uint32_t next_dword) {
    const uint32_t W[5] = {lo.x, lo.y, lo.z, lo.w, next_dword};
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t x = W[i];
        const uint32_t b1 = __builtin_amdgcn_alignbyte(W[i + 1], x, 1u);
        const uint32_t f = ~((x & 0x77777777u) + 0x7D7D7D7Du) & b1 & 0x80808080u;
        m |= (((f >> 7) & 1u) | ((f >> 14) & 2u) | ((f >> 21) & 4u) | ((f >> 28) & 8u)) << (4 * i);
    }
    return m;
}

// k_scan's form: the 32 offsets of bytes w0:w1 (next dword nx) packed in a
// permuted order, bit 8j + 4h + i <=> offset 16h + 4i + j (i, j < 4, h < 2):
// each dword's flags (bit 7 of its bytes) shift right by 7 - i and OR
// together, so no flag is moved on its own (about half the VALU of the
// in-order form). cand_pbit / cand_off convert.
__device__ __forceinline__ uint32_t cand_flags(uint32_t x, uint32_t next_dword) {
    const uint32_t b1 = __builtin_amdgcn_alignbyte(next_dword, x, 1u);
    return ~((x & 0x77777777u) + 0x7D7D7D7Du) & b1 & 0x80808080u;
}
__device__ __forceinline__ uint32_t cand_bits32p(const u32x4 &w0, const u32x4 &w1, uint32_t nx) {
    const uint32_t W[9] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, nx};
    uint32_t g0 = 0, g1 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        g0 |= cand_flags(W[i], W[i + 1]) >> (7 - i);
        g1 |= cand_flags(W[i + 4], W[i + 5]) >> (7 - i);
    }
    return g0 | (g1 << 4);
}
__device__ __forceinline__ uint32_t cand_pbit(uint32_t o) { return ((o & 3u) << 3) | ((o >> 2) & 7u); }
__device__ __forceinline__ uint32_t cand_off(uint32_t b) { return ((b & 7u) << 2) | (b >> 3); }

// Bytes b..b+15 (b < 16) of the 32-byte window lo:hi as four dwords: shift by
// 8 bytes, then 4, then v_alignbyte -- selects on named values, no indexing.
__device__ __forceinline__ void window16(const u32x4 &lo, const u32x4 &hi, uint32_t b, uint32_t out[4]) {
    const bool s8 = (b & 8u) != 0, s4 = (b & 4u) != 0;
    const uint32_t a0 = s8 ? lo.z : lo.x, a1 = s8 ? lo.w : lo.y, a2 = s8 ? hi.x : lo.z;
    const uint32_t a3 = s8 ? hi.y : lo.w, a4 = s8 ? hi.z : hi.x, a5 = s8 ? hi.w : hi.y;
    const uint32_t c0 = s4 ? a1 : a0, c1 = s4 ? a2 : a1, c2 = s4 ? a3 : a2;
    const uint32_t c3 = s4 ? a4 : a3, c4 = s4 ? a5 : a4;
    const uint32_t sh = b & 3u;
    out[0] = __builtin_amdgcn_alignbyte(c1, c0, sh);
    out[1] = __builtin_amdgcn_alignbyte(c2, c1, sh);
    out[2] = __builtin_amdgcn_alignbyte(c3, c2, sh);
    out[3] = __builtin_amdgcn_alignbyte(c4, c3, sh);
}

// parse_hdr (server side) on a register window; same codes and order of checks
// as ParseFrameHdr (w_socket.h:435-524), with the key picked by its length form
// so no byte index is dynamic (a dynamic index would spill the window).
__device__ __forceinline__ int parse_window(const u32x4 &lo, const u32x4 &hi, uint32_t b, uint64_t avail, Hdr &h) {
    uint32_t d[4];
    window16(lo, hi, b, d);
    if (avail < 2) return 0;                                       // :443-445
    const uint32_t b0 = d[0] & 0xFFu, b1 = (d[0] >> 8) & 0xFFu;
    h.opcode = b0 & 15u;
    if (!valid_opcode(h.opcode)) return FWS_ERR_OPCODE;            // :451-454
    h.fin = b0 >> 7;
    if (b0 & 112u) return FWS_ERR_RSV;                             // :466-470
    uint64_t plen = b1 & 127u;
    int n = 2;
    uint32_t key = __builtin_amdgcn_alignbyte(d[1], d[0], 2u);     // bytes 2..5
    if (plen == 126u) {                                            // :476-482
        if (avail < 4) return 0;
        plen = ((d[0] >> 8) & 0xFF00u) | (d[0] >> 24);
        n = 4;
        key = d[1];                                                // bytes 4..7
    } else if (plen == 127u) {                                     // :483-492
        if (avail < 10) return 0;
        const uint32_t hi32 = __builtin_amdgcn_alignbyte(d[1], d[0], 2u);   // bytes 2..5
        const uint32_t lo32 = __builtin_amdgcn_alignbyte(d[2], d[1], 2u);   // bytes 6..9
        plen = (uint64_t(__builtin_bswap32(hi32)) << 32) | __builtin_bswap32(lo32);
        n = 10;
        key = __builtin_amdgcn_alignbyte(d[3], d[2], 2u);          // bytes 10..13
    }
    if (plen > (1ull << 32)) return FWS_ERR_TOO_LARGE;             // :493-498
    h.plen = plen;
    if (!(b1 >> 7)) return FWS_ERR_NOT_MASKED;                     // :502-507
    if (avail < (uint64_t)n + 4u) return 0;                        // :508-511
    h.key = key;
    return n + 4;
}


// The chain-building part of ParseFrameHdr (w_socket.h:435-524) for an offset
// that passed the two-byte test (so RSV, opcode and MASK are valid): header
// length (> 0), 0 = incomplete (the same avail checks in the same order), or
// FWS_ERR_TOO_LARGE; payload length and key. Window d = bytes p..p+15.
// (avail: bytes from the header to the stream end, any width -- only its
// comparisons with 2..14 matter, so k_scan passes a saturated 32-bit count)
template <typename Avail>
__device__ __forceinline__ int lean_parse(const uint32_t d[4], Avail avail, uint64_t &plen, uint32_t &key) {
    if (avail < 2) return 0;                                       // :443-445
    const uint32_t len7 = (d[0] >> 8) & 127u;
    if (len7 < 126u) {
        plen = len7;
        key = __builtin_amdgcn_alignbyte(d[1], d[0], 2u);          // bytes 2..5
        return avail < 6 ? 0 : 6;                                  // :508-511
    }
    if (len7 == 126u) {                                            // :476-482
        if (avail < 4) return 0;
        plen = ((d[0] >> 8) & 0xFF00u) | (d[0] >> 24);
        key = d[1];                                                // bytes 4..7
        return avail < 8 ? 0 : 8;
    }
    if (avail < 10) return 0;                                      // :483-492
    const uint32_t hi32 = __builtin_amdgcn_alignbyte(d[1], d[0], 2u);
    const uint32_t lo32 = __builtin_amdgcn_alignbyte(d[2], d[1], 2u);
    plen = (uint64_t(__builtin_bswap32(hi32)) << 32) | __builtin_bswap32(lo32);
    if (plen > (1ull << 32)) return FWS_ERR_TOO_LARGE;             // :493-498
    key = __builtin_amdgcn_alignbyte(d[3], d[2], 2u);              // bytes 10..13
    return avail < 14 ? 0 : 14;
}

// LDS of one dense_tile() wavefront. Tiles with <= kWCap candidates use
// nodes[] as pos[kWCap] | nval[kWCap]; denser ones as nval[kTile].
struct ScanWaveLds {
    uint8_t bytes[kTile + kHalo];
    uint16_t nodes[2 * kWCap];
    uint32_t cm[64];                         // candidate bits of lane L's 32 offsets
    uint32_t cpre[64];                       // node index of lane L's first candidate
    uint64_t sbits[kTile / 64];              // surviving nodes
    uint32_t spre[kTile / 64];
};
static_assert(2 * kWCap >= kTile, "dense node table must fit");
static_assert(sizeof(ScanWaveLds) % 16 == 0, "16-B aligned per-wave areas");

// LDS ordering among the lanes of one wavefront (a wave's LDS ops execute in order)
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t x, uint32_t *total) {
    const int lane = threadIdx.x & 63;
    uint32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    *total = __shfl(inc, 63, 64);
    return inc - x;
}


// Wavefront-wide scans on DPP (row shifts, then row broadcasts 15 / 31): VALU
// only, no LDS round trip per step.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return x;
}
__device__ __forceinline__ uint32_t wave_excl_scan_dpp(uint32_t x, uint32_t *total) {
    const uint32_t inc = wave_incl_scan_dpp(x);
    *total = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    return inc - x;
}
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint32_t lane_read(uint32_t v, uint32_t src_lane) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}


// One tile by the per-candidate algorithm, for tiles k_scan leaves (more than
// kCandCap candidates, kLiveCap live nodes or kSlots survivors: frames under
// ~40 B), called by one wavefront of k_merge (merge_kernels.hip). Every
// candidate is a node: parsed (ParseFrameHdr semantics, w_socket.h:435-524),
// pointed at the candidate at its next header offset (a node index, kLeaf |
// itself when the chain leaves the tile or the stream, kDead), and
// pointer-jumped in LDS. Survivors (chains ending at a leaf) go to a spill
// run reserved with one atomic. Returns survivors | spill offset << 32 (the
// offset is kNone when there are none, or when the spill area is full:
// kCntOverflow is set).
__device__ __noinline__ uint64_t dense_tile(ScanWaveLds &W, const uint8_t *__restrict__ wire, uint64_t N, uint32_t t,
                                            fws_frame_info *__restrict__ spill_info, uint32_t *__restrict__ counters,
                                            uint32_t s_cap) {
    const uint32_t lane = threadIdx.x & 63;
    uint8_t *const B = W.bytes;
    const uint64_t t0 = uint64_t(t) * kTile;
    const uint32_t L32 = lane * 32u;
    for (uint32_t i = lane * 16u; i < kTile + kHalo; i += 64u * 16u) {
        const uint64_t q = t0 + i;
        if (q + 16u <= N) {
            *reinterpret_cast<u32x4 *>(B + i) = gload16(reinterpret_cast<uintptr_t>(wire + q));
        } else {
#pragma unroll
            for (int b = 0; b < 16; ++b) B[i + b] = (q + b < N) ? wire[q + b] : 0;
        }
    }
    wave_sync();
    uint32_t cm;
    {
        const u32x4 w0 = *reinterpret_cast<const u32x4 *>(B + L32);
        const u32x4 w1 = *reinterpret_cast<const u32x4 *>(B + L32 + 16u);
        const uint32_t nx = *reinterpret_cast<const uint32_t *>(B + L32 + 32u);
        cm = cand_bits16(w0, w1.x) | (cand_bits16(w1, nx) << 16);
        const uint64_t q = t0 + L32;                   // the last byte: an incomplete header
        if (q >= N) cm = 0;
        else if (N - q <= 32u) cm |= 1u << ((uint32_t)(N - q) - 1u);
    }
    uint32_t nc;
    const uint32_t cp = wave_excl_scan(__popc(cm), &nc);
    W.cm[lane] = cm;
    W.cpre[lane] = cp;
    wave_sync();
    // node value of the candidate at tile offset p: next node, kLeaf|k, or kDead
    auto node_value = [&](uint32_t p, uint32_t k, int r, uint64_t plen) -> uint16_t {
        if (r == 0) return (uint16_t)(kLeaf | k);
        if (r < 0) return kDead;
        const uint64_t nxo = t0 + p + (uint64_t)r + plen;
        if (nxo >= t0 + kTile || nxo >= N) return (uint16_t)(kLeaf | k);
        const uint32_t pn = (uint32_t)(nxo - t0);
        const uint32_t m = W.cm[pn >> 5];
        const uint32_t bit = pn & 31u;
        return ((m >> bit) & 1u) ? (uint16_t)(W.cpre[pn >> 5] + (uint32_t)__popc(m & ((1u << bit) - 1u))) : kDead;
    };
    auto parse_at = [&](uint32_t p, Hdr &h) -> int {
        const uint32_t a = p & ~15u;
        const u32x4 wl = *reinterpret_cast<const u32x4 *>(B + a);
        const u32x4 wh = *reinterpret_cast<const u32x4 *>(B + a + 16u);
        return parse_window(wl, wh, p & 15u, N - (t0 + p), h);
    };
    const bool sparse = nc <= kWCap;                   // wave-uniform
    uint16_t *const pos = W.nodes;
    uint16_t *const nv = sparse ? W.nodes + kWCap : W.nodes;
    {
        uint32_t bits = cm, k = cp;
        while (bits) {
            const uint32_t b = (uint32_t)__ffs(bits) - 1u;
            bits &= bits - 1u;
            if (sparse) {
                pos[k] = (uint16_t)(L32 + b);
            } else {
                Hdr h;
                const int r = parse_at(L32 + b, h);
                nv[k] = node_value(L32 + b, k, r, h.plen);
            }
            ++k;
        }
    }
    wave_sync();
    if (sparse) {
        for (uint32_t k = lane; k < nc; k += 64) {
            const uint32_t p = pos[k];
            Hdr h;
            const int r = parse_at(p, h);
            nv[k] = node_value(p, k, r, h.plen);
        }
        wave_sync();
    }
    for (;;) {                                         // pointer jumping: leaf or dead
        bool ch = false;
        for (uint32_t k = lane; k < nc; k += 64) {
            const uint16_t v = nv[k];
            if (v < kLeaf) {
                nv[k] = nv[v];
                ch = true;
            }
        }
        wave_sync();
        if (!__any(ch)) break;
    }
    uint32_t ns = 0;
    for (uint32_t k0 = 0; k0 < nc; k0 += 64) {         // survivors by node index
        const uint32_t k = k0 + lane;
        const uint64_t m = __ballot(k < nc && nv[k] != kDead);
        if (lane == 0) {
            W.sbits[k0 >> 6] = m;
            W.spre[k0 >> 6] = ns;
        }
        ns += (uint32_t)__popcll(m);
    }
    uint32_t spill = kNone;
    if (ns) {
        if (lane == 0) spill = spill_shared(counters, s_cap, ns);
        spill = __shfl(spill, 0, 64);
        if (spill == kNone) ns = 0;
    }
    wave_sync();
    if (ns) {
        auto emit = [&](uint32_t k, uint32_t p) {
            Hdr h;
            const int r = parse_at(p, h);
            const uint32_t idx = W.spre[k >> 6] + (uint32_t)__popcll(W.sbits[k >> 6] & ((1ull << (k & 63u)) - 1ull));
            const uint64_t q = t0 + p;
            fws_frame_info fi;
            fi.hdr_off = q;
            fi.payload_len = r > 0 ? h.plen : 0;
            fi.key = r > 0 ? h.key : 0;
            fi.opcode = r > 0 ? (uint8_t)h.opcode : (uint8_t)0;
            fi.fin = r > 0 ? (uint8_t)h.fin : (uint8_t)0;
            fi.hdr_len = r > 0 ? (uint8_t)r : (uint8_t)0;
            fi.flags = (r > 0 && q + (uint64_t)r + h.plen > N) ? (uint8_t)FWS_FRAME_TRUNCATED : (uint8_t)0;
            spill_info[spill + idx] = fi;
        };
        if (sparse) {
            for (uint32_t k = lane; k < nc; k += 64)
                if (nv[k] != kDead) emit(k, pos[k]);
        } else {
            uint32_t bits = cm, k = cp;
            while (bits) {
                const uint32_t b = (uint32_t)__ffs(bits) - 1u;
                bits &= bits - 1u;
                if (nv[k] != kDead) emit(k, L32 + b);
                ++k;
            }
        }
    }
    wave_sync();
    return (uint64_t)ns | ((uint64_t)spill << 32);
}

}  // namespace fwsk
